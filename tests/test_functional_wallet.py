"""Wallet functional tests against real bcpd processes (regtest).

Parity: reference qa/rpc-tests wallet.py (balances, sendtoaddress/sendmany, listunspent,
lockunspent, gettransaction, fee accounting), wallet-accounts.py / receivedby.py
(accounts, listreceivedby*), encryptwallet.py (encrypt / unlock / relock / change
passphrase), wallet-dump.py + importprunedfunds.py (dump/import), fundrawtransaction.py,
abandonconflict.py, wallet-hd.py (HD key paths, restore from backup), keypool.py.
"""
import os
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def wait_until(pred, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.1)
    raise AssertionError("timeout")


def D(x):
    return Decimal(str(x))


@pytest.fixture
def pair(tmp_path):
    a = BcpdProcess(str(tmp_path / "wa"), extra_args=["-gpu=0", "-keypool=20"])
    b = BcpdProcess(str(tmp_path / "wb"), extra_args=["-gpu=0", "-keypool=20"])
    a.start()
    b.start()
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    wait_until(lambda: a.rpc.getconnectioncount() == 1 and b.rpc.getconnectioncount() == 1)
    yield a, b
    a.stop()
    b.stop()


def sync(a, b):
    wait_until(lambda: a.rpc.getbestblockhash() == b.rpc.getbestblockhash())


def test_balance_send_receive(pair):
    a, b = pair
    info = a.rpc.getwalletinfo()
    assert info["keypoolsize"] >= 20 and "hdmasterkeyid" in info
    a.rpc.generate(101)
    sync(a, b)
    subsidy = D(a.rpc.getblock(a.rpc.getblockhash(1), 2)["tx"][0]["vout"][0]["value"])
    assert D(a.rpc.getbalance()) == subsidy
    assert D(a.rpc.getwalletinfo()["immature_balance"]) == subsidy * 100
    addr_b = b.rpc.getnewaddress("savings")
    assert b.rpc.validateaddress(addr_b)["ismine"] is True
    assert a.rpc.validateaddress(addr_b)["ismine"] is False
    txid = a.rpc.sendtoaddress(addr_b, 10, "c1", "to-b")
    wait_until(lambda: txid in b.rpc.getrawmempool())
    assert D(b.rpc.getunconfirmedbalance()) == D(10)
    tx = a.rpc.gettransaction(txid)
    fee = -D(tx["fee"])
    assert D(0) < fee < D("0.01")
    assert tx["comment"] == "c1" and tx["to"] == "to-b"
    assert D(tx["amount"]) == D(-10)
    a.rpc.generate(1)
    sync(a, b)
    wait_until(lambda: D(b.rpc.getbalance()) == D(10))
    assert D(b.rpc.getreceivedbyaddress(addr_b)) == D(10)
    assert D(b.rpc.getbalance("savings")) == D(10)
    assert b.rpc.getaccount(addr_b) == "savings"
    assert addr_b in b.rpc.getaddressesbyaccount("savings")
    # a: 2 mature coinbases now (block 1 and 2) minus 10 and the fee
    assert D(a.rpc.getbalance()) == subsidy * 2 - 10 - fee
    lt = b.rpc.listtransactions()
    assert lt[-1]["category"] == "receive" and lt[-1]["txid"] == txid and lt[-1]["confirmations"] == 1
    lu = b.rpc.listunspent()
    assert len(lu) == 1 and lu[0]["txid"] == txid and D(lu[0]["amount"]) == D(10)
    rba = b.rpc.listreceivedbyaddress()
    assert any(r["address"] == addr_b and D(r["amount"]) == D(10) for r in rba)
    # sendmany with fee subtraction
    a1, a2 = b.rpc.getnewaddress(), b.rpc.getnewaddress()
    txid2 = a.rpc.sendmany("", {a1: 1, a2: 2}, 1, "multi", [a1])
    a.rpc.generate(1)
    sync(a, b)
    wait_until(lambda: b.rpc.gettransaction(txid2)["confirmations"] == 1)
    assert D(b.rpc.getreceivedbyaddress(a2)) == D(2)
    assert D(b.rpc.getreceivedbyaddress(a1)) < D(1)
    # b spends back; change goes to a fresh key
    back = a.rpc.getnewaddress()
    t3 = b.rpc.sendtoaddress(back, 5)
    assert len(b.rpc.gettransaction(t3)["details"]) == 1
    groups = b.rpc.listaddressgroupings()
    assert groups


def test_lockunspent_and_fundraw(pair):
    a, b = pair
    a.rpc.generate(110)
    sync(a, b)
    unspent = a.rpc.listunspent()
    assert len(unspent) == 10
    first = {"txid": unspent[0]["txid"], "vout": unspent[0]["vout"]}
    assert a.rpc.lockunspent(False, [first]) is True
    assert a.rpc.listlockunspent() == [first]
    assert len(a.rpc.listunspent()) == 9
    assert a.rpc.lockunspent(True, [first]) is True
    assert a.rpc.listlockunspent() == []
    dest = b.rpc.getnewaddress()
    raw = a.rpc.createrawtransaction([], {dest: 3})
    funded = a.rpc.fundrawtransaction(raw)
    assert D(funded["fee"]) > 0
    dec = a.rpc.decoderawtransaction(funded["hex"])
    assert len(dec["vin"]) >= 1 and len(dec["vout"]) == 2
    signed = a.rpc.signrawtransaction(funded["hex"])
    assert signed["complete"]
    txid = a.rpc.sendrawtransaction(signed["hex"])
    wait_until(lambda: txid in b.rpc.getrawmempool())
    # abandon: a tx that never reaches a mempool can be abandoned
    assert a.rpc.getrawmempool() == [txid]
    with pytest.raises(RPCError):
        a.rpc.abandontransaction(txid)  # still in the mempool


def test_encryption_lifecycle(tmp_path):
    n = BcpdProcess(str(tmp_path / "enc"), extra_args=["-gpu=0", "-keypool=5"])
    n.start()
    try:
        n.rpc.generate(101)
        addr = n.rpc.getnewaddress()
        priv = n.rpc.dumpprivkey(addr)
        assert n.rpc.encryptwallet("pw1").startswith("wallet encrypted")
        with pytest.raises(RPCError) as e:
            n.rpc.dumpprivkey(addr)
        assert e.value.code == -13
        with pytest.raises(RPCError) as e:
            n.rpc.walletpassphrase("wrong", 10)
        assert e.value.code == -14
        n.rpc.walletpassphrase("pw1", 60)
        assert n.rpc.dumpprivkey(addr) == priv
        assert n.rpc.getwalletinfo()["unlocked_until"] > 0
        n.rpc.walletlock()
        with pytest.raises(RPCError):
            n.rpc.sendtoaddress(addr, 1)
        n.rpc.walletpassphrasechange("pw1", "pw2")
        with pytest.raises(RPCError):
            n.rpc.walletpassphrase("pw1", 10)
        n.rpc.walletpassphrase("pw2", 2)
        txid = n.rpc.sendtoaddress(addr, 1)
        assert txid in n.rpc.getrawmempool()
        wait_until(lambda: n.rpc.getwalletinfo()["unlocked_until"] == 0 or
                   _locked(n), 10)
    finally:
        n.stop()
    # restart: encrypted keys reload, still locked, balance intact
    n2 = BcpdProcess(str(tmp_path / "enc"), extra_args=["-gpu=0"], port=n.rpcport)
    n2.start()
    try:
        with pytest.raises(RPCError):
            n2.rpc.dumpprivkey(addr)
        n2.rpc.walletpassphrase("pw2", 30)
        assert n2.rpc.dumpprivkey(addr) == priv
        assert D(n2.rpc.getbalance()) > 0
    finally:
        n2.stop()


def _locked(n):
    try:
        n.rpc.signmessage(n.rpc.getnewaddress(), "x")
        return False
    except RPCError:
        return True


def test_dump_import_backup(tmp_path):
    n = BcpdProcess(str(tmp_path / "d1"), extra_args=["-gpu=0", "-keypool=5"])
    n.start()
    try:
        addr = n.rpc.getnewaddress("lbl")
        n.rpc.generatetoaddress(1, addr)
        n.rpc.generate(100)
        bal = D(n.rpc.getbalance())
        assert bal > 0
        info = n.rpc.validateaddress(addr)
        assert info["hdkeypath"].startswith("m/0'/0'/")
        dump = str(tmp_path / "dump.txt")
        n.rpc.dumpwallet(dump)
        text = open(dump).read()
        assert "extended private masterkey" in text and addr in text
        bk = str(tmp_path / "backup.dat")
        n.rpc.backupwallet(bk)
        sig = n.rpc.signmessage(addr, "hello")
        assert n.rpc.verifymessage(addr, sig, "hello") is True
    finally:
        n.stop()
    # import the dump into a fresh node sharing the same chain
    m = BcpdProcess(str(tmp_path / "d1"), extra_args=["-gpu=0", "-wallet=fresh.dat"], port=n.rpcport)
    m.start()
    try:
        assert D(m.rpc.getbalance()) == 0
        m.rpc.importwallet(dump)
        assert D(m.rpc.getbalance()) == bal
        assert m.rpc.getaccount(addr) == "lbl"
    finally:
        m.stop()
    # restore from the backup store
    os.rename(bk, str(tmp_path / "d1" / "regtest" / "restored.dat"))
    r = BcpdProcess(str(tmp_path / "d1"), extra_args=["-gpu=0", "-wallet=restored.dat"], port=n.rpcport)
    r.start()
    try:
        assert D(r.rpc.getbalance()) == bal
    finally:
        r.stop()


def test_watchonly_and_accounts(tmp_path):
    n = BcpdProcess(str(tmp_path / "w1"), extra_args=["-gpu=0", "-keypool=5"])
    n.start()
    try:
        from bitcoincashplus_amd import native
        sec = bytes([5]) * 32
        pub = native.ec_pubkey_create(sec, True)
        watch = native.encode_destination("pubkey", native.hash160(pub), "regtest", None)
        n.rpc.importaddress(watch, "watched", False)
        assert n.rpc.validateaddress(watch)["iswatchonly"] is True
        n.rpc.generatetoaddress(1, watch)
        n.rpc.generate(100)
        assert D(n.rpc.getbalance("*", 1, True)) > D(n.rpc.getbalance("*", 1, False))
        lu = [u for u in n.rpc.listunspent() if u["address"] == watch]
        assert lu and lu[0]["spendable"] is False
        # accounts: move between labels
        n.rpc.move("", "acct2", 1)
        accts = n.rpc.listaccounts()
        assert D(accts["acct2"]) == D(1)
        assert any(t["category"] == "move" for t in n.rpc.listtransactions("*", 50))
        # importprivkey makes the watch-only coin spendable
        wif = native.encode_secret(sec, True, "regtest")
        n.rpc.importprivkey(wif, "now-mine", True)
        assert n.rpc.validateaddress(watch)["ismine"] is True
        lu = [u for u in n.rpc.listunspent() if u["address"] == watch]
        assert lu and lu[0]["spendable"] is True
        n.rpc.keypoolrefill(30)
        assert n.rpc.getwalletinfo()["keypoolsize"] >= 30
        n.rpc.settxfee(0.001)
        assert D(n.rpc.getwalletinfo()["paytxfee"]) == D("0.001")
    finally:
        n.stop()


def test_coin_control_send(tmp_path):
    """Coin control (reference Qt CoinControlDialog + SendCoinsDialog, CCoinControl with
    fAllowOtherInputs = false): only the selected outputs are spent, change goes to the chosen
    address."""
    n = BcpdProcess(str(tmp_path / "cc"), extra_args=["-gpu=0", "-keypool=5"])
    n.start()
    try:
        n.rpc.generate(103)
        coins = sorted(n.rpc.listunspent(), key=lambda c: (c["txid"], c["vout"]))
        assert len(coins) >= 3
        pick = coins[0]
        dest, change = n.rpc.getnewaddress(), n.rpc.getnewaddress()
        r = n.rpc.sendwithcoincontrol({dest: 1}, [{"txid": pick["txid"], "vout": pick["vout"]}], change)
        tx = n.rpc.decoderawtransaction(n.rpc.gettransaction(r["txid"])["hex"])
        assert [(i["txid"], i["vout"]) for i in tx["vin"]] == [(pick["txid"], pick["vout"])]
        outs = {o["scriptPubKey"]["addresses"][0]: o["value"] for o in tx["vout"]}
        assert D(outs[dest]) == D(1) and change in outs
        assert D(outs[change]) == D(pick["amount"]) - 1 - D(r["fee"])
        # more than the selected coin holds: refused, although the wallet could pay it
        other = coins[1]
        with pytest.raises(RPCError):
            n.rpc.sendwithcoincontrol({dest: float(D(other["amount"]) + 1)}, [{"txid": other["txid"], "vout": other["vout"]}])
    finally:
        n.stop()
