"""Reference RPC scenarios that had no test here, against a live regtest bcpd.

Parity (reference test/functional/):
* merkle_blocks.py: gettxoutproof / verifytxoutproof — proofs for one and two transactions, with
  and without the block hash, no proof for an unconfirmed transaction, none for a fully spent
  one unless its block is named or the node keeps -txindex.
* listsinceblock.py: after a reorg, listsinceblock(<block of the losing branch>) finds the fork
  point and reports the transaction confirmed on the winning branch.
* preciousblock.py: two equal-work tips; preciousblock switches the active tip back and forth,
  and a longer chain still wins.
* zapwallettxes.py: -zapwallettxes drops the unconfirmed wallet transactions and the rescan
  restores the confirmed ones (-persistmempool=0, so the mempool does not re-add them).
* prioritise_transaction.py: fee and priority deltas show in getmempoolentry and decide which
  transactions a block template takes.
* importprunedfunds.py: importprunedfunds with a txoutproof adds the coin without a rescan;
  removeprunedfunds drops it again.
* receivedby.py: listreceivedbyaccount / getreceivedbyaccount.
* importmulti.py: the request shapes (address, scriptPubKey, pubkeys, keys, P2SH redeem
  script, watch-only, internal, timestamps) and their error codes.
* -usecashaddr (reference src/init.cpp:2119-2120): destinations print as Base58 unless
  -usecashaddr=1; both forms are accepted as input.
"""
import os
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess, RPCError

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def D(x):
    return Decimal(str(x))


def wait_until(pred, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.05)
    raise AssertionError("timeout")


def connect(a, b):
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    wait_until(lambda: a.rpc.getconnectioncount() >= 1 and b.rpc.getconnectioncount() >= 1)


def disconnect(a, b):
    for p in a.rpc.getpeerinfo():
        a.rpc.disconnectnode(p["addr"])
    wait_until(lambda: a.rpc.getconnectioncount() == 0 and b.rpc.getconnectioncount() == 0)


def sync_tip(*nodes, timeout=60):
    wait_until(lambda: len({n.rpc.getbestblockhash() for n in nodes}) == 1, timeout)


def raises(code, fn, *args):
    with pytest.raises(RPCError) as e:
        fn(*args)
    if code is not None:
        assert e.value.code == code, (e.value.code, str(e.value))
    return e.value


def node(tmp_path, name, *args):
    n = BcpdProcess(str(tmp_path / name), extra_args=["-gpu=0", *args])
    n.start()
    return n


def test_address_format_default(tmp_path):
    a = node(tmp_path, "a")
    b = node(tmp_path, "b", "-usecashaddr=1")
    try:
        base58 = a.rpc.getnewaddress()
        assert ":" not in base58 and base58[0] in "mn2", base58  # regtest P2PKH Base58
        assert a.rpc.getrawchangeaddress()[0] in "mn"
        cash = b.rpc.getnewaddress()
        assert cash.startswith("bcpreg:"), cash
        # both encodings are accepted as input, and each node prints its own format
        info = a.rpc.validateaddress(cash)
        assert info["isvalid"] and ":" not in info["address"]
        info = b.rpc.validateaddress(base58)
        assert info["isvalid"] and info["address"].startswith("bcpreg:")
        a.rpc.generatetoaddress(1, cash)
        blk = a.rpc.getblock(a.rpc.getbestblockhash(), 2)
        assert blk["tx"][0]["vout"][0]["scriptPubKey"]["addresses"][0][0] in "mn"
    finally:
        a.stop()
        b.stop()


def test_merkle_blocks(tmp_path):
    a = node(tmp_path, "a")
    b = node(tmp_path, "b", "-txindex=1")
    try:
        a.rpc.generate(105)
        connect(a, b)
        sync_tip(a, b)
        height = a.rpc.getblockcount()
        utxos = a.rpc.listunspent(1)
        dest = b.rpc.getnewaddress()

        def pay(u):
            raw = a.rpc.createrawtransaction([{"txid": u["txid"], "vout": u["vout"]}],
                                             {dest: float(D(u["amount"]) - D("0.01"))})
            return a.rpc.sendrawtransaction(a.rpc.signrawtransaction(raw, None, None, "ALL|FORKID")["hex"])

        txid1, txid2 = pay(utxos.pop()), pay(utxos.pop())
        raises(None, a.rpc.gettxoutproof, [txid1])  # not yet in a block
        a.rpc.generate(1)
        blockhash = a.rpc.getblockhash(height + 1)
        sync_tip(a, b)
        txlist = a.rpc.getblock(blockhash, True)["tx"][1:3]
        assert sorted(txlist) == sorted([txid1, txid2])
        assert b.rpc.verifytxoutproof(b.rpc.gettxoutproof([txid1])) == [txid1]
        assert b.rpc.verifytxoutproof(b.rpc.gettxoutproof([txid1, txid2])) == txlist
        assert b.rpc.verifytxoutproof(b.rpc.gettxoutproof([txid1, txid2], blockhash)) == txlist
        # spend txid1's only output completely on node b
        spent = [u for u in b.rpc.listunspent(1) if u["txid"] == txid1][0]
        raw = b.rpc.createrawtransaction([{"txid": txid1, "vout": spent["vout"]}],
                                         {a.rpc.getnewaddress(): float(D(spent["amount"]) - D("0.01"))})
        a.rpc.sendrawtransaction(b.rpc.signrawtransaction(raw, None, None, "ALL|FORKID")["hex"])
        a.rpc.generate(1)
        sync_tip(a, b)
        raises(None, a.rpc.gettxoutproof, [txid1])  # fully spent, no -txindex, no block named
        assert a.rpc.verifytxoutproof(a.rpc.gettxoutproof([txid1], blockhash)) == [txid1]
        assert a.rpc.verifytxoutproof(a.rpc.gettxoutproof([txid2])) == [txid2]  # unspent output: found
        assert a.rpc.verifytxoutproof(b.rpc.gettxoutproof([txid1])) == [txid1]  # -txindex node finds it
        # a proof whose merkle root is not in the chain verifies to nothing
        proof = bytearray.fromhex(b.rpc.gettxoutproof([txid1]))
        proof[40] ^= 1  # inside the merkle root field of the header
        assert b.rpc.verifytxoutproof(proof.hex()) == []
    finally:
        a.stop()
        b.stop()


def test_listsinceblock_after_reorg(tmp_path):
    a = node(tmp_path, "a")
    b = node(tmp_path, "b")
    try:
        a.rpc.generate(101)
        connect(a, b)
        sync_tip(a, b)
        disconnect(a, b)
        # a (the longer side) pays b; b mines a shorter branch of its own meanwhile
        senttx = a.rpc.sendtoaddress(b.rpc.getnewaddress(), 1)
        a.rpc.generate(7)
        lastblockhash = b.rpc.generate(6)[5]
        connect(a, b)
        sync_tip(a, b)
        assert b.rpc.getbestblockhash() == a.rpc.getbestblockhash()
        res = b.rpc.listsinceblock(lastblockhash)
        assert any(t["txid"] == senttx for t in res["transactions"])
        assert res["lastblock"] == b.rpc.getbestblockhash()
        # from the tip: nothing confirmed is new (the orphaned coinbases of b's losing branch are
        # still listed, with depth 0, as in the reference)
        assert all(t["category"] == "orphan" or t["confirmations"] < 1
                   for t in b.rpc.listsinceblock(b.rpc.getbestblockhash())["transactions"])
    finally:
        a.stop()
        b.stop()


def sync_via_rpc(src, dst):
    """Copy the blocks dst lacks from src by submitblock (reference preciousblock.py)."""
    todo = []
    h = src.rpc.getbestblockhash()
    while True:
        try:
            dst.rpc.getblockheader(h)
            break
        except RPCError:
            todo.append(h)
            h = src.rpc.getblockheader(h)["previousblockhash"]
    for h in reversed(todo):
        assert dst.rpc.submitblock(src.rpc.getblock(h, False)) in (None, "inconclusive")


def test_preciousblock(tmp_path):
    n0 = node(tmp_path, "n0")
    n1 = node(tmp_path, "n1")
    try:
        n0.rpc.generate(1)
        _, hashZ = n1.rpc.generate(2)
        sync_via_rpc(n1, n0)
        sync_via_rpc(n0, n1)
        assert n0.rpc.getbestblockhash() == hashZ
        hashC = n0.rpc.generate(3)[2]
        hashG = n1.rpc.generate(3)[2]
        assert hashC != hashG
        sync_via_rpc(n0, n1)
        sync_via_rpc(n1, n0)
        # equal work: each keeps the tip it saw first
        assert n0.rpc.getbestblockhash() == hashC
        assert n1.rpc.getbestblockhash() == hashG
        n0.rpc.preciousblock(hashG)
        assert n0.rpc.getbestblockhash() == hashG
        n0.rpc.preciousblock(hashC)
        assert n0.rpc.getbestblockhash() == hashC
        n1.rpc.preciousblock(hashC)
        assert n1.rpc.getbestblockhash() == hashC
        n1.rpc.preciousblock(hashG)
        assert n1.rpc.getbestblockhash() == hashG
        # more work beats precious
        hashH = n0.rpc.generate(1)[0]
        sync_via_rpc(n0, n1)
        assert n1.rpc.getbestblockhash() == hashH
        n1.rpc.preciousblock(hashG)  # less work: no effect
        assert n1.rpc.getbestblockhash() == hashH
        raises(-5, n1.rpc.preciousblock, "00" * 32)  # unknown block
    finally:
        n0.stop()
        n1.stop()


def test_zapwallettxes(tmp_path):
    a = node(tmp_path, "a", "-persistmempool=0")
    try:
        a.rpc.generate(101)
        dst = a.rpc.getnewaddress()
        txid0 = a.rpc.sendtoaddress(dst, 11)
        txid1 = a.rpc.sendtoaddress(dst, 10)
        a.rpc.generate(1)
        txid2 = a.rpc.sendtoaddress(dst, 11)
        txid3 = a.rpc.sendtoaddress(dst, 10)
        for t in (txid0, txid1, txid2, txid3):
            assert a.rpc.gettransaction(t)["txid"] == t
        a.stop()
        a.start()
        assert a.rpc.gettransaction(txid3)["txid"] == txid3  # the wallet keeps unconfirmed ones
        a.stop()
        a.extra_args = a.extra_args + ["-zapwallettxes=1"]
        a.start()
        raises(-5, a.rpc.gettransaction, txid3)  # zapped, and no mempool to bring it back
        raises(-5, a.rpc.gettransaction, txid2)
        assert a.rpc.gettransaction(txid0)["txid"] == txid0  # confirmed: restored by the rescan
        assert a.rpc.gettransaction(txid1)["confirmations"] == 1
    finally:
        a.stop()


def test_prioritisetransaction(tmp_path):
    a = node(tmp_path, "a", "-printpriority=1", "-blockmaxsize=2000", "-blockprioritysize=0")
    try:
        a.rpc.generate(110)
        dst = a.rpc.getnewaddress()
        txids = [a.rpc.sendtoaddress(dst, 1) for _ in range(12)]
        base = {t: D(a.rpc.getmempoolentry(t)["modifiedfee"]) for t in txids}
        low = txids[5]
        # a large negative fee delta sends one transaction to the back, a positive one to the front
        a.rpc.prioritisetransaction(low, 0, -10**8)
        assert D(a.rpc.getmempoolentry(low)["modifiedfee"]) == base[low] - 1
        high = txids[7]
        a.rpc.prioritisetransaction(high, 0, 10**8)
        assert D(a.rpc.getmempoolentry(high)["modifiedfee"]) == base[high] + 1
        # deltas accumulate
        a.rpc.prioritisetransaction(high, 0, 5 * 10**7)
        assert D(a.rpc.getmempoolentry(high)["modifiedfee"]) == base[high] + D("1.5")
        from bitcoincashplus_amd.testing.p2p import P2PPeer
        peer = P2PPeer().connect("127.0.0.1", a.p2p_port)  # templates need a connected node
        tmpl = a.rpc.getblocktemplate()
        peer.close()
        picked = [t["txid"] for t in tmpl["transactions"]]
        assert high in picked and low not in picked
        assert picked[0] == high  # highest modified fee rate first
        # a delta for a transaction not (yet) in the mempool is kept and applied on arrival
        raw = a.rpc.createrawtransaction([], {dst: 1})
        funded = a.rpc.fundrawtransaction(raw)["hex"]
        signed = a.rpc.signrawtransaction(funded)["hex"]
        pending = a.rpc.decoderawtransaction(signed)["txid"]
        assert a.rpc.prioritisetransaction(pending, 0, 10**6) is True
        a.rpc.sendrawtransaction(signed)
        e = a.rpc.getmempoolentry(pending)
        assert D(e["modifiedfee"]) == D(e["fee"]) + D("0.01")
    finally:
        a.stop()


def test_importprunedfunds_and_removeprunedfunds(tmp_path):
    n0 = node(tmp_path, "n0")
    n1 = node(tmp_path, "n1")
    try:
        n0.rpc.generate(101)
        connect(n0, n1)
        sync_tip(n0, n1)
        address1, address2, address3 = (n0.rpc.getnewaddress() for _ in range(3))
        address3_privkey = n0.rpc.dumpprivkey(address3)
        for a in (address1, address2, address3):
            info = n1.rpc.validateaddress(a)
            assert not info["ismine"] and not info["iswatchonly"]
        raw, proof, txid = {}, {}, {}
        for i, (a, v) in enumerate(((address1, 0.1), (address2, 0.05), (address3, 0.025)), 1):
            txid[i] = n0.rpc.sendtoaddress(a, v)
            n0.rpc.generate(1)
            raw[i] = n0.rpc.gettransaction(txid[i])["hex"]
            proof[i] = n0.rpc.gettxoutproof([txid[i]])
        sync_tip(n0, n1)
        e = raises(-5, n1.rpc.importprunedfunds, raw[1], proof[1])
        assert "No addresses" in str(e)
        assert D(n1.rpc.getbalance("", 0, True)) == 0
        n1.rpc.importaddress(address2, "add2", False)
        n1.rpc.importprunedfunds(raw[2], proof[2])
        assert D(n1.rpc.getbalance("add2", 0, True)) == D("0.05")
        n1.rpc.importprivkey(address3_privkey, "add3", False)
        n1.rpc.importprunedfunds(raw[3], proof[3])
        assert D(n1.rpc.getbalance("add3", 0, False)) == D("0.025")
        assert D(n1.rpc.getbalance("*", 0, True)) == D("0.075")
        raises(-5, n1.rpc.importprunedfunds, raw[3], proof[2])  # "Transaction given doesn't exist in proof"
        # removeprunedfunds
        raises(-8, n1.rpc.removeprunedfunds, txid[1])  # never in this wallet
        n1.rpc.removeprunedfunds(txid[2])
        assert D(n1.rpc.getbalance("*", 0, True)) == D("0.025")
        n1.rpc.removeprunedfunds(txid[3])
        assert D(n1.rpc.getbalance("*", 0, True)) == 0
        raises(-5, n1.rpc.gettransaction, txid[3])
    finally:
        n0.stop()
        n1.stop()


def test_received_by_account(tmp_path):
    a = node(tmp_path, "a")
    b = node(tmp_path, "b")
    try:
        a.rpc.generate(101)
        connect(a, b)
        sync_tip(a, b)
        addr = b.rpc.getnewaddress("acct")
        txid = a.rpc.sendtoaddress(addr, 0.1)
        wait_until(lambda: txid in b.rpc.getrawmempool())
        assert D(b.rpc.getreceivedbyaccount("acct", 0)) == D("0.1")
        assert D(b.rpc.getreceivedbyaccount("acct")) == 0  # minconf 1
        a.rpc.generate(1)
        sync_tip(a, b)
        rows = {r["account"]: r for r in b.rpc.listreceivedbyaccount()}
        assert D(rows["acct"]["amount"]) == D("0.1") and rows["acct"]["confirmations"] == 1
        assert "" not in rows  # empty accounts only with include_empty
        rows = {r["account"]: r for r in b.rpc.listreceivedbyaccount(0, True)}
        assert "" in rows and D(rows[""]["amount"]) == 0
        assert D(b.rpc.getreceivedbyaccount("acct", 2)) == 0
        a.rpc.generate(1)
        sync_tip(a, b)
        assert D(b.rpc.getreceivedbyaccount("acct", 2)) == D("0.1")
        rows = {r["address"]: r for r in b.rpc.listreceivedbyaddress()}
        assert rows[addr]["txids"] == [txid]
    finally:
        a.stop()
        b.stop()


def test_importmulti(tmp_path):
    a = node(tmp_path, "a")
    b = node(tmp_path, "b")
    try:
        a.rpc.generate(1)
        now = a.rpc.getblockheader(a.rpc.getbestblockhash())["mediantime"]

        def fresh():
            addr = b.rpc.getnewaddress()
            return b.rpc.validateaddress(addr)

        # bitcoin address
        info = fresh()
        r = a.rpc.importmulti([{"scriptPubKey": {"address": info["address"]}, "timestamp": "now"}])
        assert r == [{"success": True}]
        got = a.rpc.validateaddress(info["address"])
        assert got["iswatchonly"] and not got["ismine"]
        # scriptPubKey without internal: error
        info = fresh()
        r = a.rpc.importmulti([{"scriptPubKey": info["scriptPubKey"], "timestamp": "now"}])
        assert not r[0]["success"] and r[0]["error"]["code"] == -8
        assert r[0]["error"]["message"] == "Internal must be set for hex scriptPubKey"
        r = a.rpc.importmulti([{"scriptPubKey": info["scriptPubKey"], "timestamp": "now", "internal": True}])
        assert r == [{"success": True}]
        assert a.rpc.validateaddress(info["address"])["iswatchonly"]
        # address + public key
        info = fresh()
        r = a.rpc.importmulti([{"scriptPubKey": {"address": info["address"]}, "timestamp": "now",
                                "pubkeys": [info["pubkey"]]}])
        assert r == [{"success": True}]
        assert a.rpc.validateaddress(info["address"])["iswatchonly"]
        # address + private key: spendable
        info = fresh()
        r = a.rpc.importmulti([{"scriptPubKey": {"address": info["address"]}, "timestamp": "now",
                                "keys": [b.rpc.dumpprivkey(info["address"])]}])
        assert r == [{"success": True}]
        got = a.rpc.validateaddress(info["address"])
        assert got["ismine"] and not got["iswatchonly"]
        # private key together with watchonly: error
        info = fresh()
        r = a.rpc.importmulti([{"scriptPubKey": {"address": info["address"]}, "timestamp": "now",
                                "keys": [b.rpc.dumpprivkey(info["address"])], "watchonly": True}])
        assert not r[0]["success"] and r[0]["error"]["code"] == -8
        assert r[0]["error"]["message"] == "Incompatibility found between watchonly and keys"
        # key that does not match the address: error
        info, other = fresh(), fresh()
        r = a.rpc.importmulti([{"scriptPubKey": {"address": info["address"]}, "timestamp": "now",
                                "keys": [b.rpc.dumpprivkey(other["address"])]}])
        assert not r[0]["success"] and r[0]["error"]["code"] == -5
        assert r[0]["error"]["message"] == "Consistency check failed"
        # P2SH multisig with redeem script: watch-only until the keys come too
        k1, k2, k3 = fresh(), fresh(), fresh()
        ms = b.rpc.createmultisig(2, [k1["pubkey"], k2["pubkey"], k3["pubkey"]])
        r = a.rpc.importmulti([{"scriptPubKey": {"address": ms["address"]}, "timestamp": "now",
                                "redeemscript": ms["redeemScript"]}])
        assert r == [{"success": True}]
        assert a.rpc.validateaddress(ms["address"])["isscript"]
        # invalid address: error, and a batch reports each request
        r = a.rpc.importmulti([{"scriptPubKey": {"address": "not-an-address"}, "timestamp": "now"},
                               {"scriptPubKey": {"address": fresh()["address"]}, "timestamp": "now"}])
        assert not r[0]["success"] and r[0]["error"]["code"] == -5
        assert r[0]["error"]["message"] == "Invalid address"
        assert r[1] == {"success": True}
        # timestamp is required, "now" or a number
        raises(-3, a.rpc.importmulti, [{"scriptPubKey": {"address": fresh()["address"]}}])
        r = a.rpc.importmulti([{"scriptPubKey": {"address": fresh()["address"]}, "timestamp": now}])
        assert r == [{"success": True}]
        # rescan option false: no rescan, still imported
        info = fresh()
        r = a.rpc.importmulti([{"scriptPubKey": {"address": info["address"]}, "timestamp": "now"}],
                              {"rescan": False})
        assert r == [{"success": True}]
    finally:
        a.stop()
        b.stop()
