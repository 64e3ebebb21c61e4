"""Wallet behaviour under a double spend across a network split, and fee estimation fed by
real blocks.

Parity:
* reference test/functional/txn_doublespend.py: the network splits. One side confirms a
  payment. The other side mines a conflicting spend of the same coin, made by the same wallet,
  on a longer chain. After the reorg:
  - the payment is conflicted (negative confirmations, listed in walletconflicts);
  - the double spend is confirmed;
  - the balance counts only the double spend.
* reference test/functional/txn_clone.py: the same split, but the conflicting spend is a malleated
  clone of the payment (signed ALL|FORKID|ANYONECANPAY); account balances follow the clone.
* reference test/functional/smartfees.py: transactions at a spread of fee rates, with blocks too
  small to take all of them, so cheaper ones wait longer. From the estimator's data:
  - estimatefee(n) stays within the range of fee rates that were paid;
  - estimatefee(n) does not increase with n;
  - estimatesmartfee answers for a target at least as long as the one asked for.
"""
import os
import random
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

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
        time.sleep(0.1)
    raise AssertionError("timeout")


def connect(a, b):
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    wait_until(lambda: a.rpc.getconnectioncount() >= 1 and b.rpc.getconnectioncount() >= 1)


def test_txn_doublespend(tmp_path):
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0"])
    b = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpu=0"])
    a.start()
    b.start()
    try:
        a.rpc.generate(110)
        connect(a, b)
        wait_until(lambda: b.rpc.getblockcount() == 110)
        # split the network
        for p in a.rpc.getpeerinfo():
            a.rpc.disconnectnode(p["addr"])
        wait_until(lambda: a.rpc.getconnectioncount() == 0 and b.rpc.getconnectioncount() == 0)
        start_balance = D(a.rpc.getbalance())
        assert start_balance == 10 * 50  # coinbases 1..10 are mature
        # the payment, and a conflicting spend of the same coin back to the wallet itself
        payee = b.rpc.getnewaddress()
        tx1 = a.rpc.sendtoaddress(payee, 40)
        raw1 = a.rpc.getrawtransaction(tx1, 1)
        ins = [{"txid": i["txid"], "vout": i["vout"]} for i in raw1["vin"]]
        in_value = sum(D(a.rpc.getrawtransaction(i["txid"], 1)["vout"][i["vout"]]["value"]) for i in ins)
        fee2 = D("0.001")
        raw2 = a.rpc.createrawtransaction(ins, {a.rpc.getnewaddress(): float(in_value - fee2)})
        tx2hex = a.rpc.signrawtransaction(raw2)["hex"]
        # a confirms the payment on its side
        a.rpc.generate(1)
        assert a.rpc.gettransaction(tx1)["confirmations"] == 1
        # b mines the double spend on a longer chain
        tx2 = b.rpc.sendrawtransaction(tx2hex)
        b.rpc.generate(2)
        # the network rejoins: a reorganises onto b's chain
        connect(a, b)
        wait_until(lambda: a.rpc.getbestblockhash() == b.rpc.getbestblockhash())
        t1 = a.rpc.gettransaction(tx1)
        t2 = a.rpc.gettransaction(tx2)
        assert t1["confirmations"] == -2, t1["confirmations"]  # conflicted by a block 2 deep
        assert tx2 in t1["walletconflicts"]
        assert t2["confirmations"] == 2
        assert tx1 not in a.rpc.getrawmempool()
        # the balance: coinbases 1..12 are mature on the final chain (a mined 1..110; 111 and 112
        # are b's), the coin moved by the double spend lost only its fee, the payment never happened
        wait_until(lambda: D(a.rpc.getbalance()) == 12 * 50 - fee2)
        assert D(b.rpc.getreceivedbyaddress(payee, 0)) == 0
    finally:
        a.stop()
        b.stop()


def test_smartfees(tmp_path):
    # blocks of at most ~20 small transactions, so cheaper ones wait
    n = BcpdProcess(str(tmp_path / "f"), extra_args=["-gpu=0", "-blockmaxsize=6000", "-spendzeroconfchange=1"])
    n.start()
    try:
        n.rpc.generate(130)
        rng = random.Random(7)
        rates = [D("0.00005"), D("0.0001"), D("0.0002"), D("0.0005"), D("0.001")]  # BCP/kB
        addr = n.rpc.getnewaddress()
        # split coins so each round has many independent inputs
        n.rpc.sendmany("", {n.rpc.getnewaddress(): 1 for _ in range(200)})
        n.rpc.generate(1)
        for _ in range(40):
            for _ in range(25):
                n.rpc.settxfee(float(rng.choice(rates)))
                try:
                    n.rpc.sendtoaddress(addr, 0.01)
                except Exception:
                    pass  # out of confirmed coins this round: the next block frees some
            n.rpc.generate(1)
        lo, hi = min(rates), max(rates)
        prev = None
        seen = 0
        for target in range(1, 26):
            e = n.rpc.estimatefee(target)
            if e == -1:
                continue
            seen += 1
            e = D(e)
            # within the paid range (the estimator reports bucket boundaries: allow its spacing)
            assert lo / 2 <= e <= hi * 2, (target, e)
            if prev is not None:
                assert e <= prev, (target, e, prev)
            prev = e
        assert seen >= 1
        s = n.rpc.estimatesmartfee(2)
        assert s["blocks"] >= 2 or D(s["feerate"]) == -1
        if D(s["feerate"]) != -1:
            assert lo / 2 <= D(s["feerate"]) <= hi * 2
    finally:
        n.stop()


def test_txn_clone(tmp_path):
    """reference test/functional/txn_clone.py: a malleated clone of a wallet payment (same input
    and outputs, signed ALL|FORKID|ANYONECANPAY) is mined on the other side of a split and wins."""
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0"])
    b = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpu=0"])
    a.start()
    b.start()
    try:
        a.rpc.generate(110)
        connect(a, b)
        wait_until(lambda: b.rpc.getblockcount() == 110)
        for p in a.rpc.getpeerinfo():
            a.rpc.disconnectnode(p["addr"])
        wait_until(lambda: a.rpc.getconnectioncount() == 0 and b.rpc.getconnectioncount() == 0)
        starting = D(a.rpc.getbalance())
        assert starting == 500
        a.rpc.getnewaddress("")
        a.rpc.settxfee(0.001)
        fund_foo_txid = a.rpc.sendfrom("", a.rpc.getnewaddress("foo"), 219)
        fund_foo = a.rpc.gettransaction(fund_foo_txid)
        fund_bar_txid = a.rpc.sendfrom("", a.rpc.getnewaddress("bar"), 29)
        fund_bar = a.rpc.gettransaction(fund_bar_txid)
        assert D(a.rpc.getbalance("")) == starting - 219 - 29 + D(fund_foo["fee"]) + D(fund_bar["fee"])
        to_b = b.rpc.getnewaddress("from0")
        txid1 = a.rpc.sendfrom("foo", to_b, 40, 0)
        txid2 = a.rpc.sendfrom("bar", to_b, 20, 0)
        # the clone: tx1's input and outputs, another signature hash type
        raw1 = a.rpc.getrawtransaction(txid1, 1)
        assert len(raw1["vin"]) == 1
        outs = {o["scriptPubKey"]["addresses"][0]: float(o["value"]) for o in raw1["vout"]}
        clone_raw = a.rpc.createrawtransaction([{"txid": raw1["vin"][0]["txid"], "vout": raw1["vin"][0]["vout"]}],
                                               outs, raw1["locktime"])
        clone = a.rpc.signrawtransaction(clone_raw, None, None, "ALL|FORKID|ANYONECANPAY")
        assert clone["complete"]
        tx1 = a.rpc.gettransaction(txid1)
        tx2 = a.rpc.gettransaction(txid2)
        expected = starting + D(fund_foo["fee"]) + D(fund_bar["fee"])
        expected += D(tx1["amount"]) + D(tx1["fee"]) + D(tx2["amount"]) + D(tx2["fee"])
        assert D(a.rpc.getbalance()) == expected
        assert D(a.rpc.getbalance("foo", 0)) == 219 + D(tx1["amount"]) + D(tx1["fee"])
        assert D(a.rpc.getbalance("bar", 0)) == 29 + D(tx2["amount"]) + D(tx2["fee"])
        assert tx1["confirmations"] == 0 and tx2["confirmations"] == 0
        # the clone (and its parent) are mined on b's side
        b.rpc.sendrawtransaction(fund_foo["hex"])
        clone_txid = b.rpc.sendrawtransaction(clone["hex"])
        assert clone_txid != txid1
        b.rpc.generate(1)
        connect(a, b)
        b.rpc.sendrawtransaction(fund_bar["hex"])
        b.rpc.sendrawtransaction(tx2["hex"])
        b.rpc.generate(1)
        wait_until(lambda: a.rpc.getbestblockhash() == b.rpc.getbestblockhash())
        tx1 = a.rpc.gettransaction(txid1)
        tx1_clone = a.rpc.gettransaction(clone_txid)
        tx2 = a.rpc.gettransaction(txid2)
        assert tx1["confirmations"] == -2
        assert tx1_clone["confirmations"] == 2
        assert tx2["confirmations"] == 1
        # two more coinbases matured; the clone moved exactly what tx1 would have
        expected += 100
        wait_until(lambda: D(a.rpc.getbalance()) == expected)
        assert D(a.rpc.getbalance("*", 0)) == expected
        assert D(a.rpc.getbalance("foo")) == 219 + D(tx1["amount"]) + D(tx1["fee"])
        assert D(a.rpc.getbalance("bar", 0)) == 29 + D(tx2["amount"]) + D(tx2["fee"])
        assert D(a.rpc.getbalance("", 0)) == starting - 219 + D(fund_foo["fee"]) - 29 + D(fund_bar["fee"]) + 100
        assert D(b.rpc.getbalance("from0", 0)) == -(D(tx1["amount"]) + D(tx2["amount"]))
    finally:
        a.stop()
        b.stop()
