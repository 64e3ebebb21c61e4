"""Wallet behaviour under a double spend across a network split, and fee estimation fed by
real blocks.

Parity:
* reference test/functional/txn_doublespend.py: the network splits. One side confirms a
  payment. The other side mines a conflicting spend of the same coin, made by the same wallet,
  on a longer chain. After the reorg:
  - the payment is conflicted (negative confirmations, listed in walletconflicts);
  - the double spend is confirmed;
  - the balance counts only the double spend.
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
