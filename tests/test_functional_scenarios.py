"""Functional scenarios ported from the reference's test/functional/ (each against a real bcpd):

* pruning.py: manual pruning (-prune=1) over many small block files (-fastprune), pruned blocks
  unavailable, prune height reported, restart keeps working;
* mempool_limit.py: a small -maxmempool evicts the cheapest package and raises the minimum fee;
* mempool_packages.py: the 25-transaction ancestor limit (-limitancestorcount);
* mempool_reorg.py: transactions of a disconnected block return to the mempool;
* getblocktemplate_longpoll.py: a long poll returns when a block arrives;
* getblocktemplate_proposals.py: BIP23 proposals - a valid block, a bad merkle root, a stale parent;
* abandonconflict.py: abandontransaction on a transaction that cannot confirm frees its inputs.
"""
import os
import threading
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase
from bitcoincashplus_amd.testing.messages import CTransaction, from_hex
from bitcoincashplus_amd.testing.p2p import P2PPeer

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def start(tmp_path, name, *args):
    n = BcpdProcess(str(tmp_path / name), extra_args=["-gpu=0", *args])
    n.start()
    return n


def test_manual_pruning(tmp_path):
    n = start(tmp_path, "p", "-prune=1", "-fastprune")
    try:
        addr = n.rpc.getnewaddress()
        # blocks with some payload so many 64 KiB block files fill up
        n.rpc.generatetoaddress(101, addr)  # a mature coinbase to spend from
        for _ in range(11):
            for _ in range(3):
                n.rpc.sendtoaddress(n.rpc.getnewaddress(), 1)
            n.rpc.generatetoaddress(100, addr)
        height = n.rpc.getblockcount()
        assert height == 1201
        files = sorted(f for f in os.listdir(os.path.join(n.datadir, "regtest", "blocks")) if f.startswith("blk"))
        assert len(files) > 4
        info = n.rpc.getblockchaininfo()
        assert info["pruned"] is True
        pruned_to = n.rpc.pruneblockchain(700)
        assert 0 < pruned_to <= 700
        info = n.rpc.getblockchaininfo()
        assert 0 < info["pruneheight"] <= 700
        low = n.rpc.getblockhash(5)
        with pytest.raises(Exception, match="pruned"):
            n.rpc.getblock(low)
        # recent blocks stay readable; files really went away
        n.rpc.getblock(n.rpc.getblockhash(height - 10))
        after = sorted(f for f in os.listdir(os.path.join(n.datadir, "regtest", "blocks")) if f.startswith("blk"))
        assert len(after) < len(files)
        port = n.rpcport
    finally:
        n.stop()
    # restart on the pruned store, and keep extending the chain
    n2 = BcpdProcess(n.datadir, extra_args=["-gpu=0", "-prune=1", "-fastprune"], port=port)
    n2.start()
    try:
        assert n2.rpc.getblockcount() == height
        n2.rpc.generate(5)
        assert n2.rpc.getblockchaininfo()["pruneheight"] > 0
    finally:
        n2.stop()


def test_mempool_limit_and_packages(tmp_path):
    n = start(tmp_path, "m", "-maxmempool=5", "-limitancestorcount=25", "-spendzeroconfchange=1")
    try:
        n.rpc.generate(230)  # 130 mature coinbases
        info = n.rpc.getmempoolinfo()
        assert Decimal(str(info["mempoolminfee"])) == 0
        # ancestor limit: a chain of 25 unconfirmed transactions, the 26th refused
        addr = n.rpc.getnewaddress()
        utxo = next(u for u in n.rpc.listunspent() if Decimal(str(u["amount"])) >= 10)
        prev, value = (utxo["txid"], utxo["vout"]), Decimal(str(utxo["amount"]))
        for i in range(26):
            value -= Decimal("0.001")
            raw = n.rpc.createrawtransaction([{"txid": prev[0], "vout": prev[1]}], {addr: float(value)})
            signed = n.rpc.signrawtransaction(raw)["hex"]
            if i < 25:
                prev = (n.rpc.sendrawtransaction(signed), 0)
            else:
                with pytest.raises(Exception, match="too-long-mempool-chain"):
                    n.rpc.sendrawtransaction(signed)
        assert n.rpc.getmempoolinfo()["size"] == 25
        n.rpc.generate(1)
        # fill a 5 MB mempool with big low-fee transactions until eviction raises the floor
        big_out = {n.rpc.getnewaddress(): 0.0001 for _ in range(1500)}  # ~50 kB each
        sent = 0
        while Decimal(str(n.rpc.getmempoolinfo()["mempoolminfee"])) == 0 and sent < 120:
            us = [u for u in n.rpc.listunspent() if Decimal(str(u["amount"])) >= 1][:1]
            assert us
            raw = n.rpc.createrawtransaction([{"txid": us[0]["txid"], "vout": us[0]["vout"]}],
                                             {**big_out, addr: float(Decimal(str(us[0]["amount"])) - Decimal("0.2"))})
            try:
                n.rpc.sendrawtransaction(n.rpc.signrawtransaction(raw)["hex"], True)
            except Exception as e:  # the newest, cheapest package itself was evicted
                assert "mempool full" in str(e)
                break
            sent += 1
        info = n.rpc.getmempoolinfo()
        assert Decimal(str(info["mempoolminfee"])) > 0
        assert info["usage"] <= info["maxmempool"]
    finally:
        n.stop()


def test_mempool_reorg_returns_transactions(tmp_path):
    n = start(tmp_path, "r")
    try:
        n.rpc.generate(110)
        txid = n.rpc.sendtoaddress(n.rpc.getnewaddress(), 3)
        assert txid in n.rpc.getrawmempool()
        blk = n.rpc.generate(1)[0]
        assert txid not in n.rpc.getrawmempool()
        n.rpc.invalidateblock(blk)
        assert txid in n.rpc.getrawmempool()  # back from the disconnected block
        n.rpc.reconsiderblock(blk)
        assert n.rpc.getbestblockhash() == blk
        assert txid not in n.rpc.getrawmempool()
    finally:
        n.stop()


def test_getblocktemplate_longpoll_and_proposals(tmp_path):
    n = start(tmp_path, "g")
    peer = None
    try:
        n.rpc.generate(105)
        # templates are refused to a node without peers (-9): a P2P peer keeps one connection up
        peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
        tmpl = n.rpc.getblocktemplate()
        lp = tmpl["longpollid"]
        result = {}

        def poll():
            from bitcoincashplus_amd.node.process import RPCProxy
            p = RPCProxy(n.rpcport, n.user, n.password, timeout=120)
            t0 = time.time()
            result["tmpl"] = p.getblocktemplate({"longpollid": lp})
            result["dt"] = time.time() - t0

        th = threading.Thread(target=poll)
        th.start()
        time.sleep(2)
        assert th.is_alive()  # still waiting: nothing changed
        n.rpc.generate(1)
        th.join(60)
        assert not th.is_alive()
        assert result["tmpl"]["previousblockhash"] == n.rpc.getbestblockhash()
        assert result["dt"] >= 1.5

        # BIP23 proposals on a block built from a fresh template
        tmpl = n.rpc.getblocktemplate()
        height = tmpl["height"]
        cb = create_coinbase(height)
        cb.vout[0].nValue = tmpl["coinbasevalue"]
        cb.rehash()
        txs = [from_hex(CTransaction(), t["data"]) for t in tmpl["transactions"]]
        blk = create_block(int(tmpl["previousblockhash"], 16), cb, tmpl["curtime"], height,
                           int(tmpl["bits"], 16), tmpl["version"], txs)
        assert n.rpc.getblocktemplate({"mode": "proposal", "data": blk.serialize().hex()}) is None
        bad = create_block(int(tmpl["previousblockhash"], 16), cb, tmpl["curtime"], height,
                           int(tmpl["bits"], 16), tmpl["version"], txs)
        bad.hashMerkleRoot ^= 1
        assert n.rpc.getblocktemplate({"mode": "proposal", "data": bad.serialize().hex()}) == "bad-txnmrklroot"
        stale = create_block(int(n.rpc.getblockhash(3), 16), cb, tmpl["curtime"], 4, int(tmpl["bits"], 16),
                             tmpl["version"], [])
        assert n.rpc.getblocktemplate({"mode": "proposal", "data": stale.serialize().hex()}) == \
            "inconclusive-not-best-prevblk"
    finally:
        if peer:
            peer.close()
        n.stop()


def test_abandon_conflicting_transaction(tmp_path):
    n = start(tmp_path, "a")
    try:
        n.rpc.generate(110)
        # a coin one block old: spending it has low priority, so once the relay fee floor is
        # raised the wallet cannot put the spend back into the mempool (reference
        # abandonconflict.py: "make sure tx did not have AllowFree priority")
        young = n.rpc.getnewaddress()
        n.rpc.sendtoaddress(young, 10)
        n.rpc.generate(1)
        utxo = next(u for u in n.rpc.listunspent() if u["address"] == young)
        bal0 = Decimal(str(n.rpc.getbalance()))
        raw = n.rpc.createrawtransaction([{"txid": utxo["txid"], "vout": utxo["vout"]}],
                                         {n.rpc.getnewaddress(): float(Decimal(str(utxo["amount"])) - Decimal("0.001"))})
        txid = n.rpc.sendrawtransaction(n.rpc.signrawtransaction(raw)["hex"])
        assert txid in n.rpc.getrawmempool()
        n.stop()
        n.extra_args += ["-persistmempool=0", "-minrelaytxfee=0.5"]
        n.start()
        assert txid not in n.rpc.getrawmempool()
        # the wallet still counts the coin spent, and the change not received
        assert Decimal(str(n.rpc.getbalance())) == bal0 - Decimal(str(utxo["amount"]))
        with pytest.raises(Exception):
            n.rpc.abandontransaction(n.rpc.getbestblockhash())  # not a wallet transaction
        n.rpc.abandontransaction(txid)
        # the input is spendable again: the full balance is back
        assert Decimal(str(n.rpc.getbalance())) == bal0
        # once abandoned, it is not re-added on startup even at a low relay fee
        n.stop()
        n.extra_args.remove("-minrelaytxfee=0.5")
        n.start()
        assert txid not in n.rpc.getrawmempool()
        assert Decimal(str(n.rpc.getbalance())) == bal0
        n.rpc.sendtoaddress(n.rpc.getnewaddress(), float(bal0 - 1))
    finally:
        n.stop()
