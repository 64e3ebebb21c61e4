"""Rescans of importaddress / importpubkey / importprivkey / importmulti, with and without pruning.

Parity: reference test/functional/import-rescan.py. A key-source node makes one address per
import variant (call single/multi x data address/pubkey/privkey x rescan no/yes/late timestamp x
pruned or not) and the miner pays each a distinct amount in one block; a second block comes
past the 2-hour rescan window. Each variant is imported on one of four nodes (pruned or not x
expected to rescan or not, so that one import's rescan never picks up another's payment):
* a rescanning import finds the first payment (balance, one "receive" listtransactions entry
  with the label, address, amount, 2 confirmations, involvesWatchonly for watch-only imports);
* a single-key import with rescan on a pruned node fails with "Rescan is disabled in pruned
  mode" (-4) and imports nothing;
* importmulti with a timestamp past the window (late_timestamp) or without rescan finds nothing;
* a second payment to every address is seen by every importing node that holds the key, whether
  or not it rescanned before.
"""
import collections
import enum
import itertools
import os
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess, RPCError

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

Call = enum.Enum("Call", "single multi")
Data = enum.Enum("Data", "address pub priv")
Rescan = enum.Enum("Rescan", "no yes late_timestamp")
RESCAN_WINDOW = 2 * 60 * 60

ImportNode = collections.namedtuple("ImportNode", "prune rescan")
IMPORT_NODES = [ImportNode(*f) for f in itertools.product((False, True), repeat=2)]


class Variant:
    def __init__(self, call, data, rescan, prune):
        self.call, self.data, self.rescan, self.prune = call, data, rescan, prune

    def do_import(self, timestamp):
        if self.call == Call.single:
            fn = {Data.address: (self.node.rpc.importaddress, self.address["address"]),
                  Data.pub: (self.node.rpc.importpubkey, self.address["pubkey"]),
                  Data.priv: (self.node.rpc.importprivkey, self.key)}[self.data]
            try:
                res, err = fn[0](fn[1], self.label, self.rescan == Rescan.yes), None
            except RPCError as e:
                res, err = None, (e.code, str(e))
            assert res is None
            if self.expect_disabled:
                assert err is not None and err[0] == -4 and "Rescan is disabled in pruned mode" in err[1], err
            else:
                assert err is None, err
        else:
            res = self.node.rpc.importmulti([{
                "scriptPubKey": {"address": self.address["address"]},
                "timestamp": timestamp + RESCAN_WINDOW + (1 if self.rescan == Rescan.late_timestamp else 0),
                "pubkeys": [self.address["pubkey"]] if self.data == Data.pub else [],
                "keys": [self.key] if self.data == Data.priv else [],
                "label": self.label,
                "watchonly": self.data != Data.priv,
            }], {"rescan": self.rescan in (Rescan.yes, Rescan.late_timestamp)})
            assert res == [{"success": True}], res

    def check(self, txid=None, amount=None, confirmations=None):
        assert Decimal(str(self.node.rpc.getbalance(self.label, 0, True))) == self.expected_balance, self.label
        txs = self.node.rpc.listtransactions(self.label, 10000, 0, True)
        assert len(txs) == self.expected_txs, (self.label, txs)
        if txid is not None:
            tx, = [t for t in txs if t["txid"] == txid]
            assert tx["account"] == self.label
            assert tx["address"] == self.address["address"]
            assert Decimal(str(tx["amount"])) == amount
            assert tx["category"] == "receive"
            assert tx["label"] == self.label
            assert tx["confirmations"] == confirmations
            assert "trusted" not in tx
            if self.data != Data.priv:
                assert tx["involvesWatchonly"] is True
            else:
                assert "involvesWatchonly" not in tx


def wait_until(pred, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.1)
    raise AssertionError("timeout")


def test_import_rescan(tmp_path):
    variants = [Variant(*v) for v in itertools.product(Call, Data, Rescan, (False, True))]
    nodes = [BcpdProcess(str(tmp_path / f"n{i}"), extra_args=["-gpu=0"] + (["-prune=1"] if i >= 2 and IMPORT_NODES[i - 2].prune else []))
             for i in range(2 + len(IMPORT_NODES))]
    for n in nodes:
        n.start()
    try:
        miner, source = nodes[0], nodes[1]
        for n in nodes[1:]:
            n.rpc.addnode(f"127.0.0.1:{miner.p2p_port}", "onetry")
        miner.rpc.generate(150)
        wait_until(lambda: all(n.rpc.getblockcount() == 150 for n in nodes))
        for i, v in enumerate(variants):
            v.label = f"label {i} {v.call.name} {v.data.name} {v.rescan.name} {v.prune}"
            v.address = source.rpc.validateaddress(source.rpc.getnewaddress(v.label))
            v.key = source.rpc.dumpprivkey(v.address["address"])
            v.initial_amount = Decimal(10) - Decimal(i + 1) / 4
            v.initial_txid = miner.rpc.sendtoaddress(v.address["address"], float(v.initial_amount))
        # the payments' block, then one past the rescan window
        miner.rpc.generate(1)
        assert miner.rpc.getrawmempool() == []
        timestamp = miner.rpc.getblockheader(miner.rpc.getbestblockhash())["time"]
        for n in nodes:
            n.rpc.setmocktime(timestamp + RESCAN_WINDOW + 1)
        miner.rpc.generate(1)
        wait_until(lambda: all(n.rpc.getblockcount() == 152 for n in nodes))

        for v in variants:
            v.expect_disabled = v.rescan == Rescan.yes and v.prune and v.call == Call.single
            expect_rescan = v.rescan == Rescan.yes and not v.expect_disabled
            v.node = nodes[2 + IMPORT_NODES.index(ImportNode(v.prune, expect_rescan))]
            v.do_import(timestamp)
            if expect_rescan:
                v.expected_balance, v.expected_txs = v.initial_amount, 1
                v.check(v.initial_txid, v.initial_amount, 2)
            else:
                v.expected_balance, v.expected_txs = Decimal(0), 0
                v.check()

        # a second payment to every address reaches every node that imported it
        for i, v in enumerate(variants):
            v.sent_amount = Decimal(10) - Decimal(2 * i + 1) / 8
            v.sent_txid = miner.rpc.sendtoaddress(v.address["address"], float(v.sent_amount))
        miner.rpc.generate(1)
        assert miner.rpc.getrawmempool() == []
        wait_until(lambda: all(n.rpc.getblockcount() == 153 for n in nodes))
        for v in variants:
            if not v.expect_disabled:
                v.expected_balance += v.sent_amount
                v.expected_txs += 1
                v.check(v.sent_txid, v.sent_amount, 1)
            else:
                v.check()
    finally:
        for n in nodes:
            n.stop()
