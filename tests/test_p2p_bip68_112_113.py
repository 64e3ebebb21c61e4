"""CSV soft fork activation and enforcement over the P2P wire: BIP68, BIP112, BIP113.

Parity: reference test/functional/bip68-112-113-p2p.py, TestInstance by TestInstance (the
numbers in the comments are the reference's). One node (-whitelist, -blockversion=4) fed blocks
by a P2P peer; the node's wallet makes and signs the transactions, as there.

The schedule runs 20 retarget periods (2880 blocks) later than the reference's, past the
regtest BCP fork at 3000: on the reference a block whose scripts fail the parallel check is
still accepted below BCPHeight (src/validation.cpp:2121-2126, "Before fork happens ... block
validation fails even if block is valid"), so its BIP112 rejections (32-123) hold only after the
fork (the reference's own script, with regtest BCPHeight = 3000, runs below it). The node mines
the first 3023 blocks with mock time (no CSV signal: -blockversion=4), so the deployment is
STARTED where the reference's step 1 leaves it; the inputs are the coinbases of blocks 1-82.
* deployment (2-5): 100 of 144 signalling stays STARTED (mixed version bits); 108 of 144 locks
  in; inputs seeded at height 3452; still LOCKED_IN at 3454;
* before activation (6-7): every BIP68 / BIP112 / BIP113 transaction, version 1 and 2, is valid;
* ACTIVE at 575 (8);
* BIP113 (9-12): nLockTime must be below the median time past, whatever the tx version;
* BIP68 (14-31): version 1 unaffected; version 2 with the disable flag unaffected; relative
  height and time locks fail until 10 blocks / 10 * 512 s have passed (time at 581, height at 582);
* BIP112 (32-125): a negative CSV argument fails; a disable flag in the CSV argument passes;
  version 1 spends of CSV outputs fail otherwise; version 2: nSequence 9 against CSV 10 fails,
  a disable flag in nSequence fails, mismatched lock types fail, the remaining combinations
  pass (masking), and two time-type locks compare.
"""
import os
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver
from bitcoincashplus_amd.testing.messages import CTransaction, from_hex
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import OP_CHECKSEQUENCEVERIFY, OP_DROP, CScript

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

BASE_RLT = 10
SEQ_DISABLE_FLAG = 1 << 31
SEQ_RANDOM_HIGH_BIT = 1 << 25
SEQ_TYPE_FLAG = 1 << 22
SEQ_RANDOM_LOW_BIT = 1 << 18


def rlt(b31, b25, b22, b18):
    """relative_locktimes[b31][b25][b22][b18]: 10 with the indicated nSequence bits set."""
    v = BASE_RLT
    if b31:
        v |= SEQ_DISABLE_FLAG
    if b25:
        v |= SEQ_RANDOM_HIGH_BIT
    if b22:
        v |= SEQ_TYPE_FLAG
    if b18:
        v |= SEQ_RANDOM_LOW_BIT
    return v


BITS = [(b31, b25, b22, b18) for b31 in range(2) for b25 in range(2) for b22 in range(2) for b18 in range(2)]


class Csv:
    def __init__(self, node, peer):
        self.n = node
        self.rpc = node.rpc
        self.peer = peer
        self.d = BlockRuleDriver(node.rpc, peer, timeout=120)

    def status(self):
        return self.rpc.getblockchaininfo()["bip9_softforks"]["csv"]["status"]

    # ---- transactions made and signed by the node's wallet
    def create_transaction(self, txid, amount):
        raw = self.rpc.createrawtransaction([{"txid": txid, "vout": 0}], {self.address: amount})
        return from_hex(CTransaction(), raw)

    def sign(self, tx):
        tx.rehash()
        return from_hex(CTransaction(), self.rpc.signrawtransaction(tx.serialize().hex(), None, None,
                                                                    "ALL|FORKID")["hex"])

    def send_generic_input_tx(self, coinbases):
        tx = self.create_transaction(self.rpc.getblock(coinbases.pop())["tx"][0], Decimal("49.99"))
        return self.rpc.sendrawtransaction(self.sign(tx).serialize().hex())

    def bip68txs(self, inputs, version, delta=0):
        out = {}
        for i, bits in enumerate(BITS):
            tx = self.create_transaction(inputs[i], Decimal("49.98"))
            tx.nVersion = version
            tx.vin[0].nSequence = rlt(*bits) + delta
            out[bits] = self.sign(tx)
        return out

    def bip112txs(self, inputs, vary_csv, version, delta=0):
        out = {}
        for i, bits in enumerate(BITS):
            tx = self.create_transaction(inputs[i], Decimal("49.98"))
            tx.vin[0].nSequence = (BASE_RLT if vary_csv else rlt(*bits)) + delta
            tx.nVersion = version
            s = self.sign(tx)
            arg = rlt(*bits) if vary_csv else BASE_RLT
            s.vin[0].scriptSig = bytes(CScript([CScript.num(arg), OP_CHECKSEQUENCEVERIFY, OP_DROP])) + \
                bytes(s.vin[0].scriptSig)
            s.rehash()
            out[bits] = s
        return out

    def bip112special(self, inp, version):
        tx = self.create_transaction(inp, Decimal("49.98"))
        tx.nVersion = version
        s = self.sign(tx)
        s.vin[0].scriptSig = bytes(CScript([CScript.num(-1), OP_CHECKSEQUENCEVERIFY, OP_DROP])) + bytes(s.vin[0].scriptSig)
        s.rehash()
        return s

    # ---- blocks
    def test_block(self, txs, version=536870912):
        b = create_block(self.tip, create_coinbase(self.tipheight + 1), self.last_block_time + 600,
                         self.tipheight + 1, version=version, txs=txs)
        solve(b)
        return b

    def generate_blocks(self, number, version, blocks=None):
        blocks = [] if blocks is None else blocks
        for _ in range(number):
            b = self.test_block([], version)
            blocks.append(b)
            self.last_block_time += 600
            self.tip = b.sha256
            self.tipheight += 1
        return blocks

    def deliver(self, blocks):
        """TestInstance(blocks, sync_every_block=False), all expected valid."""
        for b in blocks:
            self.peer.store.add_block(b)
        self.d.accept(blocks[-1])

    def valid_then_undo(self, txs):
        """TestInstance([[block(txs), True]]) followed by invalidateblock(tip)."""
        b = self.test_block(txs)
        self.d.accept(b)
        self.rpc.invalidateblock(b.hash)
        assert self.rpc.getbestblockhash() == f"{self.tip:064x}"

    def invalid(self, txs):
        """TestInstance([[block(txs), False]])."""
        self.d.reject(self.test_block(txs))


def test_bip68_112_113(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-whitelist=127.0.0.1", "-blockversion=4"])
    n.start()
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    try:
        run(Csv(n, peer))
    finally:
        peer.close()
        n.stop()


OFFSET = 20 * 144  # the reference's heights + OFFSET (see above)


def run(c):
    rpc = c.rpc
    long_past_time = int(time.time()) - 600 * 1000
    rpc.setmocktime(long_past_time - 100)
    hashes = rpc.generate(OFFSET + 143)  # through the fork; tip = the last block of a period
    rpc.setmocktime(0)
    coinbase_blocks = hashes[:1 + 16 + 2 * 32 + 1]  # blocks 1-82 for inputs (50-coin coinbases)
    c.tipheight = OFFSET + 143
    c.last_block_time = long_past_time
    c.tip = int(rpc.getbestblockhash(), 16)
    c.address = rpc.getnewaddress()
    assert rpc.getblockcount() == c.tipheight and c.tipheight >= 3000

    # ---- deployment (the reference's step 1: DEFINED -> STARTED by height 143, here by OFFSET + 143)
    assert c.status() == "started"
    blocks = c.generate_blocks(50, 0x20000001)  # signalling
    c.generate_blocks(20, 4, blocks)  # not
    c.generate_blocks(50, 0x20000101, blocks)  # signalling (another bit too)
    c.generate_blocks(24, 0x20010000, blocks)  # not
    c.deliver(blocks)  # 2
    assert c.status() == "started"  # 100 of 144: height 287 (+ OFFSET)
    blocks = c.generate_blocks(58, 0x20000001)
    c.generate_blocks(26, 4, blocks)
    c.generate_blocks(50, 0x20000101, blocks)
    c.generate_blocks(10, 0x20010000, blocks)
    c.deliver(blocks)  # 3
    assert c.status() == "locked_in"  # 108 of 144: height 431 (+ OFFSET)
    c.deliver(c.generate_blocks(140, 4))  # 4

    # inputs for every test, in the chain at height 572 (+ OFFSET)
    bip68inputs = [c.send_generic_input_tx(coinbase_blocks) for _ in range(16)]
    bip112basicinputs = [[c.send_generic_input_tx(coinbase_blocks) for _ in range(16)] for _ in range(2)]
    bip112diverseinputs = [[c.send_generic_input_tx(coinbase_blocks) for _ in range(16)] for _ in range(2)]
    bip112specialinput = c.send_generic_input_tx(coinbase_blocks)
    bip113input = c.send_generic_input_tx(coinbase_blocks)
    rpc.setmocktime(c.last_block_time + 600)
    inputblockhash = rpc.generate(1)[0]
    rpc.setmocktime(0)
    c.tip = int(inputblockhash, 16)
    c.tipheight += 1
    c.last_block_time += 600
    assert len(rpc.getblock(inputblockhash, True)["tx"]) == 82 + 1

    c.deliver(c.generate_blocks(2, 4))  # 5
    assert c.status() == "locked_in"  # height 574 (+ OFFSET): active from block 576

    bip113tx_v1 = c.create_transaction(bip113input, Decimal("49.98"))
    bip113tx_v1.vin[0].nSequence = 0xFFFFFFFE
    bip113tx_v1.nVersion = 1
    bip113tx_v2 = c.create_transaction(bip113input, Decimal("49.98"))
    bip113tx_v2.vin[0].nSequence = 0xFFFFFFFE
    bip113tx_v2.nVersion = 2
    bip68txs_v1 = c.bip68txs(bip68inputs, 1)
    bip68txs_v2 = c.bip68txs(bip68inputs, 2)
    vary_nseq_v1 = c.bip112txs(bip112basicinputs[0], False, 1)
    vary_nseq_v2 = c.bip112txs(bip112basicinputs[0], False, 2)
    vary_nseq9_v1 = c.bip112txs(bip112basicinputs[1], False, 1, -1)
    vary_nseq9_v2 = c.bip112txs(bip112basicinputs[1], False, 2, -1)
    vary_csv_v1 = c.bip112txs(bip112diverseinputs[0], True, 1)
    vary_csv_v2 = c.bip112txs(bip112diverseinputs[0], True, 2)
    vary_csv9_v1 = c.bip112txs(bip112diverseinputs[1], True, 1, -1)
    vary_csv9_v2 = c.bip112txs(bip112diverseinputs[1], True, 2, -1)
    special_v1 = c.bip112special(bip112specialinput, 1)
    special_v2 = c.bip112special(bip112specialinput, 2)

    def all16(d):
        return [d[b] for b in BITS]

    # ---- before activation: everything is valid (6, 7)
    for tx113, v68, vns, vcsv, vns9, vcsv9, special in (
            (bip113tx_v1, bip68txs_v1, vary_nseq_v1, vary_csv_v1, vary_nseq9_v1, vary_csv9_v1, special_v1),
            (bip113tx_v2, bip68txs_v2, vary_nseq_v2, vary_csv_v2, vary_nseq9_v2, vary_csv9_v2, special_v2)):
        tx113.nLockTime = c.last_block_time - 600 * 5  # = MTP of the prior block, < this block's time
        txs = [c.sign(tx113), special] + all16(v68) + all16(vns) + all16(vcsv) + all16(vns9) + all16(vcsv9)
        c.valid_then_undo(txs)

    c.deliver(c.generate_blocks(1, 4))  # 8
    assert c.status() == "active"  # height 575 (+ OFFSET)

    # ---- BIP113
    signed = []
    for tx in (bip113tx_v1, bip113tx_v2):
        tx.nLockTime = c.last_block_time - 600 * 5  # not below the MTP
        signed.append(c.sign(tx))
    for tx in signed:
        c.invalid([tx])  # 9, 10
    signed = []
    for tx in (bip113tx_v1, bip113tx_v2):
        tx.nLockTime = c.last_block_time - 600 * 5 - 1  # below the MTP
        signed.append(c.sign(tx))
    for tx in signed:
        c.valid_then_undo([tx])  # 11, 12
    c.deliver(c.generate_blocks(4, 1234))  # 13: next height 580

    # ---- BIP68
    c.valid_then_undo(all16(bip68txs_v1))  # 14: version 1 unaffected
    bip68success = [bip68txs_v2[(1, b25, b22, b18)] for b25 in range(2) for b22 in range(2) for b18 in range(2)]
    c.valid_then_undo(bip68success)  # 15: disable flag set
    timetxs = [bip68txs_v2[(0, b25, 1, b18)] for b25 in range(2) for b18 in range(2)]
    for tx in timetxs:
        c.invalid([tx])  # 16-19: 8 * 600 < 10 * 512 s
    heighttxs = [bip68txs_v2[(0, b25, 0, b18)] for b25 in range(2) for b18 in range(2)]
    for tx in heighttxs:
        c.invalid([tx])  # 20-23: 8 < 10 blocks
    c.deliver(c.generate_blocks(1, 1234))  # 24: next height 581
    bip68success += timetxs
    c.valid_then_undo(bip68success)  # 25: 9 * 600 > 10 * 512 s
    for tx in heighttxs:
        c.invalid([tx])  # 26-29
    c.deliver(c.generate_blocks(1, 1234))  # 30: next height 582
    bip68success += heighttxs
    c.valid_then_undo(bip68success)  # 31

    # ---- BIP112, version 1
    c.invalid([special_v1])  # 32: negative CSV argument
    ok = []
    for b25 in range(2):
        for b22 in range(2):
            for b18 in range(2):
                ok += [vary_csv_v1[(1, b25, b22, b18)], vary_csv9_v1[(1, b25, b22, b18)]]
    c.valid_then_undo(ok)  # 33: disable flag in the CSV argument
    fail = all16(vary_nseq_v1) + all16(vary_nseq9_v1)
    for b25 in range(2):
        for b22 in range(2):
            for b18 in range(2):
                fail += [vary_csv_v1[(0, b25, b22, b18)], vary_csv9_v1[(0, b25, b22, b18)]]
    for tx in fail:
        c.invalid([tx])  # 34-81

    # ---- BIP112, version 2
    c.invalid([special_v2])  # 82
    ok = []
    for b25 in range(2):
        for b22 in range(2):
            for b18 in range(2):
                ok += [vary_csv_v2[(1, b25, b22, b18)], vary_csv9_v2[(1, b25, b22, b18)]]
    c.valid_then_undo(ok)  # 83
    fail = all16(vary_nseq9_v2)
    for b25 in range(2):
        for b22 in range(2):
            for b18 in range(2):
                fail.append(vary_csv9_v2[(0, b25, b22, b18)])
    for tx in fail:
        c.invalid([tx])  # 84-107: nSequence 9 against CSV 10
    fail = [vary_nseq_v2[(1, b25, b22, b18)] for b25 in range(2) for b22 in range(2) for b18 in range(2)]
    for tx in fail:
        c.invalid([tx])  # 108-115: disable flag in nSequence
    fail = []
    for b25 in range(2):
        for b18 in range(2):
            fail += [vary_nseq_v2[(0, b25, 1, b18)], vary_csv_v2[(0, b25, 1, b18)]]
    for tx in fail:
        c.invalid([tx])  # 116-123: lock types differ
    ok = []
    for b25 in range(2):
        for b18 in range(2):
            ok += [vary_nseq_v2[(0, b25, 0, b18)], vary_csv_v2[(0, b25, 0, b18)]]
    c.valid_then_undo(ok)  # 124: masking
    time_txs = []
    for b25 in range(2):
        for b18 in range(2):
            tx = vary_csv_v2[(0, b25, 1, b18)]
            tx.vin[0].nSequence = BASE_RLT | SEQ_TYPE_FLAG
            # re-sign the P2PKH part, keep the CSV prefix (rlt(0, b25, 1, b18) OP_CSV OP_DROP)
            prefix = bytes(CScript([CScript.num(rlt(0, b25, 1, b18)), OP_CHECKSEQUENCEVERIFY, OP_DROP]))
            tx.vin[0].scriptSig = b""
            s = c.sign(tx)
            s.vin[0].scriptSig = prefix + bytes(s.vin[0].scriptSig)
            s.rehash()
            time_txs.append(s)
    c.valid_then_undo(time_txs)  # 125: two time-type locks compare
