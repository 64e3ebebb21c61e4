"""BCP block-size / sigop-scaling conformance over the P2P wire.

Parity: reference test/functional/bcp-p2p-fullblocktest.py:215-427: with
-excessiveblocksize=16 MB, blocks of 1..16 MB and exactly the excessive size are accepted, one
byte more is rejected ('bad-blk-length'); the block sigop limit scales with size (20k per
started MB: 'bad-blk-sigops' one past each step); one transaction may hold at most 20k sigops
('bad-txn-sigops'), P2SH redeem-script sigops included. Runs pre-fork like the reference and
again post-fork (140-byte headers, Equihash(48,5)), where size accounting includes the
solution.
"""
import os
import random

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver, RejectResult
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import (MAX_BLOCK_SIGOPS_PER_MB, MAX_TX_SIGOPS_COUNT, ONE_MEGABYTE, COutPoint,
                                                  CTransaction, CTxIn, CTxOut, ser_compact_size)
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import (OP_2DUP, OP_CHECKSIG, OP_CHECKSIGVERIFY, OP_DROP, OP_TRUE, SIGHASH_ALL,
                                                SIGHASH_FORKID, CScript, p2sh_script, push, signature_hash_forkid)

pytestmark = pytest.mark.functional

EXCESSIVE = 16 * ONE_MEGABYTE

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


@pytest.fixture
def node(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=[
        "-gpu=0", "-whitelist=127.0.0.1", "-norelaypriority", "-limitancestorcount=9999",
        "-limitancestorsize=9999", "-limitdescendantcount=9999", "-limitdescendantsize=9999", "-maxmempool=999",
        f"-excessiveblocksize={EXCESSIVE}"])
    n.start()
    yield n
    n.stop()


class SizedBuilder(FullBlockBuilder):
    """next_block with the reference's block_size / extra_sigops filling (bcp-p2p-fullblocktest
    next_block): the spend tx pays 0 to `rand OP_DROP OP_TRUE` and 1 satoshi to `script`; filler
    transactions chain through output 0 with padding pushes and extra CHECKSIGs."""

    def sized_block(self, number, spend=None, script=None, extra_sigops=0, block_size=0, rng=random.Random(7)):
        prev = self.tip_hash()
        height = self.heights[prev] + 1
        cb = create_coinbase(height, script_pubkey=self.coinbase_script)
        txs = []
        spendable = None
        if spend is not None:
            cb.vout[0].nValue += spend.value - 1
            cb.rehash()
            tx = CTransaction()
            tx.vin.append(CTxIn(COutPoint(spend.tx.calc_sha256(), spend.n), b"", 0xFFFFFFFF))
            tx.vout.append(CTxOut(0, CScript([CScript.num(rng.randint(0, 255)), OP_DROP, OP_TRUE])))
            tx.vout.append(CTxOut(1, script if script is not None else CScript([OP_TRUE])))
            self.sign_tx(tx, spend.tx, spend.n)
            txs.append(tx)
            spendable = (tx, 0)
        block = create_block(prev, cb, self.block_time, height, txs=txs, bcp_height=self.bcp_height)
        self.block_time += 1
        if spendable is not None and block_size > 0:
            size = block.consensus_size()
            while size < block_size:
                script_length = block_size - size - 79
                if script_length > 510000:
                    script_length = 500000
                tx_sigops = min(extra_sigops, script_length, MAX_TX_SIGOPS_COUNT)
                extra_sigops -= tx_sigops
                pad = script_length - tx_sigops
                t = CTransaction()
                t.vout.append(CTxOut(0, CScript([OP_TRUE])))
                t.vout.append(CTxOut(0, CScript([b"\x00" * pad] + [OP_CHECKSIG] * tx_sigops)))
                t.vin.append(CTxIn(COutPoint(spendable[0].calc_sha256(), spendable[1])))
                t.rehash()
                old_count = len(ser_compact_size(len(block.vtx)))
                block.vtx.append(t)
                size += len(t.serialize()) + len(ser_compact_size(len(block.vtx))) - old_count
                spendable = (t, 0)
            assert size == block_size and extra_sigops == 0, (size, block_size, extra_sigops)
        block.hashMerkleRoot = block.calc_merkle_root()
        solve(block, self.equihash)
        assert block_size == 0 or block.consensus_size() == block_size
        self.tip = block
        self.heights[block.sha256] = height
        self.blocks[number] = block
        return block


def run_bcp_suite(n, postfork):
    if postfork:
        n.rpc.generate(2999)
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    d = BlockRuleDriver(n.rpc, peer, timeout=180)
    B = SizedBuilder(n.rpc)
    rej = RejectResult

    B.next_block(0)
    B.save_spendable_output()
    d.accept(B.tip)
    for i in range(99):
        B.next_block(5000 + i)
        B.save_spendable_output()
        d.push(B.tip)
    d.wait_tip(B.tip.sha256)
    out = [B.get_spendable_output() for _ in range(100)]
    block = B.sized_block

    for i in range(16):
        block(i + 1, spend=out[i], block_size=(i + 1) * ONE_MEGABYTE)
        d.accept(B.tip)
    block(17, spend=out[16], block_size=EXCESSIVE)
    d.accept(B.tip)
    block(18, spend=out[17], block_size=EXCESSIVE + 1)
    d.reject(B.tip, rej(16, b"bad-blk-length"))
    B.set_tip(17)

    lots = CScript([OP_CHECKSIG] * (MAX_BLOCK_SIGOPS_PER_MB - 1))
    block(19, spend=out[17], script=lots, block_size=ONE_MEGABYTE)
    d.accept(B.tip)
    block(20, spend=out[18], script=CScript([OP_CHECKSIG] * MAX_BLOCK_SIGOPS_PER_MB), block_size=ONE_MEGABYTE)
    d.reject(B.tip, rej(16, b"bad-blk-sigops"))
    B.set_tip(19)
    block(21, spend=out[18], script=lots, extra_sigops=MAX_BLOCK_SIGOPS_PER_MB, block_size=ONE_MEGABYTE + 1)
    d.accept(B.tip)
    block(22, spend=out[19], script=lots, extra_sigops=MAX_BLOCK_SIGOPS_PER_MB, block_size=2 * ONE_MEGABYTE)
    d.accept(B.tip)
    block(23, spend=out[20], script=lots, extra_sigops=MAX_BLOCK_SIGOPS_PER_MB + 1, block_size=ONE_MEGABYTE + 1)
    d.reject(B.tip, rej(16, b"bad-blk-sigops"))
    B.set_tip(22)
    block(24, spend=out[20], script=lots, extra_sigops=MAX_BLOCK_SIGOPS_PER_MB + 1, block_size=2 * ONE_MEGABYTE)
    d.reject(B.tip, rej(16, b"bad-blk-sigops"))
    B.set_tip(22)
    block(25, spend=out[20], script=lots, extra_sigops=2 * MAX_BLOCK_SIGOPS_PER_MB,
          block_size=2 * ONE_MEGABYTE + 1)
    d.accept(B.tip)
    block(26, spend=out[21], script=lots, extra_sigops=2 * MAX_BLOCK_SIGOPS_PER_MB, block_size=3 * ONE_MEGABYTE)
    d.accept(B.tip)
    block(27, spend=out[22], script=lots, extra_sigops=2 * MAX_BLOCK_SIGOPS_PER_MB + 1,
          block_size=2 * ONE_MEGABYTE + 1)
    d.reject(B.tip, rej(16, b"bad-blk-sigops"))
    B.set_tip(26)
    block(28, spend=out[22], script=lots, extra_sigops=2 * MAX_BLOCK_SIGOPS_PER_MB + 1,
          block_size=3 * ONE_MEGABYTE)
    d.reject(B.tip, rej(16, b"bad-blk-sigops"))
    B.set_tip(26)
    block(29, spend=out[22], script=CScript([OP_CHECKSIG] * (MAX_BLOCK_SIGOPS_PER_MB + 1)),
          block_size=ONE_MEGABYTE + 1)
    d.reject(B.tip, rej(16, b"bad-txn-sigops"))
    B.set_tip(26)

    # P2SH: the redeem script's 6 sigops count against the per-transaction limit
    redeem = CScript([B.key.pubkey] + [OP_2DUP, OP_CHECKSIGVERIFY] * 5 + [OP_CHECKSIG])
    p2sh_tx = B.create_and_sign_tx(out[22].tx, out[22].n, 1, p2sh_script(redeem))
    B.next_block(30)
    B.update_block(30, [p2sh_tx])
    d.accept(B.tip)

    def spend_p2sh(output_script):
        t = CTransaction()
        t.vin.append(CTxIn(COutPoint(p2sh_tx.calc_sha256(), 0), b""))
        t.vout.append(CTxOut(1, output_script))
        h = signature_hash_forkid(redeem, t, 0, SIGHASH_ALL | SIGHASH_FORKID, p2sh_tx.vout[0].nValue)
        t.vin[0].scriptSig = CScript([B.key.sign(h) + bytes([SIGHASH_ALL | SIGHASH_FORKID]), redeem])
        t.rehash()
        return t

    limit = MAX_BLOCK_SIGOPS_PER_MB - redeem.sigop_count(accurate=True)
    block(31, spend=out[23], block_size=ONE_MEGABYTE + 1)
    B.update_block(31, [spend_p2sh(CScript([OP_CHECKSIG] * (limit + 1)))])
    d.reject(B.tip, rej(16, b"bad-txn-sigops"))
    B.set_tip(30)
    block(32, spend=out[23], block_size=ONE_MEGABYTE + 1)
    B.update_block(32, [spend_p2sh(CScript([OP_CHECKSIG] * limit))])
    d.accept(B.tip)
    assert n.rpc.getexcessiveblock()["excessiveBlockSize"] == EXCESSIVE
    peer.close()


@pytest.mark.slow
def test_bcp_fullblock_prefork(node):
    run_bcp_suite(node, postfork=False)


@pytest.mark.slow
def test_bcp_fullblock_postfork(node):
    run_bcp_suite(node, postfork=True)
