"""A block whose signatures fail after its UTXO pass updated the coins tip in place
(`-connectinplace`, csrc/node/validation.cpp ConnectBlock: the tip is taken back from the undo
records) must leave the node exactly where the merged-view connect (`-connectinplace=0`, the
reference's per-block view) leaves it: tip on its parent, the block invalid, the blocks after it
not connected, the coins of the good blocks in and nothing of the bad one, and a reorg onto a
branch that turns out invalid rolled back. Every block takes the parallel UTXO pass
(`-parallelutxo=1`); the batch of blocks arrives out of order and connects in one
ActivateBestChain.

Parity: reference src/validation.cpp:2698-2746 (ActivateBestChainStep connects one block at a
time; the end state for any failure is the same) and :2121-2126 (script failures reject blocks
after the fork).
"""
import os

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import CBlockHeader
from bitcoincashplus_amd.testing.p2p import P2PPeer

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


@pytest.fixture(params=["in-place", "merged-view"])
def node(request, tmp_path):
    inplace = "1" if request.param == "in-place" else "0"
    n = BcpdProcess(str(tmp_path / "n"),
                    extra_args=["-gpu=0", "-whitelist=127.0.0.1", f"-connectinplace={inplace}", "-parallelutxo=1",
                                "-debug=bench"])
    n.inplace = request.param == "in-place"
    n.start()
    yield n
    n.stop()


def setup_chain(n):
    n.rpc.generate(2999)  # post-fork blocks from the builder on: NULLFAIL, deferred ECDSA
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    d = BlockRuleDriver(n.rpc, peer)
    B = FullBlockBuilder(n.rpc)
    B.next_block(0)
    B.save_spendable_output()
    d.accept(B.tip)
    for i in range(110):
        B.next_block(1000 + i)
        B.save_spendable_output()
        d.push(B.tip)
    d.wait_tip(B.tip.sha256)
    return peer, d, B


def bad_sig_spend(B, out):
    tx = B.create_and_sign_tx(out.tx, out.n, out.tx.vout[out.n].nValue - 1000)
    sig = bytearray(tx.vin[0].scriptSig)
    sig[-3] ^= 0x01  # DER-valid, wrong signature: fails only in the batch
    tx.vin[0].scriptSig = bytes(sig)
    tx.rehash()
    return tx


def parallel_passes(n):
    log = open(os.path.join(n.datadir, "regtest", "debug.log"), errors="replace").read()
    return log.count("(parallel UTXO pass)")


def deliver_out_of_order(d, blocks):
    """Headers first, then the blocks last-to-first: nothing connects until the first block
    arrives, and then the whole run connects in one step."""
    d.headers([CBlockHeader(b) for b in blocks])
    for b in reversed(blocks[1:]):
        d.push(b)
    d.push(blocks[0])


def test_batch_with_a_bad_block_in_the_middle(node):
    peer, d, B = setup_chain(node)
    base = B.tip
    outs = [B.get_spendable_output() for _ in range(6)]
    blocks = []
    for i in range(6):
        B.next_block(i + 1, spend=outs[i])
        if i == 3:  # the fourth block also spends a coin with a bad signature
            B.update_block(i + 1, [bad_sig_spend(B, outs[5])])
        blocks.append(B.tip)
    deliver_out_of_order(d, blocks)
    d.wait_tip(blocks[2].sha256)
    assert node.rpc.getblockcount() == node.rpc.getblock(f"{base.sha256:064x}")["height"] + 3
    tips = {t["hash"]: t["status"] for t in node.rpc.getchaintips()}
    assert tips.get(blocks[-1].hash) == "invalid"
    # the chain state is consistent: the good blocks' spends are in, nothing of the bad run is
    assert node.rpc.gettxout(f"{blocks[0].vtx[1].sha256:064x}", 0) is not None
    assert node.rpc.gettxout(f"{blocks[4].vtx[1].sha256:064x}", 0) is None
    assert parallel_passes(node) > 0  # the blocks took the pass that updates the tip in place
    # and the node goes on: a valid sibling of the bad block connects
    B.set_tip(3)
    B.next_block(40, spend=outs[3])
    d.accept(B.tip)
    peer.close()


def test_reorg_onto_a_branch_that_fails_rolls_back(node):
    peer, d, B = setup_chain(node)
    outs = [B.get_spendable_output() for _ in range(6)]
    fork = B.tip
    # current chain: 2 blocks
    B.next_block(1, spend=outs[0])
    d.accept(B.tip)
    B.next_block(2, spend=outs[1])
    d.accept(B.tip)
    old_tip = B.tip
    # competing branch from the fork point: 4 blocks, the third with a bad signature
    B.tip = fork
    branch = []
    for i in range(4):
        B.next_block(10 + i, spend=outs[2 + i])
        if i == 2:
            B.update_block(10 + i, [bad_sig_spend(B, outs[0])])
        branch.append(B.tip)
    deliver_out_of_order(d, branch)
    # the branch's first two blocks connected, the third failed: its work is below the old tip,
    # so the node reorganises back
    d.wait_tip(old_tip.sha256)
    tips = {t["hash"]: t["status"] for t in node.rpc.getchaintips()}
    assert tips.get(branch[-1].hash) == "invalid"
    assert node.rpc.gettxout(f"{old_tip.vtx[1].sha256:064x}", 0) is not None
    peer.close()
