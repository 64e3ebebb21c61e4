"""Cross-block connect pipeline: block N+1's UTXO pass overlaps block N's signature batch
(`-connectpipeline`, csrc/node/validation.cpp ConnectTipsPipelined). A batch of blocks that arrives
out of order connects in one step; a block whose signatures fail - found only when its batch
verdict comes back, after the next block was already prepared on top of it - must leave the
node exactly where one-at-a-time connection would: tip on its parent, the block invalid, the
blocks after it not connected, and a reorg onto a branch that turns out invalid rolled back.

Parity: reference src/validation.cpp:2698-2746 (ActivateBestChainStep connects one block at a
time; the end state for any failure is the same).
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


@pytest.fixture(params=["pipelined", "one-by-one"])
def node(request, tmp_path):
    depth = "3" if request.param == "pipelined" else "1"
    n = BcpdProcess(str(tmp_path / "n"),
                    extra_args=["-gpu=0", "-whitelist=127.0.0.1", f"-connectpipeline={depth}", "-debug=bench"])
    n.pipelined = request.param == "pipelined"
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


def pipeline_runs(n):
    log = open(os.path.join(n.datadir, "regtest", "debug.log"), errors="replace").read()
    return log.count("ConnectTipsPipelined: ")


def deliver_out_of_order(d, blocks):
    """Headers first, then the blocks last-to-first: nothing connects until the first block
    arrives, and then the whole run connects in one step."""
    d.headers([CBlockHeader(b) for b in blocks])
    for b in reversed(blocks[1:]):
        d.push(b)
    d.push(blocks[0])


def test_pipelined_run_with_a_bad_block_in_the_middle(node):
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
    assert pipeline_runs(node) == (1 if node.pipelined else 0)
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
