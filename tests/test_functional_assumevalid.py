"""-assumevalid: script checks are skipped for ancestors of an assumed-valid block once enough
work is built on it.

Parity: reference test/functional/assumevalid.py. A chain past the BCP fork holds a block with
an invalid signature (post-fork script failures invalidate blocks) and a little over two weeks of
blocks on top of it. The node sync cases:

* a node without -assumevalid rejects the bad block and stays on its parent;
* a node with -assumevalid=<a descendant of the bad block> accepts the whole chain;
* a node with the same -assumevalid accepts nothing past the bad block if it only learns
  headers for fewer than two weeks' worth of blocks on top. Then
  GetBlockProofEquivalentTime(best header, block) is below 2 weeks, so scripts are checked.
  (reference src/validation.cpp ConnectBlock fScriptChecks.)

All nodes share the same pre-fork prefix, submitted from one node.
"""
import os

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import CBlockHeader, msg_headers
from bitcoincashplus_amd.testing.p2p import P2PPeer

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

ON_TOP = 2100  # blocks after the bad one: > 2016 x 600 s = two weeks of proof-equivalent time


def start(tmp_path, name, *args):
    n = BcpdProcess(str(tmp_path / name), extra_args=["-gpu=0", "-whitelist=127.0.0.1", *args])
    n.start()
    return n


def copy_prefix(src, dst, height):
    for h in range(1, height + 1):
        dst.rpc.submitblock(src.rpc.getblock(src.rpc.getblockhash(h), 0))
    assert dst.rpc.getblockcount() == height


def deliver(n, blocks, upto=None):
    """Headers (2000 per message) for blocks[:upto], then let the node fetch the blocks."""
    upto = len(blocks) if upto is None else upto
    peer = P2PPeer()
    for b in blocks[:upto]:
        peer.store.add_block(b)
    peer.connect("127.0.0.1", n.p2p_port)
    for i in range(0, upto, 2000):
        peer.send(msg_headers([CBlockHeader(b) for b in blocks[i:i + 2000]]))
        peer.sync_with_ping(timeout=120)
    return peer


def wait_height(n, h, timeout=240):
    import time
    deadline = time.time() + timeout
    while time.time() < deadline:
        if n.rpc.getblockcount() >= h:
            return
        time.sleep(0.2)
    raise AssertionError(f"height {n.rpc.getblockcount()}, expected {h}")


def settle(n, timeout=30):
    """Wait until the node's height stops changing."""
    import time
    last, still = -1, 0
    deadline = time.time() + timeout
    while time.time() < deadline and still < 10:
        h = n.rpc.getblockcount()
        still = still + 1 if h == last else 0
        last = h
        time.sleep(0.2)
    return last


def test_assumevalid(tmp_path):
    a = start(tmp_path, "a")
    try:
        a.rpc.generate(2999)  # up to the block before the fork
        prefix = 2999
        B = FullBlockBuilder(a.rpc)
        blocks = []
        # 101 post-fork blocks: the builder's first coinbase matures
        for i in range(101):
            B.next_block(i + 1)
            B.save_spendable_output()
            blocks.append(B.tip)
        # the bad block: spends that coinbase with a signature that does not verify
        out = B.get_spendable_output()
        tx = B.create_and_sign_tx(out.tx, out.n, out.tx.vout[out.n].nValue - 1000)
        sig = bytearray(tx.vin[0].scriptSig)
        sig[-3] ^= 0x01
        tx.vin[0].scriptSig = bytes(sig)
        tx.rehash()
        B.next_block(500)
        B.update_block(500, [tx])
        bad = len(blocks)
        blocks.append(B.tip)
        for i in range(ON_TOP):
            B.next_block(1000 + i)
            blocks.append(B.tip)
        bad_height = prefix + 1 + bad
        assumed = blocks[bad + 1].hash  # a descendant of the bad block

        # no -assumevalid: stops before the bad block
        p = deliver(a, blocks, upto=bad + 50)
        wait_height(a, bad_height - 1)
        assert settle(a) == bad_height - 1
        tips = {t["hash"]: t["status"] for t in a.rpc.getchaintips()}
        assert tips.get(blocks[bad].hash) == "invalid" or blocks[bad].hash not in tips
        p.close()
    finally:
        a.stop()

    b = start(tmp_path, "b", f"-assumevalid={assumed}")
    c = start(tmp_path, "c", f"-assumevalid={assumed}")
    try:
        # the shared pre-fork prefix, from the first node's block files
        src = BcpdProcess(a.datadir, extra_args=["-gpu=0"], port=a.rpcport)
        src.start()
        try:
            for n in (b, c):
                copy_prefix(src, n, prefix)
        finally:
            src.stop()
        # -assumevalid and two weeks on top: the whole chain is accepted
        pb = deliver(b, blocks)
        wait_height(b, prefix + len(blocks))
        assert b.rpc.getbestblockhash() == blocks[-1].hash
        pb.close()
        # -assumevalid but too little on top: scripts are checked, the bad block is rejected
        pc = deliver(c, blocks, upto=bad + 100)
        wait_height(c, bad_height - 1)
        assert settle(c) == bad_height - 1
        pc.close()
    finally:
        for n in (b, c):
            n.stop()
