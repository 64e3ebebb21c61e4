"""Script failures before and after the BCP fork, over the P2P wire.

Parity: reference src/validation.cpp:2121-2126 — ConnectBlock ignores failed (parallel) script
checks for blocks below the fork height ("Before fork happens from mainnet some block validation
fails even if block is valid. For instance 506396") and rejects them with "blk-bad-inputs" from
the fork on. Both failure paths of the node are driven: a wrong signature (the deferred ECDSA
batch fails) and a signature that does not parse (the script fails on the CPU before any batch).
A block accepted that way really spends its inputs: spending the same coin again is a
missing-input rejection.
"""
import os

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver, RejectResult
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import CScript, push

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


@pytest.fixture
def node(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-whitelist=127.0.0.1"])
    n.start()
    yield n
    n.stop()


def _bad_spends(B, out):
    """Two spends of the coinbase output `out`: one with a corrupted (but DER-valid) signature,
    one whose 'signature' is a bare push of 1 (fails to parse)."""
    value = out.tx.vout[out.n].nValue - 1000
    wrong = B.create_and_sign_tx(out.tx, out.n, value)
    sig = bytearray(wrong.vin[0].scriptSig)
    sig[-3] ^= 0x01  # inside s, before the hash-type byte: still DER, no longer valid
    wrong.vin[0].scriptSig = bytes(sig)
    wrong.rehash()
    garbage = B.create_tx(out.tx, out.n, value - 1)
    garbage.vin[0].scriptSig = bytes(push(b"\x01"))
    garbage.rehash()
    return wrong, garbage


def run(n, postfork: bool):
    if postfork:
        n.rpc.generate(2999)
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    d = BlockRuleDriver(n.rpc, peer)
    B = FullBlockBuilder(n.rpc)
    B.next_block(0)
    B.save_spendable_output()
    d.accept(B.tip)
    for i in range(101):
        B.next_block(1000 + i)
        B.save_spendable_output()
        d.push(B.tip)
    d.wait_tip(B.tip.sha256)
    out = [B.get_spendable_output() for _ in range(2)]
    assert B.tip.is_new_format() == postfork

    wrong, garbage = _bad_spends(B, out[0])
    B.next_block(1)
    B.update_block(1, [wrong])
    if postfork:
        d.reject(B.tip, RejectResult(16, b"blk-bad-inputs"))
        B.set_tip(1100)
    else:
        d.accept(B.tip)
        # the coin is spent by the accepted block: spending it again finds no input
        B.next_block(2)
        B.update_block(2, [garbage])
        d.reject(B.tip, RejectResult(16, b"bad-txns-inputs-missingorspent"))
        B.set_tip(1)

    _, garbage2 = _bad_spends(B, out[1])
    B.next_block(3)
    B.update_block(3, [garbage2])
    if postfork:
        d.reject(B.tip, RejectResult(16, b"blk-bad-inputs"))
    else:
        d.accept(B.tip)
    peer.close()
    return B


def test_prefork_failing_scripts_connect(node):
    B = run(node, postfork=False)
    assert node.rpc.getbestblockhash() == B.tip.hash


def test_postfork_failing_scripts_rejected(node):
    run(node, postfork=True)
