"""Invalid blocks and transactions delivered over P2P: exact reject messages, no poisoning.

Parity: reference test/functional/invalidblockrequest.py (a mutated block with a duplicated
transaction is rejected 'bad-txns-duplicate' without marking its hash invalid, so the honest
block with the same hash is then accepted; a coinbase paying too much is rejected
'bad-cb-amount'), invalidtxrequest.py (a transaction with an invalid scriptSig is rejected
'mandatory-script-verify-flag-failed'), plus the orphan pool path (a child arriving before its parent waits,
then both enter the mempool) and mempool conflicts (refused with an internal code, so no
reject message).
"""
import copy
import os

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver, RejectResult
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import CBlock, msg_tx
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import OP_CHECKSIG, OP_TRUE, CScript

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


@pytest.fixture(params=[False, True], ids=["prefork", "postfork"])
def setup(request, tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-whitelist=127.0.0.1"])
    n.start()
    if request.param:
        n.rpc.generate(2999)
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    d = BlockRuleDriver(n.rpc, peer)
    B = FullBlockBuilder(n.rpc)
    for i in range(101):
        B.next_block(i)
        B.save_spendable_output()
        d.push(B.tip)
    d.wait_tip(B.tip.sha256)
    yield n, peer, d, B
    peer.close()
    n.stop()


def test_invalid_block_requests(setup):
    n, peer, d, B = setup
    out = B.get_spendable_output()
    # a block whose last transaction is repeated: same merkle root, same hash, invalid
    B.next_block("good", spend=out)
    tx = B.create_tx(B.tip.vtx[1], 0, 0, CScript([OP_TRUE]))
    good = B.update_block("good", [tx])
    assert len(good.vtx) == 3
    bad = CBlock(good, bcp_height=B.bcp_height)
    bad.vtx = list(good.vtx) + [good.vtx[2]]
    assert bad.calc_merkle_root() == good.hashMerkleRoot and bad.calc_sha256() == good.sha256
    d.reject(bad, RejectResult(16, b"bad-txns-duplicate"))
    # the hash is not marked invalid: the honest block with that hash is accepted
    d.accept(good)
    # a coinbase claiming one satoshi more than subsidy + fees
    B.next_block("rich", additional_coinbase_value=1)
    d.reject(B.tip, RejectResult(16, b"bad-cb-amount"))
    assert n.rpc.getbestblockhash() == good.hash
    assert len(n.rpc.getpeerinfo()) == 1  # whitelisted: not disconnected


def test_invalid_tx_requests(setup):
    n, peer, d, B = setup
    out = B.get_spendable_output()
    # reference invalidtxrequest.py: scriptSig OP_NOTIF (0x64) on a P2PK coinbase output
    tx = B.create_tx(out.tx, out.n, out.value - 1000, CScript([B.key.pubkey, OP_CHECKSIG]))
    tx.vin[0].scriptSig = b"\x64"
    tx.rehash()
    peer.send(msg_tx(tx))
    peer.sync_with_ping()
    r = peer.reject_for(tx.calc_sha256())
    assert r is not None and r.message == b"tx" and r.code == 16
    assert r.reason.startswith(b"mandatory-script-verify-flag-failed"), r
    assert n.rpc.getrawmempool() == []
    # a transaction creating value pays a negative fee: with -limitfreerelay=0 (the default) it is
    # refused as a free transaction before its inputs are checked (reference ATMP order)
    tx = B.create_and_sign_tx(out.tx, out.n, out.value + 1, CScript([B.key.pubkey, OP_CHECKSIG]))
    peer.send(msg_tx(tx))
    peer.sync_with_ping()
    r = peer.reject_for(tx.calc_sha256())
    # (post-fork regtest coins are tiny, so the priority check refuses it first: same code)
    assert r is not None and r.code == 66, r
    assert r.reason in (b"rate limited free transaction", b"insufficient priority"), r
    # a bad signature
    tx = B.create_and_sign_tx(out.tx, out.n, out.value - 500, CScript([B.key.pubkey, OP_CHECKSIG]))
    sig = bytearray(tx.vin[0].scriptSig)
    sig[10] ^= 1
    tx.vin[0].scriptSig = bytes(sig)
    tx.rehash()
    peer.send(msg_tx(tx))
    peer.sync_with_ping()
    r = peer.reject_for(tx.calc_sha256())
    assert r is not None and r.code == 16 and b"script-verify-flag-failed" in r.reason, r
    # orphan: the child first (no reject, not in the mempool), then the parent: both accepted
    parent = B.create_and_sign_tx(out.tx, out.n, out.value - 500, CScript([B.key.pubkey, OP_CHECKSIG]))
    child = B.create_and_sign_tx(parent, 0, parent.vout[0].nValue - 500, CScript([B.key.pubkey, OP_CHECKSIG]))
    peer.send(msg_tx(child))
    peer.sync_with_ping()
    assert n.rpc.getrawmempool() == [] and peer.reject_for(child.calc_sha256()) is None
    peer.send(msg_tx(parent))
    peer.sync_with_ping()
    d.peer.wait_for(lambda: len(n.rpc.getrawmempool()) == 2, 30, "orphan resolution")
    assert set(n.rpc.getrawmempool()) == {parent.hash, child.hash}
    # a conflicting spend of the parent's input
    dbl = B.create_and_sign_tx(out.tx, out.n, out.value - 900, CScript([B.key.pubkey, OP_CHECKSIG]))
    peer.send(msg_tx(dbl))
    peer.sync_with_ping()
    # refused, but REJECT_CONFLICT (0x102) is an internal code: no reject message goes out
    assert peer.reject_for(dbl.calc_sha256()) is None
    assert dbl.hash not in n.rpc.getrawmempool()
    # the same transaction again: already in the mempool
    peer.send(msg_tx(parent))
    peer.sync_with_ping()
    assert set(n.rpc.getrawmempool()) == {parent.hash, child.hash}
