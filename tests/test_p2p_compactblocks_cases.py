"""The remaining BIP152 cases of the reference's p2p-compactblocks.py.

Parity: reference test/functional/p2p-compactblocks.py
* test_invalid_cmpctblock_message (:278-290): a cmpctblock whose prefilled index points past the
  block's transactions is invalid (InitData READ_STATUS_INVALID): the tip does not move and the
  sender is punished (100 points: disconnected);
* test_incorrect_blocktxn_response (:566-627): a blocktxn with the right count but a wrong
  transaction fails reconstruction (merkle mismatch, READ_STATUS_FAILED): no new tip, the node
  asks for the full block instead, and the block is not marked failed (delivering it connects
  it); a blocktxn with the wrong NUMBER of transactions is invalid and punished;
* test_getblocktxn_handler (:629-682): getblocktxn is answered with blocktxn for blocks up to
  MAX_BLOCKTXN_DEPTH = 10 deep, with exactly the requested transactions; deeper, with the full
  block and no blocktxn;
* test_compactblocks_not_at_tip (:684-741): getdata(MSG_CMPCT_BLOCK) returns a cmpctblock for a
  block up to MAX_CMPCTBLOCK_DEPTH = 5 deep and the full block past it; a cmpctblock building on
  a block 5 below the tip is stored as a headers-only tip; a getblocktxn for it is ignored
  (fingerprinting);
* test_invalid_tx_in_compactblock (:764-784): a fully prefilled cmpctblock with a valid header
  and an invalid transaction does not connect and does not get the sender disconnected;
* test_compactblock_reconstruction_multiple_peers (:796-850): a block in flight from a stalling
  peer is reconstructed from the mempool when another peer announces the same cmpctblock; a
  corrupt announcement (here a prefilled coinbase that does not match the merkle root, the
  BCH analogue of the reference's witness corruption) does not break relay, and the stalling
  peer's blocktxn still completes the block.
"""
import os
import random

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.messages import (MSG_BLOCK, MSG_CMPCT_BLOCK, BlockTransactions,
                                                  BlockTransactionsRequest, CBlock, CBlockHeader, CInv,
                                                  HeaderAndShortIDs, PrefilledTransaction, from_hex, msg_blocktxn,
                                                  msg_cmpctblock, msg_getblocktxn, msg_getdata, msg_sendcmpct,
                                                  msg_tx)
from bitcoincashplus_amd.testing.p2p import P2PPeer
from test_p2p_compactblocks import mature_chain, spend_chain, sync_headers

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

MAX_BLOCKTXN_DEPTH = 10
MAX_CMPCTBLOCK_DEPTH = 5


def start(tmp_path, name, whitelist):
    args = ["-gpu=0"] + (["-whitelist=127.0.0.1"] if whitelist else [])
    n = BcpdProcess(str(tmp_path / name), extra_args=args)
    n.start()
    return n


@pytest.fixture
def wl_node(tmp_path):
    n = start(tmp_path, "wl", True)
    yield n
    n.stop()


@pytest.fixture
def plain_node(tmp_path):
    n = start(tmp_path, "plain", False)
    yield n
    n.stop()


def tip(n):
    return int(n.rpc.getbestblockhash(), 16)


def cmpct_of(block, prefill=(0,), nonce=0):
    c = HeaderAndShortIDs()
    c.initialize_from_block(block, nonce=nonce, prefill_list=list(prefill))
    return c


def test_invalid_cmpctblock_message(plain_node):
    n = plain_node
    n.rpc.generate(101)
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    before = tip(n)
    height = n.rpc.getblockcount() + 1
    blk = create_block(before, create_coinbase(height), n.rpc.getblock(n.rpc.getbestblockhash())["time"] + 1, height)
    solve(blk)
    c = HeaderAndShortIDs()
    c.header = CBlockHeader(blk)
    c.prefilled_txn = [PrefilledTransaction(1, blk.vtx[0])]  # index 1: past the block's one transaction
    peer.send(msg_cmpctblock(c))
    peer.wait_for_disconnect(30)  # misbehaving 100
    assert tip(n) == before
    assert n.rpc.listbanned() != [] or n.rpc.getconnectioncount() == 0


def test_incorrect_blocktxn_response(wl_node, plain_node):
    n = wl_node
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    B, d, out = mature_chain(n, peer)
    txs = spend_chain(B, out[0], 10)
    B.next_block("b")
    blk = B.update_block("b", txs)
    for t in blk.vtx[1:6]:  # the first five reach the mempool ahead of the block
        peer.send(msg_tx(t))
    peer.sync_with_ping()
    assert {t.hash for t in blk.vtx[1:6]} <= set(n.rpc.getrawmempool())
    before = peer.counts.get(b"getblocktxn", 0)
    peer.send(msg_cmpctblock(cmpct_of(blk)))
    req = peer.wait_for_message(b"getblocktxn", since=before).block_txn_request
    assert req.indexes == [6, 7, 8, 9, 10]
    # the right number of transactions, one of them wrong
    n_gd = len(peer.getdata_requests)
    peer.send(msg_blocktxn(BlockTransactions(blk.sha256, [blk.vtx[5]] + blk.vtx[7:])))
    peer.sync_with_ping()
    assert tip(n) == blk.hashPrevBlock
    peer.wait_for(lambda: len(peer.getdata_requests) > n_gd, 10, "getdata for the full block")
    gd = peer.getdata_requests[n_gd:]
    assert len(gd) == 1 and gd[0].type == MSG_BLOCK and gd[0].hash == blk.sha256
    # not failed for good: the full block connects (served from the peer's store)
    peer.store.add_block(blk)
    d.push(blk)
    d.wait_tip(blk.sha256)
    peer.close()

    # a blocktxn with the wrong number of transactions is invalid: 100 points
    m = plain_node
    m.rpc.generate(101)
    mpeer = P2PPeer().connect("127.0.0.1", m.p2p_port)
    from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
    from bitcoincashplus_amd.testing.comparison import BlockRuleDriver
    MB = FullBlockBuilder(m.rpc)
    md = BlockRuleDriver(m.rpc, mpeer)
    for i in range(101):
        MB.next_block(i)
        MB.save_spendable_output()
        md.accept(MB.tip)  # announced and fetched (unsolicited blocks are the whitelist's)
    mtxs = spend_chain(MB, MB.get_spendable_output(), 4)
    MB.next_block("m")
    mblk = MB.update_block("m", mtxs)
    before = mpeer.counts.get(b"getblocktxn", 0)
    mpeer.send(msg_cmpctblock(cmpct_of(mblk)))
    req = mpeer.wait_for_message(b"getblocktxn", since=before).block_txn_request
    assert req.indexes == [1, 2, 3, 4]
    mpeer.send(msg_blocktxn(BlockTransactions(mblk.sha256, mblk.vtx[1:3])))  # two of four
    mpeer.wait_for_disconnect(30)
    assert tip(m) == mblk.hashPrevBlock


def test_getblocktxn_handler(wl_node):
    n = wl_node
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    B, d, out = mature_chain(n, peer)
    for k in range(MAX_BLOCKTXN_DEPTH + 3):  # blocks with a few transactions each
        B.next_block(f"t{k}")
        B.update_block(f"t{k}", spend_chain(B, out[k % len(out)], 3) if k < len(out) else [])
        d.push(B.tip)
    d.wait_tip(B.tip.sha256)
    rng = random.Random(5)
    chain_height = n.rpc.getblockcount()
    height = chain_height
    while height >= chain_height - MAX_BLOCKTXN_DEPTH:
        bh = n.rpc.getblockhash(height)
        block = from_hex(CBlock(), n.rpc.getblock(bh, False))
        want = sorted(rng.sample(range(len(block.vtx)), rng.randint(1, len(block.vtx))))
        before = peer.counts.get(b"blocktxn", 0)
        peer.send(msg_getblocktxn(BlockTransactionsRequest(int(bh, 16), want)))
        bt = peer.wait_for_message(b"blocktxn", since=before).block_transactions
        assert bt.blockhash == int(bh, 16)
        assert [t.rehash() for t in bt.transactions] == [block.vtx[i].rehash() for i in want]
        height -= 1
    # one deeper: the full block, no blocktxn
    bh = n.rpc.getblockhash(height)
    before_b, before_t = peer.counts.get(b"block", 0), peer.counts.get(b"blocktxn", 0)
    peer.send(msg_getblocktxn(BlockTransactionsRequest(int(bh, 16), [0])))
    assert peer.wait_for_message(b"block", since=before_b).block.rehash() == int(bh, 16)
    peer.sync_with_ping()
    assert peer.counts.get(b"blocktxn", 0) == before_t
    peer.close()


def test_compactblocks_not_at_tip(wl_node):
    n = wl_node
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    n.rpc.generate(101)
    sync_headers(n, peer)
    peer.send(msg_sendcmpct(announce=True, version=1))
    peer.sync_with_ping()
    new_blocks = []
    for _ in range(MAX_CMPCTBLOCK_DEPTH + 1):
        before = peer.counts.get(b"cmpctblock", 0)
        new_blocks.append(n.rpc.generate(1)[0])
        peer.wait_for_message(b"cmpctblock", since=before)
    # MAX_CMPCTBLOCK_DEPTH deep: still a cmpctblock
    before = peer.counts.get(b"cmpctblock", 0)
    peer.send(msg_getdata([CInv(MSG_CMPCT_BLOCK, int(new_blocks[0], 16))]))
    m = peer.wait_for_message(b"cmpctblock", since=before)
    assert m.header_and_shortids.header.rehash() == int(new_blocks[0], 16)
    # one more block: the full block instead
    before = peer.counts.get(b"cmpctblock", 0)
    n.rpc.generate(1)
    peer.wait_for_message(b"cmpctblock", since=before)
    before_b = peer.counts.get(b"block", 0)
    peer.send(msg_getdata([CInv(MSG_CMPCT_BLOCK, int(new_blocks[0], 16))]))
    assert peer.wait_for_message(b"block", since=before_b).block.rehash() == int(new_blocks[0], 16)
    # an old compact block (parent 5 below the tip) is kept as a headers-only tip
    cur = n.rpc.getblockcount()
    parent = n.rpc.getblockhash(cur - 5)
    ph = n.rpc.getblockheader(parent)
    old = create_block(int(parent, 16), create_coinbase(ph["height"] + 1), ph["time"] + 1, ph["height"] + 1)
    solve(old)
    peer.send(msg_cmpctblock(cmpct_of(old)))
    peer.sync_with_ping()
    tips = {t["hash"]: t for t in n.rpc.getchaintips()}
    assert old.hash in tips and tips[old.hash]["status"] == "headers-only"
    # and a getblocktxn for it is silently ignored
    before_t = peer.counts.get(b"blocktxn", 0)
    peer.send(msg_getblocktxn(BlockTransactionsRequest(old.sha256, [0])))
    peer.sync_with_ping()
    assert peer.counts.get(b"blocktxn", 0) == before_t
    peer.close()


def test_invalid_tx_in_compactblock(plain_node):
    n = plain_node
    n.rpc.generate(101)
    peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
    from bitcoincashplus_amd.testing.comparison import BlockRuleDriver
    from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
    B = FullBlockBuilder(n.rpc)
    d = BlockRuleDriver(n.rpc, peer)
    for i in range(101):
        B.next_block(i)
        B.save_spendable_output()
        d.accept(B.tip)
    txs = spend_chain(B, B.get_spendable_output(), 5)
    B.next_block("bad")
    blk = B.update_block("bad", txs)  # coinbase + 5 chained spends
    del blk.vtx[3]  # tx 4 now spends an output that does not exist
    blk.hashMerkleRoot = blk.calc_merkle_root()
    B.resolve(blk)
    before = tip(n)
    peer.send(msg_cmpctblock(cmpct_of(blk, prefill=range(len(blk.vtx)))))
    peer.sync_with_ping()
    assert tip(n) == before and tip(n) != blk.sha256
    peer.sync_with_ping()  # still connected
    assert n.rpc.getconnectioncount() == 1


def test_compactblock_reconstruction_multiple_peers(wl_node):
    n = wl_node
    stalling = P2PPeer().connect("127.0.0.1", n.p2p_port)
    delivery = P2PPeer().connect("127.0.0.1", n.p2p_port)
    B, d, out = mature_chain(n, stalling)

    def announce(k):
        txs = spend_chain(B, out[k], 5)
        B.next_block(f"mp{k}")
        blk = B.update_block(f"mp{k}", txs)
        c = cmpct_of(blk)
        before = stalling.counts.get(b"getblocktxn", 0)
        stalling.send(msg_cmpctblock(c))
        stalling.wait_for_message(b"getblocktxn", since=before)  # in flight from the stalling peer
        return blk, c

    blk, c = announce(0)
    for t in blk.vtx[1:]:
        delivery.send(msg_tx(t))
    delivery.sync_with_ping()
    assert {t.hash for t in blk.vtx[1:]} <= set(n.rpc.getrawmempool())
    delivery.send(msg_cmpctblock(c))  # reconstructed from the mempool
    delivery.sync_with_ping()
    assert tip(n) == blk.sha256

    # a corrupt announcement from the delivery peer does not break relay
    blk, c = announce(1)
    for t in blk.vtx[1:]:
        delivery.send(msg_tx(t))
    delivery.sync_with_ping()
    bad_cb = from_hex(type(blk.vtx[0])(), blk.vtx[0].serialize().hex())
    bad_cb.vout[0].nValue -= 1
    bad_cb.rehash()
    c.prefilled_txn[0] = PrefilledTransaction(0, bad_cb)
    delivery.send(msg_cmpctblock(c))
    delivery.sync_with_ping()
    assert tip(n) != blk.sha256
    stalling.send(msg_blocktxn(BlockTransactions(blk.sha256, blk.vtx[1:])))
    stalling.sync_with_ping()
    d.wait_tip(blk.sha256)
    stalling.close()
    delivery.close()
