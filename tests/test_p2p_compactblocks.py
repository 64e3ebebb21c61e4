"""BIP152 compact blocks, headers announcements and legacy-header peers over the P2P wire.

Parity:
* reference test/functional/p2p-compactblocks.py (sendcmpct negotiation, high-bandwidth
  cmpctblock announcements whose SipHash short ids are checked here by an independent
  implementation, getdata(MSG_CMPCT_BLOCK) depth rule, getblocktxn/blocktxn serving, and
  node-side reconstruction: cmpctblock -> getblocktxn for exactly the missing indexes ->
  blocktxn -> new tip; src/blockencodings.cpp:196-230 FillBlock);
* reference test/functional/sendheaders.py (headers announcements after sendheaders,
  inv otherwise);
* the BCP legacy-peer downgrade (reference src/net.h:813-815, src/net_processing.cpp
  1236,2054,2622,2824,3513): a peer below protocol 70016 exchanges 80-byte headers and blocks.
"""
import os

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import (LEGACY_VERSION, MSG_BLOCK, MSG_CMPCT_BLOCK, BlockTransactions,
                                                  BlockTransactionsRequest, CBlockHeader, CInv, HeaderAndShortIDs,
                                                  msg_block, msg_blocktxn, msg_cmpctblock, msg_getblocktxn,
                                                  msg_getdata, msg_getheaders, msg_headers, msg_sendcmpct,
                                                  msg_sendheaders, msg_tx)
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import OP_CHECKSIG, CScript

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


def mature_chain(n, peer, postfork=False):
    """110 blocks paying the test key (P2PK), delivered over P2P; returns the builder and the
    spendable coinbase outputs."""
    if postfork:
        n.rpc.generate(2999)
    d = BlockRuleDriver(n.rpc, peer)
    B = FullBlockBuilder(n.rpc)
    for i in range(110):
        B.next_block(i)
        B.save_spendable_output()
        d.push(B.tip)
    d.wait_tip(B.tip.sha256)
    return B, d, [B.get_spendable_output() for _ in range(10)]


def sync_headers(node, peer):
    """getheaders(locator = tip): the node records that we have its best header, which it
    requires before announcing the next block by header or compact block (reference
    p2p-compactblocks.py request_headers_and_sync)."""
    before = peer.counts.get(b"headers", 0)
    peer.send(msg_getheaders([int(node.rpc.getbestblockhash(), 16)], 0))
    peer.wait_for_message(b"headers", since=before)


def spend_chain(B, out, count):
    """`count` chained P2PK spends (standard, fee 250 sat each: post-fork regtest subsidies are
    4768 sat) starting at one coinbase output."""
    txs = []
    prev, n, value = out.tx, out.n, out.value
    for _ in range(count):
        value -= 250
        tx = B.create_and_sign_tx(prev, n, value, CScript([B.key.pubkey, OP_CHECKSIG]))
        txs.append(tx)
        prev, n = tx, 0
    return txs


def test_sendcmpct_and_announcements(node):
    peer = P2PPeer().connect("127.0.0.1", node.p2p_port)
    B, d, out = mature_chain(node, peer)
    # the node offers low-bandwidth compact blocks (version 1) on connect
    sc = peer.wait_for_message(b"sendcmpct")
    assert sc.version == 1 and sc.announce is False
    # ask for high-bandwidth mode; then a new block arrives as a cmpctblock
    peer.send(msg_sendcmpct(announce=True, version=1))
    peer.sync_with_ping()
    txs = spend_chain(B, out[0], 3)
    for t in txs:
        peer.send(msg_tx(t))
    peer.sync_with_ping()
    assert set(node.rpc.getrawmempool()) == {t.hash for t in txs}
    sync_headers(node, peer)
    before = peer.counts.get(b"cmpctblock", 0)
    best = node.rpc.generate(1)[0]
    m = peer.wait_for_message(b"cmpctblock", since=before)
    hs = m.header_and_shortids
    hs.header.calc_sha256()
    assert hs.header.hash == best
    blk = node.rpc.getblock(best)
    assert [p.index for p in hs.prefilled_txn] == [0]  # the coinbase is always prefilled
    assert hs.prefilled_txn[0].tx.rehash() == blk["tx"][0]
    # short ids: SipHash-2-4 keyed by SHA256(header || nonce), low 48 bits of the txid hash
    want = [hs.short_id(int(h, 16)) for h in blk["tx"][1:]]
    assert hs.shortids == want
    # getdata(MSG_CMPCT_BLOCK) for the tip -> cmpctblock; for a block deeper than 5 -> full block
    before = peer.counts.get(b"cmpctblock", 0)
    peer.send(msg_getdata([CInv(MSG_CMPCT_BLOCK, int(best, 16))]))
    assert peer.wait_for_message(b"cmpctblock", since=before).header_and_shortids.header.rehash() == int(best, 16)
    old = node.rpc.getblockhash(node.rpc.getblockcount() - 7)
    before = peer.counts.get(b"block", 0)
    peer.send(msg_getdata([CInv(MSG_CMPCT_BLOCK, int(old, 16))]))
    assert peer.wait_for_message(b"block", since=before).block.rehash() == int(old, 16)
    # getblocktxn -> blocktxn with exactly the requested transactions
    before = peer.counts.get(b"blocktxn", 0)
    peer.send(msg_getblocktxn(BlockTransactionsRequest(int(best, 16), [1, 3])))
    bt = peer.wait_for_message(b"blocktxn", since=before).block_transactions
    assert bt.blockhash == int(best, 16)
    assert [t.rehash() for t in bt.transactions] == [blk["tx"][1], blk["tx"][3]]
    peer.close()


@pytest.mark.parametrize("postfork", [False, True])
def test_node_reconstructs_compact_block(node, postfork):
    peer = P2PPeer().connect("127.0.0.1", node.p2p_port)
    B, d, out = mature_chain(node, peer, postfork)
    peer.send(msg_sendcmpct(announce=True, version=1))
    # txs 0..4 reach the mempool; txs 5..7 are only in the block
    txs = spend_chain(B, out[0], 8)
    for t in txs[:5]:
        peer.send(msg_tx(t))
    peer.sync_with_ping()
    assert len(node.rpc.getrawmempool()) == 5
    B.next_block("c1")
    blk = B.update_block("c1", txs)
    cmpct = HeaderAndShortIDs()
    cmpct.initialize_from_block(blk, nonce=0x1234ABCD, prefill_list=[0])
    before = peer.counts.get(b"getblocktxn", 0)
    peer.send(msg_cmpctblock(cmpct))
    req = peer.wait_for_message(b"getblocktxn", since=before).block_txn_request
    assert req.blockhash == blk.sha256
    assert req.indexes == [6, 7, 8]  # block positions of the three transactions not in the mempool
    peer.send(msg_blocktxn(BlockTransactions(blk.sha256, [blk.vtx[i] for i in req.indexes])))
    d.wait_tip(blk.sha256)
    assert node.rpc.getrawmempool() == []

    # a compact block whose every transaction is in the mempool connects without a round trip
    txs2 = spend_chain(B, out[1], 4)
    for t in txs2:
        peer.send(msg_tx(t))
    peer.sync_with_ping()
    B.next_block("c2")
    blk2 = B.update_block("c2", txs2)
    cmpct = HeaderAndShortIDs()
    cmpct.initialize_from_block(blk2, nonce=7, prefill_list=[0, 2])
    before = peer.counts.get(b"getblocktxn", 0)
    peer.send(msg_cmpctblock(cmpct))
    d.wait_tip(blk2.sha256)
    peer.sync_with_ping()
    assert peer.counts.get(b"getblocktxn", 0) == before

    # a wrong transaction in blocktxn (not the one committed to) leaves the block unconnected;
    # the node falls back to requesting the full block
    txs3 = spend_chain(B, out[2], 2)
    B.next_block("c3")
    blk3 = B.update_block("c3", txs3)
    cmpct = HeaderAndShortIDs()
    cmpct.initialize_from_block(blk3, nonce=9)
    before_gbt = peer.counts.get(b"getblocktxn", 0)
    peer.send(msg_cmpctblock(cmpct))
    req = peer.wait_for_message(b"getblocktxn", since=before_gbt).block_txn_request
    assert req.indexes == [1, 2]
    peer.serve_store = True
    peer.store.add_block(blk3)
    n_getdata = len(peer.getdata_requests)
    peer.send(msg_blocktxn(BlockTransactions(blk3.sha256, [txs3[1], txs3[0]])))  # swapped
    peer.wait_for(lambda: any(i.hash == blk3.sha256 for i in peer.getdata_requests[n_getdata:]), 30,
                  "getdata for the full block")
    d.wait_tip(blk3.sha256)  # served from the store by the peer
    peer.close()


def test_sendheaders_announcements(node):
    peer = P2PPeer().connect("127.0.0.1", node.p2p_port)
    node.rpc.generate(5)
    peer.sync_with_ping()
    # without sendheaders (and not high-bandwidth compact) new blocks are announced by inv
    before = peer.counts.get(b"inv", 0)
    h = node.rpc.generate(1)[0]
    inv = peer.wait_for_message(b"inv", since=before)
    assert any(i.type == MSG_BLOCK and i.hash == int(h, 16) for i in inv.inv)
    # after a getheaders the node knows our best header; with sendheaders it announces headers
    peer.send(msg_getheaders([int(h, 16)], 0))
    peer.send(msg_sendheaders())
    peer.sync_with_ping()
    before = peer.counts.get(b"headers", 0)
    h2 = node.rpc.generate(1)[0]
    hm = peer.wait_for_message(b"headers", since=before)
    assert [x.rehash() for x in hm.headers] == [int(h2, 16)]
    # our own headers announcement of a block the node lacks makes it ask for the block
    B = FullBlockBuilder(node.rpc)
    B.next_block(1)
    peer.store.add_block(B.tip)
    n_gd = len(peer.getdata_requests)
    peer.send(msg_headers([CBlockHeader(B.tip)]))
    peer.wait_for(lambda: any(i.hash == B.tip.sha256 for i in peer.getdata_requests[n_gd:]), 30, "getdata")
    BlockRuleDriver(node.rpc, peer).wait_tip(B.tip.sha256)
    peer.close()


def test_legacy_peer_gets_80_byte_headers(node):
    """A 70014 peer: the node serves legacy 80-byte headers and blocks and accepts them from it."""
    node.rpc.generate(20)
    peer = P2PPeer(version=LEGACY_VERSION).connect("127.0.0.1", node.p2p_port)
    assert peer.legacy and peer.peer_version.nVersion == 70016
    best = node.rpc.getbestblockhash()
    before = peer.counts.get(b"headers", 0)
    peer.send(msg_getheaders([int(node.rpc.getblockhash(10), 16)], 0))
    hm = peer.wait_for_message(b"headers", since=before)
    assert len(hm.headers) == 10
    # parsed as 80-byte headers, the hashes are the node's (pre-fork hashing is legacy)
    assert hm.headers[-1].rehash() == int(best, 16)
    assert all(h.nHeight == 0 and h.nSolution == b"" for h in hm.headers)
    before = peer.counts.get(b"block", 0)
    peer.send(msg_getdata([CInv(MSG_BLOCK, int(best, 16))]))
    b = peer.wait_for_message(b"block", since=before).block
    assert b.rehash() == int(best, 16) and len(b.vtx) == 1
    # a legacy peer's 80-byte block is accepted (pre-fork)
    B = FullBlockBuilder(node.rpc)
    B.next_block(1)
    peer.send(msg_block(B.tip))
    peer.sync_with_ping()
    assert node.rpc.getbestblockhash() == B.tip.hash
    info = [p for p in node.rpc.getpeerinfo() if p["version"] == LEGACY_VERSION]
    assert len(info) == 1
    peer.close()


def test_legacy_headers_after_fork(node):
    """Post-fork the legacy layout drops nHeight and the solution: a legacy peer receives
    80-byte headers whose legacy hash is not the block hash (reference quirk kept)."""
    node.rpc.generate(3001)
    peer = P2PPeer(version=LEGACY_VERSION).connect("127.0.0.1", node.p2p_port)
    before = peer.counts.get(b"headers", 0)
    peer.send(msg_getheaders([int(node.rpc.getblockhash(2998), 16)], 0))
    hm = peer.wait_for_message(b"headers", since=before)
    assert len(hm.headers) == 3
    assert hm.headers[0].rehash() == int(node.rpc.getblockhash(2999), 16)  # pre-fork: legacy hash
    assert hm.headers[1].rehash() != int(node.rpc.getblockhash(3000), 16)  # post-fork: lost fields
    # the modern peer gets the full 140-byte + solution header with the right hash
    peer2 = P2PPeer().connect("127.0.0.1", node.p2p_port)
    before = peer2.counts.get(b"headers", 0)
    peer2.send(msg_getheaders([int(node.rpc.getblockhash(2998), 16)], 0))
    hm2 = peer2.wait_for_message(b"headers", since=before)
    assert [h.rehash() for h in hm2.headers] == [int(node.rpc.getblockhash(x), 16) for x in (2999, 3000, 3001)]
    assert hm2.headers[1].nHeight == 3000 and len(hm2.headers[1].nSolution) == 36
    peer.close()
    peer2.close()
