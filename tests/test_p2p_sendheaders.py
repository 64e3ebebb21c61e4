"""Headers announcements (before and after sendheaders, after reorgs), direct fetch, and
unconnecting headers.

Parity: reference test/functional/sendheaders.py Parts 1-5, driven as there by an
"inv node" (never sends sendheaders) and a "test node" (sendheaders, nServices 0 so the node
fetches blocks from it only by direct fetch):
* Part 1 (:300-334): before sendheaders every block is announced by inv, whatever the peer
  requests meanwhile (getdata, getheaders + getdata, its own header announcement);
* Part 2 (:336-402): after sendheaders and a getheaders from the tip, new blocks are announced by
  header, also after the peer mined 1..10 blocks of its own and announced them by inv (the node
  answers with getheaders, then getdata) or by headers (getdata); duplicate inv / headers
  announcements from the inv node bring no second getdata;
* Part 3 (:405-476): a reorg of up to 8 new blocks is announced to the test node by headers,
  a longer one by a single inv; headers announcements then stay off through getblocks,
  getdata and a getheaders whose best header is too old, and resume after a getheaders from
  the tip (j = 0) or an inv of the tip (j = 1). The inv node gets an inv for every tip.
* Part 4 (:478-566): direct fetch - headers of blocks the node already has bring no getdata;
  headers of new blocks on the best chain are fetched at once; a fork with less work is not
  fetched, one with equal work is (both blocks), at most 16 blocks in flight per peer
  (MAX_BLOCKS_IN_TRANSIT_PER_PEER), nothing past that.
* Part 5 (:571-643): an unconnecting header brings a getheaders and does not stop sync; the
  node answers each of MAX_UNCONNECTING_HEADERS unconnecting headers with a getheaders, a
  connecting header resets the count, and after 5 * MAX_UNCONNECTING_HEADERS more the peer has
  accumulated 100 misbehaviour points and is disconnected (csrc/net/net_processing.cpp, the
  nUnconnectingHeaders logic).
The node is not whitelisted (a whitelisted peer would not be disconnected).
"""
import os
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.messages import (MSG_BLOCK, CBlockHeader, CInv, msg_block, msg_getblocks,
                                                  msg_getdata, msg_getheaders, msg_headers, msg_inv,
                                                  msg_sendheaders)
from bitcoincashplus_amd.testing.p2p import P2PPeer

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

DIRECT_FETCH_TIMEOUT = 10
MAX_UNCONNECTING_HEADERS = 10


def wait_until(pred, timeout=60, what="condition"):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.02)
    raise AssertionError(f"timed out waiting for {what}")


class AnnouncePeer(P2PPeer):
    """The reference's BaseNode: remembers the last inv / headers announcement, block,
    getdata and getheaders; answers nothing from a block store."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.serve_store = False
        self.reset_announcement()
        self.last_block = None
        self.last_getdata = None
        self.last_getheaders = None
        self.last_announced = None

    def reset_announcement(self):
        with self.cv:
            self.announced = False
            self.last_inv = None
            self.last_headers = None

    def on_inv(self, msg):
        with self.cv:
            self.last_inv = msg
            self.announced = True
            self.last_announced = msg.inv[-1].hash

    def on_headers(self, msg):
        with self.cv:
            self.last_headers = msg
            if msg.headers:
                self.announced = True
                self.last_announced = msg.headers[-1].rehash()

    def on_block(self, msg):
        msg.block.rehash()
        with self.cv:
            self.last_block = msg.block

    def on_getdata(self, msg):
        with self.cv:
            self.last_getdata = msg

    def on_getheaders(self, msg):
        with self.cv:
            self.last_getheaders = msg

    def check_last_announcement(self, headers=(), inv=()):
        """The next block announcement is exactly these headers (hashes) or this inv."""
        self.wait_for(lambda: self.announced, 60, "a block announcement")
        with self.cv:
            got_inv = [x.hash for x in self.last_inv.inv] if self.last_inv is not None else []
            got_hdr = [h.rehash() for h in self.last_headers.headers] if self.last_headers is not None else []
            self.announced = False
            self.last_inv = None
            self.last_headers = None
        return got_inv == list(inv) and got_hdr == list(headers)

    def wait_for_block_announcement(self, h, timeout=60):
        self.wait_for(lambda: self.last_announced == h, timeout, "announcement")

    def wait_for_block(self, h, timeout=60):
        self.wait_for(lambda: self.last_block is not None and self.last_block.sha256 == h, timeout, "block")

    def wait_for_getdata(self, hashes, timeout=60):
        self.wait_for(lambda: self.last_getdata is not None and [x.hash for x in self.last_getdata.inv] == hashes,
                      timeout, "getdata")

    def wait_for_getheaders(self, timeout=60):
        self.wait_for(lambda: self.last_getheaders is not None, timeout, "getheaders")

    def send_header_for_blocks(self, blocks):
        self.send(msg_headers([CBlockHeader(b) for b in blocks]))

    def get_data(self, hashes):
        self.send(msg_getdata([CInv(MSG_BLOCK, h) for h in hashes]))


@pytest.fixture
def net(tmp_path):
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0"])
    b = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpu=0"])
    a.start()
    b.start()
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "add")
    wait_until(lambda: a.rpc.getconnectioncount() == 1, what="b connected")
    inv_node = AnnouncePeer().connect("127.0.0.1", a.p2p_port)
    test_node = AnnouncePeer(services=0).connect("127.0.0.1", a.p2p_port)
    yield a, b, inv_node, test_node
    for p in (inv_node, test_node):
        p.close()
    a.stop()
    b.stop()


def sync(a, b):
    wait_until(lambda: a.rpc.getbestblockhash() == b.rpc.getbestblockhash(), 60, "sync")


def mine_blocks(a, peers, count):
    for p in peers:
        p.reset_announcement()
    a.rpc.generate(count)
    return int(a.rpc.getbestblockhash(), 16)


def mine_reorg(a, b, peers, length):
    """node a mines `length` blocks; node b replaces them with length + 1 of its own."""
    a.rpc.generate(length)
    sync(a, b)
    for p in peers:
        p.wait_for_block_announcement(int(a.rpc.getbestblockhash(), 16))
        p.reset_announcement()
    tip_height = b.rpc.getblockcount()
    b.rpc.invalidateblock(b.rpc.getblockhash(tip_height - (length - 1)))
    hashes = b.rpc.generate(length + 1)
    sync(a, b)
    return [int(x, 16) for x in hashes]


def new_blocks(tip, height, block_time, count):
    out = []
    for _ in range(count):
        blk = create_block(tip, create_coinbase(height), block_time, height)
        solve(blk)
        out.append(blk)
        tip, height, block_time = blk.sha256, height + 1, block_time + 1
    return out


def test_sendheaders_parts_1_to_5(net):
    a, b, inv_node, test_node = net
    peers = [inv_node, test_node]
    a.rpc.generate(101)  # out of initial block download
    sync(a, b)
    tip = int(a.rpc.getbestblockhash(), 16)

    # ---- Part 1: no headers announcements before sendheaders, whatever the peer requests
    for i in range(4):
        old_tip = tip
        tip = mine_blocks(a, peers, 1)
        assert inv_node.check_last_announcement(inv=[tip])
        assert test_node.check_last_announcement(inv=[tip])
        if i == 0:  # request the block
            test_node.get_data([tip])
            test_node.wait_for_block(tip)
        elif i == 1:  # request header and block
            test_node.send(msg_getheaders([old_tip], tip))
            test_node.get_data([tip])
            test_node.wait_for_block(tip)
            test_node.reset_announcement()  # (the headers reply)
        elif i == 2:  # announce a block of our own by header
            height = a.rpc.getblockcount()
            block_time = a.rpc.getblock(a.rpc.getbestblockhash())["time"] + 1
            nb = new_blocks(tip, height + 1, block_time, 1)[0]
            test_node.send_header_for_blocks([nb])
            test_node.wait_for_getdata([nb.sha256], DIRECT_FETCH_TIMEOUT)
            test_node.send(msg_block(nb))
            test_node.sync_with_ping()
            inv_node.reset_announcement()
            test_node.reset_announcement()
    sync(a, b)

    # ---- Part 2: after sendheaders (and a getheaders from the tip), announcements are headers
    test_node.send(msg_sendheaders())
    test_node.send(msg_getheaders([int(a.rpc.getbestblockhash(), 16)], 0))
    test_node.sync_with_ping()
    tip = mine_blocks(a, peers, 1)
    assert inv_node.check_last_announcement(inv=[tip])
    assert test_node.check_last_announcement(headers=[tip])
    height = a.rpc.getblockcount() + 1
    block_time = a.rpc.getblock(a.rpc.getbestblockhash())["time"] + 10
    for i in range(10):
        # the peer mines i + 1 blocks and announces them by inv of the tip or by headers;
        # the node's next block is still announced to it by header
        for j in range(2):
            blocks = new_blocks(tip, height, block_time, i + 1)
            tip, height, block_time = blocks[-1].sha256, height + i + 1, block_time + i + 1
            if j == 0:
                test_node.last_getheaders = None
                test_node.send(msg_inv([CInv(MSG_BLOCK, tip)]))
                test_node.wait_for_getheaders(DIRECT_FETCH_TIMEOUT)
                test_node.send_header_for_blocks(blocks)
                for x in blocks:  # duplicate invs bring no duplicate getdata or announcements
                    inv_node.send(msg_inv([CInv(MSG_BLOCK, x.sha256)]))
                test_node.wait_for_getdata([x.sha256 for x in blocks], DIRECT_FETCH_TIMEOUT)
                inv_node.sync_with_ping()
            else:
                test_node.send_header_for_blocks(blocks)
                test_node.wait_for_getdata([x.sha256 for x in blocks], DIRECT_FETCH_TIMEOUT)
                inv_node.send_header_for_blocks(blocks)  # duplicate headers: no second getdata
                inv_node.sync_with_ping()
            for x in blocks:
                test_node.send(msg_block(x))
            test_node.sync_with_ping()
            inv_node.sync_with_ping()
            # not announced to the inv node, which announced them itself
            assert inv_node.last_inv is None and inv_node.last_headers is None
            tip = mine_blocks(a, peers, 1)
            assert inv_node.check_last_announcement(inv=[tip])
            assert test_node.check_last_announcement(headers=[tip])
            height += 1
            block_time += 1
    sync(a, b)

    # ---- Part 3: headers announcements stop after a large reorg and resume after getheaders/inv
    for j in range(2):
        hashes = mine_reorg(a, b, peers, 7)  # 8 new blocks: announced by headers
        tip = hashes[-1]
        assert inv_node.check_last_announcement(inv=[tip])
        assert test_node.check_last_announcement(headers=hashes)
        hashes = mine_reorg(a, b, peers, 8)  # 9 new blocks: one inv
        tip = hashes[-1]
        assert inv_node.check_last_announcement(inv=[tip])
        assert test_node.check_last_announcement(inv=[tip])
        fork_point = int(a.rpc.getblock(f"{hashes[0]:064x}")["previousblockhash"], 16)
        # getblocks from the fork point: an inv of every new block
        test_node.send(msg_getblocks([fork_point], 0))
        assert test_node.check_last_announcement(inv=hashes)
        test_node.get_data(hashes)
        test_node.wait_for_block(hashes[-1])
        for i in range(3):
            tip = mine_blocks(a, peers, 1)  # still announced by inv
            assert inv_node.check_last_announcement(inv=[tip])
            assert test_node.check_last_announcement(inv=[tip])
            if i == 0:  # getdata alone does not resume headers announcements
                test_node.get_data([tip])
                test_node.wait_for_block(tip)
            elif i == 1:  # a getheaders whose best header is too old does not either
                test_node.send(msg_getheaders([fork_point], hashes[1]))
                test_node.get_data([tip])
                test_node.wait_for_block(tip)
            else:
                test_node.get_data([tip])
                test_node.wait_for_block(tip)
                if j == 0:  # a getheaders from the tip resumes them
                    test_node.send(msg_getheaders([tip], 0))
                    test_node.sync_with_ping()
                else:  # so does an inv of the tip
                    test_node.send(msg_inv([CInv(MSG_BLOCK, tip)]))
                    test_node.sync_with_ping()
        tip = mine_blocks(a, peers, 1)
        assert inv_node.check_last_announcement(inv=[tip])
        assert test_node.check_last_announcement(headers=[tip])

    # ---- Part 4: direct fetch
    tip = mine_blocks(a, peers, 1)
    height = a.rpc.getblockcount() + 1
    block_time = a.rpc.getblock(a.rpc.getbestblockhash())["time"] + 1
    blocks = new_blocks(tip, height, block_time, 2)
    for blk in blocks:  # the node gets the blocks from the inv node first
        inv_node.send(msg_block(blk))
    inv_node.sync_with_ping()
    tip, height, block_time = blocks[-1].sha256, height + 2, block_time + 2
    test_node.last_getdata = None
    test_node.send_header_for_blocks(blocks)
    test_node.sync_with_ping()
    assert test_node.last_getdata is None  # nothing to fetch
    blocks = new_blocks(tip, height, block_time, 3)
    test_node.send_header_for_blocks(blocks)
    test_node.sync_with_ping()
    test_node.wait_for_getdata([x.sha256 for x in blocks], DIRECT_FETCH_TIMEOUT)
    for blk in blocks:
        test_node.send(msg_block(blk))
    test_node.sync_with_ping()
    assert a.rpc.getbestblockhash() == blocks[-1].hash
    block_time += 3
    # a fork off blocks[0]: 20 blocks, announced a few at a time
    tip, height = blocks[0].sha256, height + 1
    blocks = new_blocks(tip, height, block_time, 20)
    test_node.last_getdata = None
    test_node.send_header_for_blocks(blocks[0:1])  # less work than the tip: no fetch
    test_node.sync_with_ping()
    assert test_node.last_getdata is None
    test_node.send_header_for_blocks(blocks[1:2])  # as much work as the tip: both fetched
    test_node.sync_with_ping()
    test_node.wait_for_getdata([x.sha256 for x in blocks[0:2]], DIRECT_FETCH_TIMEOUT)
    test_node.send_header_for_blocks(blocks[2:18])  # 16 more: 14 fetched (16 in flight per peer)
    test_node.sync_with_ping()
    test_node.wait_for_getdata([x.sha256 for x in blocks[2:16]], DIRECT_FETCH_TIMEOUT)
    test_node.last_getdata = None
    test_node.send_header_for_blocks(blocks[18:19])  # one more: nothing (still 16 in flight)
    test_node.sync_with_ping()
    assert test_node.last_getdata is None
    for blk in blocks:
        test_node.send(msg_block(blk))
    test_node.sync_with_ping()
    wait_until(lambda: a.rpc.getbestblockhash() == blocks[-1].hash, 30, "the fork's tip")
    tip = blocks[-1].sha256
    height = a.rpc.getblockcount() + 1
    block_time = blocks[-1].nTime + 1

    # ---- Part 5: unconnecting headers
    for _ in range(10):  # an unconnecting header does not stop sync
        test_node.last_getdata = None
        blocks = new_blocks(tip, height, block_time, 2)
        tip, height, block_time = blocks[-1].sha256, height + 2, block_time + 2
        test_node.last_getheaders = None
        test_node.send_header_for_blocks([blocks[1]])
        test_node.wait_for_getheaders(10)
        test_node.send_header_for_blocks(blocks)
        test_node.wait_for_getdata([x.sha256 for x in blocks])
        for blk in blocks:
            test_node.send(msg_block(blk))
        test_node.sync_with_ping()
        assert int(a.rpc.getbestblockhash(), 16) == blocks[1].sha256
    blocks = new_blocks(tip, height, block_time, MAX_UNCONNECTING_HEADERS + 1)
    for i in range(1, MAX_UNCONNECTING_HEADERS):  # each one answered with a getheaders
        test_node.last_getheaders = None
        test_node.send_header_for_blocks([blocks[i]])
        test_node.wait_for_getheaders(10)
    test_node.send_header_for_blocks([blocks[0]])  # connects: the count starts over
    blocks = blocks[2:]  # (blocks[1] would connect now)
    for i in range(5 * MAX_UNCONNECTING_HEADERS - 1):
        test_node.last_getheaders = None
        test_node.send_header_for_blocks([blocks[i % len(blocks)]])
        test_node.wait_for_getheaders(10)
    test_node.send_header_for_blocks([blocks[-1]])  # the 100th misbehaviour point
    test_node.wait_for_disconnect(30)
    # the inv node never had a block requested from it
    assert inv_node.last_getdata is None
