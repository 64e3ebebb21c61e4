"""Reference P2P and soft-fork scenarios that had no counterpart, over the wire to a regtest bcpd.

Parity (reference test/functional/):
* p2p-acceptblock.py: unrequested blocks. A block that forks the tip without more work is
  stored only as a header when it comes from an ordinary peer, and processed when it comes from
  a whitelisted one; a more-work block on top of an unknown parent waits; a block more than
  288 blocks ahead of the tip is not stored from an ordinary peer; an inv for a block whose
  parent the node never processed makes it ask for that parent.
* p2p-leaktests.py: before the version handshake completes the node sends nothing but
  version/verack; a peer that sends messages before its version is disconnected, and one that
  sends a version but never a verack is not sent ping/getaddr/inv traffic.
* nulldummy.py: a CHECKMULTISIG spend with a non-empty dummy element is refused by the mempool
  with the reference's exact message, and is still valid inside a block before the fork.
* bip65-cltv-p2p.py, bipdersig-p2p.py: the reference chain activates BIP66 and BIP65 by
  height (regtest 1251 and 1351, src/chainparams.cpp:341-342; the supermajority versions of
  these scripts predate that): from those heights, blocks of version < 3 / < 4 are rejected
  with "bad-version(0x...)", and a non-DER signature / a failing CHECKLOCKTIMEVERIFY in a
  block's transaction is rejected; one block earlier both are still valid.
* mempool_spendcoinbase.py: a coinbase spend that matures with the next block is accepted into
  the mempool, one that matures a block later is refused (bad-txns-premature-spend-of-coinbase).
* forknotify.py: more than 50 of the last 100 blocks with a version this node would not mine
  raise "Unknown block versions being mined" through -alertnotify, once.
* maxblocksinflight.py: invs for 8, 16, 128 and 1024 unknown blocks from one (whitelisted) peer
  never draw more than 128 block requests in total, and no block is requested twice.
* p2p-versionbits-warning.py: a period with fewer than threshold blocks signalling an unknown
  versionbit raises nothing; a period at the threshold shows the unknown-version warning in
  getinfo/getmininginfo/getnetworkinfo; after a restart the bit is ACTIVE and the node warns
  "unknown new rules activated (versionbit 27)" and runs -alertnotify.
"""
import os
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess, RPCError
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.messages import (MSG_BLOCK, CBlockHeader, CInv, CTransaction, from_hex, msg_block,
                                                  msg_getaddr, msg_headers, msg_inv, msg_ping, msg_verack)
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import (OP_1NEGATE, OP_CHECKLOCKTIMEVERIFY, OP_DROP, CScript)

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def wait_until(pred, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.05)
    raise AssertionError("timeout")


def node(tmp_path, name, *args):
    n = BcpdProcess(str(tmp_path / name), extra_args=["-gpu=0", *args])
    n.start()
    return n


def tip_block(n):
    h = n.rpc.getbestblockhash()
    hdr = n.rpc.getblockheader(h)
    return int(h, 16), hdr["height"], hdr["time"]


def new_block(prev, height, ntime, txs=(), version=4):
    b = create_block(prev, create_coinbase(height), ntime, height, version=version, txs=txs)
    return solve(b)


def block_status(n, h):
    for t in n.rpc.getchaintips():
        if t["hash"] == "%064x" % h:
            return t["status"]
    return None


def test_acceptblock(tmp_path):
    n0 = node(tmp_path, "n0")                          # ordinary peer
    n1 = node(tmp_path, "n1", "-whitelist=127.0.0.1")  # whitelisted peer
    try:
        for n in (n0, n1):
            n.rpc.generate(1)  # leave IBD
        peers = [P2PPeer().connect("127.0.0.1", n.p2p_port) for n in (n0, n1)]
        tips = [tip_block(n) for n in (n0, n1)]
        # 2. a block on each tip is processed
        h2 = [new_block(t[0], 2, t[2] + 1) for t in tips]
        for p, b in zip(peers, h2):
            p.send(msg_block(b))
        for p in peers:
            p.sync_with_ping()
        assert n0.rpc.getblockcount() == 2 and n1.rpc.getblockcount() == 2
        # 3. a fork of the same height: headers only from the ordinary peer, processed from the
        #    whitelisted one (which keeps its first tip at equal work)
        h2f = [new_block(t[0], 2, b.nTime + 1) for t, b in zip(tips, h2)]
        for p, b in zip(peers, h2f):
            p.send(msg_block(b))
        for p in peers:
            p.sync_with_ping()
        assert block_status(n0, h2f[0].sha256) == "headers-only"
        assert block_status(n1, h2f[1].sha256) == "valid-headers"
        # 4. a more-work block on the fork: processed by both; n1 reorgs, n0 cannot (it never
        #    processed the fork's first block)
        h3 = [new_block(b.sha256, 3, b.nTime + 1) for b in h2f]
        for p, b in zip(peers, h3):
            p.send(msg_block(b))
        for p in peers:
            p.sync_with_ping()
        assert n0.rpc.getblockcount() == 2
        assert block_status(n0, h3[0].sha256) == "headers-only"
        assert n1.rpc.getblockcount() == 3
        # 4b. 288 more blocks on the longer chain to n0: all but the last one (more than 288
        #     blocks ahead of its tip) are stored
        chain = [h3[0]]
        for i in range(288):
            prev = chain[-1]
            chain.append(new_block(prev.sha256, 4 + i, prev.nTime + 1))
        for b in chain[1:]:
            peers[0].send(msg_block(b))
        peers[0].sync_with_ping()
        for b in chain[1:-1]:
            n0.rpc.getblock("%064x" % b.sha256)
        with pytest.raises(RPCError) as e:
            n0.rpc.getblock("%064x" % chain[-1].sha256)
        assert "not found on disk" in str(e.value).lower() or e.value.code in (-1, -5)
        # the whitelisted peer's far-ahead block is accepted once its headers are known
        chain1 = [h3[1]]
        for i in range(288):
            prev = chain1[-1]
            chain1.append(new_block(prev.sha256, 4 + i, prev.nTime + 1))
        peers[1].send(msg_headers([CBlockHeader(b) for b in chain1[1:]]))
        peers[1].send(msg_block(chain1[-1]))
        peers[1].sync_with_ping()
        n1.rpc.getblock("%064x" % chain1[-1].sha256)
        # 5. the unrequested fork block again: still not processed by n0
        peers[0].send(msg_block(h2f[0]))
        peers[0].sync_with_ping()
        assert n0.rpc.getblockcount() == 2
        # 6. an inv for the block above the missing one makes n0 ask for the missing parent
        peers[0].clear()
        peers[0].send(msg_inv([CInv(MSG_BLOCK, h3[0].sha256)]))
        peers[0].sync_with_ping()
        wait_until(lambda: any(inv.hash == h2f[0].sha256 for inv in peers[0].getdata_requests), 30)
        # 7. delivering it now extends n0 to the long chain
        peers[0].send(msg_block(h2f[0]))
        peers[0].sync_with_ping()
        wait_until(lambda: n0.rpc.getblockcount() == 290, 60)
        for p in peers:
            p.close()
    finally:
        n0.stop()
        n1.stop()


class LazyPeer(P2PPeer):
    """Never completes the handshake (no verack) and records every message other than
    version/verack/reject the node sends (reference CLazyNode)."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.unexpected = []

    def _dispatch(self, cmd, payload):
        if cmd not in (b"version", b"verack", b"reject"):
            self.unexpected.append(cmd)
        return super()._dispatch(cmd, payload)

    def on_version(self, msg):
        pass  # no verack, no version of our own


def test_p2p_leaks_before_handshake(tmp_path):
    n = node(tmp_path, "n", "-banscore=10")
    try:
        n.rpc.generate(1)
        # 1. no version, only veracks: disconnected (misbehaving until the ban score)
        noversion = LazyPeer(send_version_first=False)
        noversion.connect("127.0.0.1", n.p2p_port, wait_verack=False)
        for _ in range(10):
            noversion.send(msg_verack())
        noversion.wait_for_disconnect(30)
        # 2. no version, idle: the node sends nothing at all
        idle = LazyPeer(send_version_first=False)
        idle.connect("127.0.0.1", n.p2p_port, wait_verack=False)
        # 3. a version but never a verack, then ping/getaddr: nothing but version/verack back
        noverack = LazyPeer()
        noverack.connect("127.0.0.1", n.p2p_port, wait_verack=False)
        noverack.wait_for(lambda: noverack.peer_version is not None, 30, "version")
        noverack.send(msg_ping(1))
        noverack.send(msg_getaddr())
        n.rpc.generate(1)  # an inv-worthy event while the handshake is incomplete
        time.sleep(2)
        assert idle.unexpected == [] and idle.log == []
        assert noverack.unexpected == [], noverack.unexpected
        # a properly handshaking peer still works
        good = P2PPeer().connect("127.0.0.1", n.p2p_port)
        good.sync_with_ping()
        for p in (idle, noverack, good):
            p.close()
    finally:
        n.stop()


NULLDUMMY_ERROR = "64: non-mandatory-script-verify-flag (Dummy CHECKMULTISIG argument must be zero)"


def test_nulldummy(tmp_path):
    n = node(tmp_path, "n", "-whitelist=127.0.0.1")
    try:
        address = n.rpc.getnewaddress()
        ms_address = n.rpc.addmultisigaddress(1, [address])
        coinbases = n.rpc.generate(2)
        n.rpc.generate(427)  # height 429

        def spend(txid, amount):
            raw = n.rpc.createrawtransaction([{"txid": txid, "vout": 0}], {ms_address: amount})
            tx = CTransaction()
            from_hex(tx, n.rpc.signrawtransaction(raw, None, None, "ALL|FORKID")["hex"])
            return tx

        def true_dummy(tx):
            # the 1-of-1 CHECKMULTISIG scriptSig starts with the empty dummy (OP_0): make it OP_1
            assert tx.vin[0].scriptSig[0] == 0x00
            tx.vin[0].scriptSig = bytes([0x51]) + bytes(tx.vin[0].scriptSig[1:])
            tx.rehash()

        cb0 = n.rpc.getblock(coinbases[0])["tx"][0]
        t1 = spend(cb0, 49)
        txid1 = n.rpc.sendrawtransaction(t1.serialize().hex(), True)
        t2 = spend(txid1, 48)
        txid2 = n.rpc.sendrawtransaction(t2.serialize().hex(), True)
        # compliant transactions are mined
        blk = n.rpc.generate(1)[0]
        assert set(n.rpc.getblock(blk)["tx"][1:]) == {txid1, txid2}
        # a non-null dummy: refused by policy with the reference's message
        t3 = spend(txid2, 47)
        true_dummy(t3)
        with pytest.raises(RPCError) as e:
            n.rpc.sendrawtransaction(t3.serialize().hex(), True)
        assert e.value.message == NULLDUMMY_ERROR
        # ... but valid inside a block (no consensus rule before the fork)
        prev, height, ntime = tip_block(n)
        b = new_block(prev, height + 1, ntime + 1, txs=[t3])
        assert n.rpc.submitblock(b.serialize(legacy=True).hex(), "", True) is None
        assert n.rpc.getbestblockhash() == "%064x" % b.sha256
    finally:
        n.stop()


def test_softfork_heights_bip66_bip65(tmp_path):
    n = node(tmp_path, "n", "-whitelist=127.0.0.1")
    try:
        addr = n.rpc.getnewaddress()
        cbs = n.rpc.generate(6)
        n.rpc.generate(1243)  # height 1249
        peer = P2PPeer().connect("127.0.0.1", n.p2p_port)

        def signed_spend(cbhash):
            txid = n.rpc.getblock(cbhash)["tx"][0]
            raw = n.rpc.createrawtransaction([{"txid": txid, "vout": 0}], {addr: 49.99})
            tx = CTransaction()
            from_hex(tx, n.rpc.signrawtransaction(raw, None, None, "ALL|FORKID")["hex"])
            return tx

        def push(b):
            peer.send(msg_block(b))
            peer.sync_with_ping()
            return n.rpc.getbestblockhash() == "%064x" % b.sha256

        def non_der(tx):
            # pad the DER signature's R with a leading zero: the same ECDSA signature, not strict DER
            ss = bytes(tx.vin[0].scriptSig)
            siglen = ss[0]
            sig = ss[1:1 + siglen]
            assert sig[0] == 0x30 and sig[2] == 0x02
            rlen = sig[3]
            newsig = bytes([0x30, sig[1] + 1, 0x02, rlen + 1, 0]) + sig[4:]
            tx.vin[0].scriptSig = bytes([len(newsig)]) + newsig + ss[1 + siglen:]
            tx.rehash()
            return tx

        def failing_cltv(tx):
            tx.vin[0].scriptSig = bytes(CScript([OP_1NEGATE, OP_CHECKLOCKTIMEVERIFY, OP_DROP])) + bytes(tx.vin[0].scriptSig)
            tx.rehash()
            return tx

        # height 1250: version 2 is still accepted
        prev, h, t = tip_block(n)
        assert h + 1 == 1250 and push(new_block(prev, h + 1, t + 1, version=2))
        # height 1251 (BIP66): version 2 is obsolete
        prev, h, t = tip_block(n)
        bad = new_block(prev, h + 1, t + 1, version=2)
        assert not push(bad)
        r = peer.reject_for(bad.sha256)
        assert r is not None and r.reason == b"bad-version(0x00000002)"
        # the mempool refuses a non-DER signature and a failing CHECKLOCKTIMEVERIFY
        with pytest.raises(RPCError) as e:
            n.rpc.sendrawtransaction(non_der(signed_spend(cbs[0])).serialize().hex())
        assert "Non-canonical DER signature" in e.value.message
        with pytest.raises(RPCError) as e:
            n.rpc.sendrawtransaction(failing_cltv(signed_spend(cbs[1])).serialize().hex())
        assert "Negative locktime" in e.value.message
        # ... while below the BCP fork a block carrying them connects: the reference ignores
        # script failures of pre-fork blocks (src/validation.cpp:2119-2126)
        assert push(new_block(prev, h + 1, t + 1, txs=[non_der(signed_spend(cbs[2]))], version=3))
        n.rpc.generate(99)  # the node's own blocks (version 4), up to 1350
        prev, h, t = tip_block(n)
        assert h == 1350
        # height 1351 (BIP65): version 3 is obsolete, version 4 fine
        bad = new_block(prev, h + 1, t + 1, version=3)
        assert not push(bad)
        r = peer.reject_for(bad.sha256)
        assert r is not None and r.reason == b"bad-version(0x00000003)"
        assert push(new_block(prev, h + 1, t + 1, txs=[failing_cltv(signed_spend(cbs[3]))], version=4))
        # the chain's script flags now include CLTV and DERSIG (getblockchaininfo softforks)
        forks = {f["id"]: f for f in n.rpc.getblockchaininfo()["softforks"]}
        assert forks["bip66"]["reject"]["status"] and forks["bip65"]["reject"]["status"]
        peer.close()
    finally:
        n.stop()


def test_mempool_spend_coinbase(tmp_path):
    n = node(tmp_path, "n")
    try:
        chain_height = 200
        n.rpc.generate(chain_height)
        assert n.rpc.getblockcount() == chain_height
        # coinbases of blocks 101 and 102: the first matures with the next block (201)
        spends = []
        for h in (101, 102):
            cb = n.rpc.getblock(n.rpc.getblockhash(h))["tx"][0]
            raw = n.rpc.createrawtransaction([{"txid": cb, "vout": 0}], {n.rpc.getnewaddress(): 49.99})
            spends.append(n.rpc.signrawtransaction(raw, None, None, "ALL|FORKID")["hex"])
        spend_101_id = n.rpc.sendrawtransaction(spends[0])
        with pytest.raises(RPCError) as e:
            n.rpc.sendrawtransaction(spends[1])
        assert "bad-txns-premature-spend-of-coinbase" in str(e.value)
        assert set(n.rpc.getrawmempool()) == {spend_101_id}
        n.rpc.generate(1)
        assert n.rpc.getrawmempool() == []
        # now the second one matures with the next block
        n.rpc.sendrawtransaction(spends[1])
        assert len(n.rpc.getrawmempool()) == 1
    finally:
        n.stop()


def _connect(a, b):
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    wait_until(lambda: a.rpc.getconnectioncount() >= 1 and b.rpc.getconnectioncount() >= 1)


def _sync(*nodes):
    wait_until(lambda: len({n.rpc.getbestblockhash() for n in nodes}) == 1)


def _read(path):
    with open(path, encoding="utf8") as f:
        return f.read()


def test_forknotify_unknown_block_versions(tmp_path):
    alert = tmp_path / "alert.txt"
    alert.write_text("")
    n0 = node(tmp_path, "n0", "-blockversion=2", f"-alertnotify=echo %s >> \"{alert}\"")
    n1 = node(tmp_path, "n1", "-blockversion=211")
    try:
        n0.rpc.generate(1)  # leave IBD
        _connect(n0, n1)
        _sync(n0, n1)
        n1.rpc.generate(51)
        _sync(n0, n1)
        n1.rpc.generate(1)
        _sync(n0, n1)
        wait_until(lambda: _read(alert) != "", timeout=30)
        text = _read(alert)
        assert "Unknown block versions being mined" in text
        # more up-version blocks raise no further alert
        for _ in range(2):
            n1.rpc.generate(1)
            _sync(n0, n1)
        time.sleep(1)
        assert _read(alert) == text
    finally:
        n1.stop()
        n0.stop()


VB_PERIOD, VB_THRESHOLD = 144, 108
VB_UNKNOWN_BIT = 27
WARN_UNKNOWN_RULES_MINED = "Unknown block versions being mined! It's possible unknown rules are in effect"
WARN_UNKNOWN_RULES_ACTIVE = "unknown new rules activated (versionbit %d)" % VB_UNKNOWN_BIT


def test_versionbits_warning(tmp_path):
    import re
    vb_pattern = re.compile("^Warning.*versionbit")
    alert = tmp_path / "alert.txt"
    alert.write_text("")
    args = (f"-alertnotify=echo %s >> \"{alert}\"",)
    n = node(tmp_path, "n", *args)
    try:
        peer = P2PPeer().connect("127.0.0.1", n.p2p_port)

        def send_blocks(count, version):
            prev, h, t = tip_block(n)
            for _ in range(count):
                b = new_block(prev, h + 1, t + 1, version=version)
                peer.send(msg_block(b))
                prev, h, t = b.sha256, h + 1, t + 1
            peer.sync_with_ping()
            assert n.rpc.getbestblockhash() == "%064x" % prev

        def warnings():
            return [n.rpc.getinfo()["errors"], n.rpc.getmininginfo()["errors"], n.rpc.getnetworkinfo()["warnings"]]

        n.rpc.generate(VB_PERIOD)
        version = 0x20000000 | (1 << VB_UNKNOWN_BIT)
        # a period with one block fewer than the threshold signalling the unknown bit
        send_blocks(VB_THRESHOLD - 1, version)
        n.rpc.generate(VB_PERIOD - VB_THRESHOLD + 1)
        assert not any(vb_pattern.match(w) for w in warnings())
        # a period at the threshold: more than half of the last 100 blocks are unexpected
        send_blocks(VB_THRESHOLD, version)
        n.rpc.generate(VB_PERIOD - VB_THRESHOLD)
        assert all(WARN_UNKNOWN_RULES_MINED in w for w in warnings())
        # one more period locks the bit in; after a restart it is ACTIVE
        n.rpc.generate(VB_PERIOD)
        peer.close()
        n.stop()
        alert.write_text("")
        n.start()
        n.rpc.generate(1)
        assert all(WARN_UNKNOWN_RULES_ACTIVE in w for w in warnings())
        n.stop()
        assert vb_pattern.match(_read(alert))
        n.start()
    finally:
        n.stop()


def test_max_blocks_in_flight(tmp_path):
    import random
    MAX_REQUESTS = 128
    n = node(tmp_path, "n", "-whitelist=127.0.0.1")
    try:
        n.rpc.generate(1)  # leave IBD
        peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
        rng = random.Random(5)
        for count in (8, 16, 128, 1024):
            peer.send(msg_inv([CInv(MSG_BLOCK, rng.randrange(0, 1 << 256)) for _ in range(count)]))
            peer.sync_with_ping()
            time.sleep(2)
            with peer.lock:
                asked = [inv.hash for inv in peer.getdata_requests if inv.type == MSG_BLOCK]
            assert len(asked) == len(set(asked)), "a block was requested more than once"
            assert len(asked) <= MAX_REQUESTS, len(asked)
        peer.sync_with_ping()  # still connected
        peer.close()
    finally:
        n.stop()
