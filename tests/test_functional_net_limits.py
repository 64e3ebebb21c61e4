"""Connection timeouts and the upload target, against a real bcpd.

Parity:
* reference test/functional/p2p-timeouts.py has three inbound peers:
  - one that never sends verack;
  - one that sends a ping but never a version;
  - one that sends nothing.

  They stay connected inside the connect window and are dropped after it. The reference waits
  out the fixed 60-second window. Here `-peertimeout` shortens it; in later reference versions
  that option exists with the same meaning.
* reference test/functional/maxuploadtarget.py, in three parts:
  - with `-maxuploadtarget` below what a day of maximum-size blocks needs, the node stops serving
    historical blocks (more than a week older than its best header). A peer asking for one is
    disconnected, and recent blocks are still served;
  - whitelisted peers are exempt;
  - `getnettotals` reports the target.
"""
import os
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.messages import MSG_BLOCK, CInv, msg_getdata, msg_ping
from bitcoincashplus_amd.testing.p2p import P2PPeer

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


class NoVerackPeer(P2PPeer):
    def on_version(self, msg):
        pass  # never answer with verack


def test_p2p_timeouts(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-peertimeout=4"])
    n.start()
    try:
        no_verack = NoVerackPeer().connect("127.0.0.1", n.p2p_port, wait_verack=False)
        no_version = P2PPeer(send_version_first=False).connect("127.0.0.1", n.p2p_port, wait_verack=False)
        no_send = P2PPeer(send_version_first=False).connect("127.0.0.1", n.p2p_port, wait_verack=False)
        time.sleep(1)
        assert n.rpc.getconnectioncount() == 3
        no_verack.send(msg_ping(1))
        no_version.send(msg_ping(1))
        time.sleep(1)
        assert not (no_verack.closed or no_version.closed or no_send.closed)
        assert no_verack.peer_version is not None  # the node did answer the version
        for p in (no_verack, no_version, no_send):
            p.wait_for_disconnect(timeout=20)
        assert n.rpc.getconnectioncount() == 0
        # a peer that completes the handshake is kept past the window
        ok = P2PPeer().connect("127.0.0.1", n.p2p_port)
        time.sleep(6)
        ok.sync_with_ping()
        assert not ok.closed
        ok.close()
    finally:
        n.stop()


def _getdata(peer, h):
    peer.send(msg_getdata([CInv(MSG_BLOCK, int(h, 16))]))


def _blocks(peer):
    out = []
    for m in list(peer.log):
        if m.command == b"block":
            out.append(m.block.calc_sha256())
    return out


def _got_block(peer, h, timeout=10):
    try:
        peer.wait_for(lambda: int(h, 16) in _blocks(peer), timeout, "block")
        return True
    except Exception:
        return False


def test_maxuploadtarget(tmp_path):
    # 800 MiB a day is less than a day of maximum-size blocks: no historical blocks are served
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-maxuploadtarget=800"])
    n.start()
    try:
        t0 = int(time.time()) - 30 * 24 * 3600
        n.rpc.setmocktime(t0)
        old = n.rpc.generate(5)
        n.rpc.setmocktime(t0 + 8 * 24 * 3600)  # more than a week later
        new = n.rpc.generate(2)
        totals = n.rpc.getnettotals()["uploadtarget"]
        assert totals["target"] == 800 * 1024 * 1024
        assert totals["target_reached"] is False
        assert totals["serve_historical_blocks"] is False
        assert totals["timeframe"] == 24 * 3600

        p = P2PPeer().connect("127.0.0.1", n.p2p_port)
        _getdata(p, new[-1])
        assert _got_block(p, new[-1])  # recent: served
        _getdata(p, old[0])
        p.wait_for_disconnect(timeout=30)  # historical: the peer is dropped
        assert int(old[0], 16) not in _blocks(p)
    finally:
        n.stop()
    # whitelisted peers are exempt
    n2 = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-maxuploadtarget=800", "-whitelist=127.0.0.1"],
                     port=n.rpcport)
    n2.start()
    try:
        n2.rpc.setmocktime(t0 + 8 * 24 * 3600)
        w = P2PPeer().connect("127.0.0.1", n2.p2p_port)
        _getdata(w, old[0])
        assert _got_block(w, old[0])
        w.sync_with_ping()
        assert not w.closed
        w.close()
    finally:
        n2.stop()
