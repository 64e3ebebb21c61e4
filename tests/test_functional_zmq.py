"""ZMQ notifications (reference qa/rpc-tests/zmq_test.py): a ZMTP/3.0 SUB client
written against the wire spec subscribes to hashblock/hashtx/rawblock on a bcpd started
with -zmqpub*, and checks topics, payloads and the LE32 sequence numbers."""
import os
import socket
import struct

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess, free_port

pytestmark = pytest.mark.functional


class ZmtpSub:
    def __init__(self, port, topics):
        self.s = socket.create_connection(("127.0.0.1", port), timeout=10)
        greet = b"\xff" + b"\x00" * 8 + b"\x7f" + bytes([3, 0]) + b"NULL".ljust(20, b"\x00") + b"\x00" + b"\x00" * 31
        self.s.sendall(greet)
        body = b"\x05READY" + b"\x0bSocket-Type" + struct.pack(">I", 3) + b"SUB"
        self.s.sendall(bytes([0x04, len(body)]) + body)
        assert self._recvn(64)[0] == 0xFF
        flags, body = self._frame()
        assert flags & 0x04 and body[1:6] == b"READY"
        for t in topics:
            b = b"\x01" + t
            self.s.sendall(bytes([0x00, len(b)]) + b)

    def _recvn(self, n):
        out = b""
        while len(out) < n:
            chunk = self.s.recv(n - len(out))
            if not chunk:
                raise ConnectionError("closed")
            out += chunk
        return out

    def _frame(self):
        flags = self._recvn(1)[0]
        if flags & 0x02:
            size = struct.unpack(">Q", self._recvn(8))[0]
        else:
            size = self._recvn(1)[0]
        return flags, self._recvn(size)

    def recv_multipart(self):
        parts = []
        while True:
            flags, body = self._frame()
            parts.append(body)
            if not flags & 0x01:
                return parts


def test_zmq_block_and_tx_notifications(tmp_path):
    port = free_port()
    ep = f"tcp://127.0.0.1:{port}"
    n = BcpdProcess(str(tmp_path / "z"), extra_args=["-gpu=0", f"-zmqpubhashblock={ep}", f"-zmqpubhashtx={ep}",
                                                     f"-zmqpubrawblock={ep}"])
    n.start()
    try:
        sub = ZmtpSub(port, [b"hashblock", b"rawblock"])
        import time
        time.sleep(0.3)  # subscription propagation
        hashes = n.rpc.generate(2)
        got = [sub.recv_multipart() for _ in range(4)]
        hb = [g for g in got if g[0] == b"hashblock"]
        rb = [g for g in got if g[0] == b"rawblock"]
        assert [g[1].hex() for g in hb] == hashes
        assert [struct.unpack("<I", g[2])[0] for g in hb] == [0, 1]
        assert rb[0][1].hex() == n.rpc.getblock(hashes[0], False)
        # a tx subscriber sees coinbase txids of new blocks (sequence counts from 0)
        sub2 = ZmtpSub(port, [b"hashtx"])
        time.sleep(0.3)
        h = n.rpc.generate(1)[0]
        msg = sub2.recv_multipart()
        assert msg[0] == b"hashtx" and msg[1].hex() == n.rpc.getblock(h)["tx"][0]
    finally:
        n.stop()


def test_contrib_zmq_sub_client(tmp_path):
    """contrib/zmq/zmq_sub.py (reference contrib/zmq/zmq_sub.py) subscribes and decodes."""
    import importlib.util
    import time
    spec = importlib.util.spec_from_file_location(
        "zmq_sub", os.path.join(os.path.dirname(BIN_DIR), "contrib", "zmq", "zmq_sub.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    port = free_port()
    n = BcpdProcess(str(tmp_path / "z"), extra_args=["-gpu=0", f"-zmqpubhashblock=tcp://127.0.0.1:{port}"])
    n.start()
    try:
        sub = mod.ZmtpSubscriber("127.0.0.1", port, [b"hashblock"], timeout=20)
        time.sleep(0.3)
        h = n.rpc.generate(1)[0]
        line = mod.describe(sub.recv_multipart())
        assert line == f"hashblock #0: {h}"
    finally:
        n.stop()
