#!/usr/bin/env python3
"""Print the notifications a bcpd publishes with -zmqpubhashblock/-zmqpubhashtx/
-zmqpubrawblock/-zmqpubrawtx (reference contrib/zmq/zmq_sub.py).

    zmq_sub.py [host:port] [topic ...]      (default 127.0.0.1:28332, all four topics)

No pyzmq needed: the subscriber speaks ZMTP/3.0 (NULL mechanism, SUB socket) directly. Each
message is [topic, body, LE32 sequence]; hashes are printed as hex, raw blocks/txs as their
size and leading bytes.
"""
import socket
import struct
import sys

TOPICS = [b"hashblock", b"hashtx", b"rawblock", b"rawtx"]


class ZmtpSubscriber:
    def __init__(self, host, port, topics, timeout=None):
        self.s = socket.create_connection((host, port), timeout=timeout)
        # greeting: signature, version 3.0, mechanism NULL, as-server 0, filler
        self.s.sendall(b"\xff" + b"\x00" * 8 + b"\x7f" + bytes([3, 0]) + b"NULL".ljust(20, b"\x00") + b"\x00" * 32)
        ready = b"\x05READY" + b"\x0bSocket-Type" + struct.pack(">I", 3) + b"SUB"
        self.s.sendall(bytes([0x04, len(ready)]) + ready)
        greeting = self._recvn(64)
        if greeting[0] != 0xFF or greeting[10] != 3:
            raise ConnectionError("not a ZMTP/3 peer")
        flags, body = self._frame()
        if not flags & 0x04 or body[1:6] != b"READY":
            raise ConnectionError("no READY from publisher")
        for t in topics:  # subscription = message frame 0x01 + prefix
            sub = b"\x01" + t
            self.s.sendall(bytes([0x00, len(sub)]) + sub)

    def _recvn(self, n):
        out = b""
        while len(out) < n:
            chunk = self.s.recv(n - len(out))
            if not chunk:
                raise ConnectionError("publisher closed the connection")
            out += chunk
        return out

    def _frame(self):
        flags = self._recvn(1)[0]
        size = struct.unpack(">Q", self._recvn(8))[0] if flags & 0x02 else self._recvn(1)[0]
        return flags, self._recvn(size)

    def recv_multipart(self):
        parts = []
        while True:
            flags, body = self._frame()
            if flags & 0x04:  # command frame (e.g. PING): not part of a message
                continue
            parts.append(body)
            if not flags & 0x01:
                return parts


def describe(parts):
    topic, body = parts[0], parts[1]
    seq = struct.unpack("<I", parts[2])[0] if len(parts) > 2 and len(parts[2]) == 4 else -1
    if topic in (b"hashblock", b"hashtx"):
        return f"{topic.decode()} #{seq}: {body.hex()}"
    return f"{topic.decode()} #{seq}: {len(body)} bytes {body[:16].hex()}..."


def main(argv):
    target = argv[1] if len(argv) > 1 else "127.0.0.1:28332"
    host, port = target.rsplit(":", 1)
    topics = [t.encode() for t in argv[2:]] or TOPICS
    sub = ZmtpSubscriber(host, int(port), topics)
    try:
        while True:
            print(describe(sub.recv_multipart()), flush=True)
    except KeyboardInterrupt:
        pass


if __name__ == "__main__":
    main(sys.argv)
