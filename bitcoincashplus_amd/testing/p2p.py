"""Threaded P2P test peer.

Parity: reference test/functional/test_framework/mininode.py (NodeConn framing with magic,
12-byte command, length and SHA256d checksum; NodeConnCB callbacks; sync_with_ping) and
comptool.py's TestNode (serves the blocks/headers/transactions of a shared store on
getheaders/getdata). The peer can announce a protocol version below BCP_HARD_FORK_VERSION
(70016): the node then sends and expects the legacy 80-byte header layout
(reference src/net.h:813-815, src/net_processing.cpp:1236,2054,2622,2824,3513).
"""
from __future__ import annotations

import io
import socket
import struct
import threading
import time
from typing import Callable, Dict, List, Optional

from .messages import (BCP_HARD_FORK_VERSION, MESSAGE_MAP, MSG_BLOCK, MSG_CMPCT_BLOCK, MSG_TX, MY_VERSION,
                       REGTEST_MAGIC, CBlock, CBlockHeader, CInv, CTransaction, Msg, hash256, msg_block,
                       msg_getheaders, msg_headers, msg_inv, msg_notfound, msg_ping, msg_pong, msg_tx, msg_verack,
                       msg_version)


class P2PError(Exception):
    pass


class BlockStore:
    """Blocks, headers and transactions the test offers to the node (comptool BlockStore)."""

    def __init__(self):
        self.blocks: Dict[int, CBlock] = {}
        self.headers: Dict[int, CBlockHeader] = {}
        self.txs: Dict[int, CTransaction] = {}

    def add_block(self, b: CBlock):
        b.calc_sha256()
        self.blocks[b.sha256] = b
        self.headers[b.sha256] = CBlockHeader(b)

    def add_header(self, h: CBlockHeader):
        h.calc_sha256()
        self.headers[h.sha256] = h

    def headers_for(self, locator: List[int], hashstop: int, limit: int = 2000) -> Optional[List[CBlockHeader]]:
        """Headers from the last locator hash this store's chain to `hashstop` shares, forward."""
        if hashstop not in self.headers:
            return None
        chain = []
        h = hashstop
        known = set(locator)
        while h in self.headers and h not in known:
            chain.append(self.headers[h])
            h = self.headers[h].hashPrevBlock
        chain.reverse()
        return chain[:limit]


class P2PPeer:
    """One connection to a node. Messages are parsed on a reader thread; the latest message of
    each command, every received message (``log``) and the reject messages are kept for the
    test's wait_* helpers. Subclasses or ``handlers`` add on_<command> callbacks."""

    def __init__(self, version: int = MY_VERSION, magic: bytes = REGTEST_MAGIC, store: Optional[BlockStore] = None,
                 services: int = 1, send_version_first: bool = True):
        self.our_version = version
        self.magic = magic
        self.services = services
        self.store = store if store is not None else BlockStore()
        self.sock: Optional[socket.socket] = None
        self.lock = threading.RLock()
        self.cv = threading.Condition(self.lock)
        self.last: Dict[bytes, Msg] = {}
        self.counts: Dict[bytes, int] = {}
        self.log: List[Msg] = []
        self.rejects: List = []
        self.getdata_requests: List[CInv] = []
        self.peer_version: Optional[msg_version] = None
        self.verack_received = False
        self.closed = False
        self.ping_nonce = 0
        self.handlers: Dict[bytes, Callable] = {}
        self.send_version_first = send_version_first
        self.serve_store = True
        self._reader: Optional[threading.Thread] = None
        self._sendlock = threading.Lock()
        self.bytes_sent = 0

    # ---- connection
    @property
    def negotiated_version(self) -> int:
        if self.peer_version is None:
            return self.our_version
        return min(self.our_version, self.peer_version.nVersion)

    @property
    def legacy(self) -> bool:
        """True when block headers travel in the 80-byte layout on this connection."""
        return self.negotiated_version < BCP_HARD_FORK_VERSION

    def connect(self, host: str, port: int, timeout: float = 30, wait_verack: bool = True):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.settimeout(None)
        self._reader = threading.Thread(target=self._read_loop, daemon=True)
        self._reader.start()
        if self.send_version_first:
            v = msg_version(self.our_version)
            v.nServices = self.services
            self.send(v)
        if wait_verack:
            self.wait_for(lambda: self.verack_received, timeout, "verack")
        return self

    def close(self):
        self.closed = True
        if self.sock is not None:
            try:
                self.sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            self.sock.close()
        if self._reader is not None:
            self._reader.join(timeout=10)

    # ---- framing
    def frame(self, command: bytes, payload: bytes) -> bytes:
        return (self.magic + command.ljust(12, b"\0") + struct.pack("<I", len(payload)) + hash256(payload)[:4] +
                payload)

    def send(self, msg: Msg):
        self.send_raw(msg.command, msg.serialize(legacy=self.legacy))

    def send_raw(self, command: bytes, payload: bytes, data: Optional[bytes] = None):
        buf = data if data is not None else self.frame(command, payload)
        with self._sendlock:
            if self.closed or self.sock is None:
                raise P2PError("not connected")
            self.sock.sendall(buf)
            self.bytes_sent += len(buf)

    def _read_loop(self):
        buf = b""
        try:
            while True:
                chunk = self.sock.recv(1 << 16)
                if not chunk:
                    break
                buf += chunk
                while len(buf) >= 24:
                    if buf[:4] != self.magic:
                        raise P2PError(f"bad magic {buf[:4].hex()}")
                    cmd = buf[4:16].rstrip(b"\0")
                    n = struct.unpack("<I", buf[16:20])[0]
                    if len(buf) < 24 + n:
                        break
                    payload = buf[24:24 + n]
                    if hash256(payload)[:4] != buf[20:24]:
                        raise P2PError("bad checksum")
                    buf = buf[24 + n:]
                    self._dispatch(cmd, payload)
        except (OSError, P2PError):
            pass
        finally:
            with self.cv:
                self.closed = True
                self.cv.notify_all()

    def _dispatch(self, cmd: bytes, payload: bytes):
        cls = MESSAGE_MAP.get(cmd)
        if cls is None:
            return
        msg = cls()
        msg.deserialize(io.BytesIO(payload), legacy=self.legacy)
        with self.cv:
            self.last[cmd] = msg
            self.counts[cmd] = self.counts.get(cmd, 0) + 1
            self.log.append(msg)
            if cmd == b"version":
                self.peer_version = msg
            elif cmd == b"reject":
                self.rejects.append(msg)
            self.cv.notify_all()
        h = self.handlers.get(cmd) or getattr(self, "on_" + cmd.decode(), None)
        if h is not None:
            h(msg)
        with self.cv:
            self.cv.notify_all()

    # ---- default behaviour
    def on_version(self, msg):
        if not self.send_version_first:
            v = msg_version(self.our_version)
            v.nServices = self.services
            self.send(v)
        self.send(msg_verack())

    def on_verack(self, msg):
        with self.cv:
            self.verack_received = True

    def on_ping(self, msg):
        self.send(msg_pong(msg.nonce))

    def on_getheaders(self, msg):
        if not self.serve_store:
            return
        hs = self.store.headers_for(msg.locator.vHave, msg.hashstop)
        if hs:
            self.send(msg_headers(hs))

    def on_getdata(self, msg):
        with self.cv:
            self.getdata_requests.extend(msg.inv)
        if not self.serve_store:
            return
        missing = []
        for inv in msg.inv:
            if inv.type in (MSG_BLOCK, MSG_CMPCT_BLOCK) and inv.hash in self.store.blocks:
                self.send(msg_block(self.store.blocks[inv.hash]))
            elif inv.type == MSG_TX and inv.hash in self.store.txs:
                self.send(msg_tx(self.store.txs[inv.hash]))
            else:
                missing.append(inv)
        if missing:
            self.send(msg_notfound(missing))

    # ---- waiting
    def wait_for(self, pred: Callable[[], bool], timeout: float = 60, what: str = "condition"):
        deadline = time.time() + timeout
        with self.cv:
            while not pred():
                left = deadline - time.time()
                if left <= 0:
                    raise AssertionError(f"P2PPeer: timed out waiting for {what}")
                if self.closed and not pred():
                    raise AssertionError(f"P2PPeer: disconnected while waiting for {what}")
                self.cv.wait(min(left, 0.5))

    def wait_for_disconnect(self, timeout: float = 60):
        deadline = time.time() + timeout
        with self.cv:
            while not self.closed:
                left = deadline - time.time()
                if left <= 0:
                    raise AssertionError("P2PPeer: still connected")
                self.cv.wait(min(left, 0.5))

    def wait_for_message(self, command: bytes, timeout: float = 60, since: int = 0) -> Msg:
        self.wait_for(lambda: self.counts.get(command, 0) > since, timeout, command.decode())
        return self.last[command]

    def sync_with_ping(self, timeout: float = 60):
        """Every message sent before this call has been processed by the node."""
        with self.cv:
            self.ping_nonce += 1
            nonce = self.ping_nonce
        self.send(msg_ping(nonce))
        self.wait_for(lambda: any(isinstance(m, msg_pong) and m.nonce == nonce for m in self.log[-64:]), timeout,
                      "pong")

    def clear(self):
        with self.cv:
            self.last.clear()
            self.counts.clear()
            self.log.clear()
            self.rejects.clear()
            self.getdata_requests.clear()

    def reject_for(self, h: int):
        with self.cv:
            for r in reversed(self.rejects):
                if r.data == h:
                    return r
        return None

    # ---- helpers
    def send_inv_blocks(self, hashes: List[int]):
        self.send(msg_inv([CInv(MSG_BLOCK, h) for h in hashes]))

    def send_getheaders(self, locator: List[int], hashstop: int = 0):
        self.send(msg_getheaders(locator, hashstop))
