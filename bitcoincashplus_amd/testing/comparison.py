"""Accept/reject driver for block-rule conformance tests.

Parity: reference test/functional/test_framework/comptool.py (TestManager / TestInstance /
RejectResult): a block expected to be accepted is announced (inv) and fetched by the node
through getheaders/getdata from the peer's store, then must become the tip; a block expected
to be rejected is pushed unsolicited (the peer is whitelisted, so the node processes it),
followed by a ping, and must not become the tip - with, when given, a reject message whose
code matches and whose reason starts with the expected reason.
"""
from __future__ import annotations

import time
from typing import List, Optional, Union

from .messages import CBlock, CBlockHeader, CInv, MSG_BLOCK, MSG_TX, CTransaction, msg_block, msg_headers, msg_inv
from .p2p import P2PPeer


class RejectResult:
    def __init__(self, code: int, reason: bytes = b""):
        self.code = code
        self.reason = reason

    def match(self, other) -> bool:
        return self.code == other.code and other.reason.startswith(self.reason)

    def __repr__(self):
        return f"RejectResult({self.code}, {self.reason!r})"


class BlockRuleDriver:
    def __init__(self, rpc, peer: P2PPeer, timeout: float = 60):
        self.rpc = rpc
        self.peer = peer
        self.timeout = timeout

    def tip(self) -> int:
        return int(self.rpc.getbestblockhash(), 16)

    def wait_tip(self, h: int):
        deadline = time.time() + self.timeout
        while time.time() < deadline:
            if self.tip() == h:
                return
            time.sleep(0.02)
        raise AssertionError(f"tip is {self.tip():064x}, expected {h:064x}")

    def accept(self, block: CBlock, tip: Optional[int] = None):
        """Announce `block` (and anything in the store it builds on); the node must end with
        `tip` (default: this block) as its best block."""
        block.calc_sha256()
        self.peer.store.add_block(block)
        self.peer.send(msg_inv([CInv(MSG_BLOCK, block.sha256)]))
        self.wait_tip(block.sha256 if tip is None else tip)
        self.peer.sync_with_ping()

    def reject(self, block: CBlock, result: Optional[RejectResult] = None, tip: Optional[int] = None):
        """Push `block` unsolicited; it must not become the tip (`tip`: the expected best block,
        default unchanged); with `result`, the node must answer with a matching reject."""
        block.calc_sha256()
        before = self.tip()
        self.peer.store.add_block(block)
        self.peer.send(msg_block(block))
        self.peer.sync_with_ping()
        now = self.tip()
        assert now != block.sha256, f"block {block.hash} was accepted as tip"
        assert now == (before if tip is None else tip), f"tip moved to {now:064x}"
        if result is not None:
            r = self.peer.reject_for(block.sha256)
            assert r is not None, f"no reject message for block {block.hash} (expected {result})"
            assert result.match(r), f"reject {r} for block {block.hash}, expected {result}"

    def push(self, block: CBlock):
        """Deliver a block without an outcome check (it may or may not connect)."""
        block.calc_sha256()
        self.peer.store.add_block(block)
        self.peer.send(msg_block(block))
        self.peer.sync_with_ping()

    def headers(self, headers: List[CBlockHeader]):
        for h in headers:
            self.peer.store.add_header(h)
        self.peer.send(msg_headers(headers))
        self.peer.sync_with_ping()

    def mempool_has(self, tx: Union[CTransaction, int]) -> bool:
        h = tx if isinstance(tx, int) else tx.calc_sha256()
        return f"{h:064x}" in self.rpc.getrawmempool()
