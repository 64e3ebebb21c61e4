"""Chain builder for block-rule conformance tests.

Parity: reference test/functional/p2p-fullblocktest.py:91-214 (next_block / update_block / tip /
save_spendable_output bookkeeping: numbered blocks, forks by moving the tip, one spendable
coinbase output consumed per block). Works on both sides of the BCP fork: blocks at
nHeight >= BCPHeight get the 140-byte header, an Equihash solution and the new-format hash.
"""
from __future__ import annotations

import time
import zlib
from typing import Dict, List, Optional

from .blocktools import REGTEST_BITS, SpendableOutput, create_block, create_coinbase, solve
from .messages import REGTEST_BCP_HEIGHT, REGTEST_EQUIHASH, CBlock, COutPoint, CTransaction, CTxIn, CTxOut
from .script import OP_CHECKSIG, OP_TRUE, CScript, Key, push


class FullBlockBuilder:
    def __init__(self, rpc, key: Optional[Key] = None, bcp_height: int = REGTEST_BCP_HEIGHT,
                 equihash=REGTEST_EQUIHASH):
        self.rpc = rpc
        self.key = key or Key(bytes([0x42]) * 32)
        self.bcp_height = bcp_height
        self.equihash = equihash
        best = rpc.getbestblockhash()
        hdr = rpc.getblockheader(best)
        self.base_hash = int(best, 16)
        self.heights: Dict[int, int] = {self.base_hash: hdr["height"]}
        self.block_time = max(int(time.time()), hdr["time"] + 1)
        self.blocks: Dict[int, CBlock] = {}
        self.tip: Optional[CBlock] = None
        self.spendable: List[CBlock] = []
        self.coinbase_script = CScript([self.key.pubkey, OP_CHECKSIG])

    # ---- bookkeeping
    def tip_hash(self) -> int:
        return self.tip.sha256 if self.tip is not None else self.base_hash

    def height_of(self, h: int) -> int:
        return self.heights[h]

    def set_tip(self, number: int) -> CBlock:
        self.tip = self.blocks[number]
        return self.tip

    def save_spendable_output(self):
        self.spendable.append(self.tip)

    def get_spendable_output(self) -> SpendableOutput:
        return SpendableOutput(self.spendable.pop(0).vtx[0], 0)

    # ---- transactions
    def create_tx(self, spend_tx: CTransaction, n: int, value: int, script=CScript([OP_TRUE])) -> CTransaction:
        tx = CTransaction()
        tx.vin.append(CTxIn(COutPoint(spend_tx.calc_sha256(), n), b"", 0xFFFFFFFF))
        tx.vout.append(CTxOut(value, script))
        tx.calc_sha256()
        return tx

    def sign_tx(self, tx: CTransaction, spend_tx: CTransaction, n: int, n_in: int = 0):
        spk = spend_tx.vout[n].scriptPubKey
        if spk == bytes(CScript([OP_TRUE])):  # anyone-can-spend
            tx.vin[n_in].scriptSig = b""
        else:
            tx.vin[n_in].scriptSig = push(self.key.sign_input(tx, n_in, spk, spend_tx.vout[n].nValue))
        tx.rehash()

    def create_and_sign_tx(self, spend_tx: CTransaction, n: int, value: int, script=CScript([OP_TRUE])):
        tx = self.create_tx(spend_tx, n, value, script)
        self.sign_tx(tx, spend_tx, n)
        return tx

    # ---- blocks
    def next_block(self, number: int, spend: Optional[SpendableOutput] = None, additional_coinbase_value: int = 0,
                   script=CScript([OP_TRUE]), solve_it: bool = True, nbits: int = REGTEST_BITS,
                   version: int = 4) -> CBlock:
        prev = self.tip_hash()
        height = self.heights[prev] + 1
        cb = create_coinbase(height, script_pubkey=self.coinbase_script, extra_value=additional_coinbase_value)
        txs = []
        if spend is not None:
            cb.vout[0].nValue += spend.value - 1  # all but one satoshi to fees
            cb.rehash()
            tx = self.create_tx(spend.tx, spend.n, 1, script)  # spend 1 satoshi
            # Signatures are deterministic (RFC6979) here, unlike the reference's OpenSSL signer:
            # a per-block nSequence (nLockTime 0 keeps the tx final) keeps the spends of two
            # sibling blocks distinct, as random signature nonces did there.
            tx.vin[0].nSequence = zlib.crc32(repr(number).encode()) % 0xFFFFFFFF
            self.sign_tx(tx, spend.tx, spend.n)
            txs.append(tx)
        block = create_block(prev, cb, self.block_time, height, nbits, version, txs, self.bcp_height)
        self.block_time += 1
        if solve_it:
            solve(block, self.equihash)
        self.tip = block
        self.heights[block.sha256] = height
        assert number not in self.blocks, number
        self.blocks[number] = block
        return block

    def update_block(self, number: int, new_txs: List[CTransaction], solve_it: bool = True) -> CBlock:
        block = self.blocks[number]
        old = block.sha256
        for t in block.vtx:
            t.rehash()
        for t in new_txs:
            t.rehash()
        block.vtx.extend(new_txs)
        block.hashMerkleRoot = block.calc_merkle_root()
        if solve_it:
            solve(block, self.equihash)
        else:
            block.rehash()
        self.tip = block
        if block.sha256 != old:
            self.heights[block.sha256] = self.heights.pop(old)
        self.blocks[number] = block
        return block

    def resolve(self, block: CBlock) -> CBlock:
        """Re-solve after a header field changed (keeps the height bookkeeping)."""
        old = block.sha256
        solve(block, self.equihash)
        if block.sha256 != old and old in self.heights:
            self.heights[block.sha256] = self.heights.pop(old)
        return block
