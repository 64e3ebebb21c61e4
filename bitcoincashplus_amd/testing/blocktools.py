"""Block and transaction construction for the test peer, pre- and post-fork.

Parity: reference test/functional/test_framework/blocktools.py (create_block, create_coinbase,
create_transaction, get_legacy_sigopcount_*) and mininode.py CBlock.solve (:727-731, SHA256d
only). Post-fork blocks (nHeight >= BCPHeight) are solved here: for each 256-bit nonce the
node's CPU Equihash solver (native.eh_solve_cpu, the reference's BasicSolve) enumerates the
solutions of BLAKE2b(CEquihashInput || nonce), and the first whose new-format SHA256d header
hash meets nBits is kept (reference src/rpc/mining.cpp:161-199 / src/pow.cpp:141-163).
"""
from __future__ import annotations

import struct
from typing import Iterable, List, Optional

from .messages import (COIN, REGTEST_BCP_HEIGHT, REGTEST_EQUIHASH, CBlock, COutPoint, CTransaction, CTxIn, CTxOut,
                       uint256_from_compact)
from .script import OP_CHECKSIG, OP_TRUE, CScript, push, script_num

REGTEST_BITS = 0x207FFFFF
REGTEST_HALVING = 150


def subsidy(height: int, halving: int = REGTEST_HALVING) -> int:
    h = height // halving
    return 0 if h >= 64 else (50 * COIN) >> h


def create_coinbase(height: int, pubkey: Optional[bytes] = None, extra_value: int = 0,
                    script_pubkey: Optional[bytes] = None, halving: int = REGTEST_HALVING,
                    script_sig_extra: bytes = b"") -> CTransaction:
    """Coinbase paying subsidy(height) + extra_value to pubkey (P2PK) or OP_TRUE; the height
    goes first in the scriptSig (BIP34 layout)."""
    cb = CTransaction()
    sig = push(script_num(height)) if height > 16 else bytes([0x50 + height]) if height else b"\x00"
    sig += b"\x51" + script_sig_extra  # keep scriptSig >= 2 bytes
    cb.vin.append(CTxIn(COutPoint(0, 0xFFFFFFFF), sig, 0xFFFFFFFF))
    if script_pubkey is None:
        script_pubkey = CScript([pubkey, OP_CHECKSIG]) if pubkey is not None else CScript([OP_TRUE])
    cb.vout.append(CTxOut(subsidy(height, halving) + extra_value, script_pubkey))
    cb.rehash()
    return cb


def create_transaction(prev: CTransaction, n: int, script_sig: bytes, value: int,
                       script_pubkey: bytes = CScript([OP_TRUE])) -> CTransaction:
    tx = CTransaction()
    tx.vin.append(CTxIn(COutPoint(prev.calc_sha256(), n), script_sig, 0xFFFFFFFF))
    tx.vout.append(CTxOut(value, script_pubkey))
    tx.calc_sha256()
    return tx


def create_block(prev_hash: int, coinbase: CTransaction, ntime: int, height: int, nbits: int = REGTEST_BITS,
                 version: int = 4, txs: Iterable[CTransaction] = (), bcp_height: int = REGTEST_BCP_HEIGHT) -> CBlock:
    b = CBlock(bcp_height=bcp_height)
    b.nVersion = version
    b.hashPrevBlock = prev_hash
    b.nTime = ntime
    b.nBits = nbits
    b.nHeight = height
    b.vtx = [coinbase] + list(txs)
    b.hashMerkleRoot = b.calc_merkle_root()
    if b.is_new_format():  # placeholder of the solution's size, so sizes are final before solving
        b.nSolution = bytes(solution_width(*REGTEST_EQUIHASH))
    b.calc_sha256()
    return b


def solution_width(n: int, k: int) -> int:
    """Bytes of a minimal Equihash solution: 2^K indices of N/(K+1)+1 bits."""
    return (1 << k) * (n // (k + 1) + 1) // 8


def solve(block: CBlock, equihash=REGTEST_EQUIHASH, max_tries: int = 1 << 20) -> CBlock:
    """Find a nonce (and, post-fork, an Equihash solution) meeting nBits."""
    target = uint256_from_compact(block.nBits)
    if not block.is_new_format():
        block.nSolution = b""
        for _ in range(max_tries):
            if block.rehash() <= target:
                return block
            block.nNonce = (block.nNonce + 1) & 0xFFFFFFFF
        raise RuntimeError("solve: no legacy nonce found")
    from bitcoincashplus_amd import native
    n, k = equihash
    inp = block.equihash_input()
    for _ in range(max_tries):
        st = native.EquihashState(n, k)
        st.update(inp + block.nNonce.to_bytes(32, "little"))
        for sol in native.eh_solve_cpu(n, k, st)[0]:
            block.nSolution = bytes(sol)
            if block.rehash() <= target:
                return block
        block.nNonce += 1
    raise RuntimeError("solve: no Equihash solution met the target")


def legacy_sigop_count_tx(tx: CTransaction) -> int:
    """GetSigOpCount(false) over scriptSigs and scriptPubKeys (reference GetLegacySigOpCount)."""
    return sum(CScript(i.scriptSig).sigop_count() for i in tx.vin) + \
        sum(CScript(o.scriptPubKey).sigop_count() for o in tx.vout)


def legacy_sigop_count_block(block: CBlock) -> int:
    return sum(legacy_sigop_count_tx(t) for t in block.vtx)


class SpendableOutput:
    def __init__(self, tx: CTransaction, n: int):
        self.tx = tx
        self.n = n

    @property
    def value(self) -> int:
        return self.tx.vout[self.n].nValue


__all__ = ["subsidy", "create_coinbase", "create_transaction", "create_block", "solve", "legacy_sigop_count_tx",
           "legacy_sigop_count_block", "SpendableOutput", "REGTEST_BITS", "REGTEST_HALVING"]
