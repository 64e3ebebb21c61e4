"""Script construction, sigop counting and FORKID signature hashes for the test peer.

Parity: reference test/functional/test_framework/script.py (CScript, opcodes,
SignatureHashForkId) and src/script/interpreter.cpp:1321-1404 (BIP143-style digest when
SIGHASH_FORKID is set, fork value 0; the legacy digest otherwise), src/script/script.cpp
GetSigOpCount (accurate counting for P2SH redeem scripts, 20 per bare CHECKMULTISIG).
"""
from __future__ import annotations

import struct
from typing import Iterable, Union

from .messages import CTransaction, hash160, hash256, ser_compact_size, ser_string, ser_uint256, sha256

SIGHASH_ALL = 1
SIGHASH_NONE = 2
SIGHASH_SINGLE = 3
SIGHASH_FORKID = 0x40
SIGHASH_ANYONECANPAY = 0x80

OP_0 = OP_FALSE = 0x00
OP_PUSHDATA1, OP_PUSHDATA2, OP_PUSHDATA4 = 0x4C, 0x4D, 0x4E
OP_1NEGATE = 0x4F
OP_1 = OP_TRUE = 0x51
OP_2, OP_3, OP_16 = 0x52, 0x53, 0x60
OP_NOP = 0x61
OP_IF, OP_NOTIF, OP_ELSE, OP_ENDIF, OP_VERIFY, OP_RETURN = 0x63, 0x64, 0x67, 0x68, 0x69, 0x6A
OP_DROP, OP_DUP, OP_2DUP = 0x75, 0x76, 0x6E
OP_CAT, OP_SUBSTR, OP_MUL = 0x7E, 0x7F, 0x95
OP_EQUAL, OP_EQUALVERIFY = 0x87, 0x88
OP_ADD = 0x93
OP_HASH160 = 0xA9
OP_CHECKSIG, OP_CHECKSIGVERIFY, OP_CHECKMULTISIG, OP_CHECKMULTISIGVERIFY = 0xAC, 0xAD, 0xAE, 0xAF
OP_CHECKLOCKTIMEVERIFY, OP_CHECKSEQUENCEVERIFY = 0xB1, 0xB2
OP_INVALIDOPCODE = 0xFF


def push(data: bytes) -> bytes:
    n = len(data)
    if n < OP_PUSHDATA1:
        return bytes([n]) + data
    if n <= 0xFF:
        return bytes([OP_PUSHDATA1, n]) + data
    if n <= 0xFFFF:
        return bytes([OP_PUSHDATA2]) + struct.pack("<H", n) + data
    return bytes([OP_PUSHDATA4]) + struct.pack("<I", n) + data


def script_num(n: int) -> bytes:
    if n == 0:
        return b""
    neg, a, out = n < 0, abs(n), bytearray()
    while a:
        out.append(a & 0xFF)
        a >>= 8
    if out[-1] & 0x80:
        out.append(0x80 if neg else 0)
    elif neg:
        out[-1] |= 0x80
    return bytes(out)


class CScript(bytes):
    """A script assembled from opcodes (ints), byte strings (pushed minimally) and integers
    given as ``CScript.num(n)``."""

    class num(int):
        pass

    def __new__(cls, items: Union[bytes, Iterable] = b""):
        if isinstance(items, (bytes, bytearray)):
            return super().__new__(cls, bytes(items))
        out = bytearray()
        for it in items:
            if isinstance(it, CScript.num):
                if it == 0:
                    out.append(OP_0)
                elif it == -1 or 1 <= it <= 16:
                    out.append(OP_1NEGATE if it == -1 else OP_1 + it - 1)
                else:
                    out += push(script_num(int(it)))
            elif isinstance(it, int):
                out.append(it)
            else:
                out += push(bytes(it))
        return super().__new__(cls, bytes(out))

    def ops(self):
        """(opcode, pushed data or None) pairs; a truncated push ends the iteration with
        (OP_INVALIDOPCODE, None) like the node's GetOp failure."""
        i, b = 0, bytes(self)
        while i < len(b):
            op = b[i]
            i += 1
            if op <= OP_PUSHDATA4:
                if op < OP_PUSHDATA1:
                    n = op
                elif op == OP_PUSHDATA1:
                    if i + 1 > len(b):
                        yield OP_INVALIDOPCODE, None
                        return
                    n, i = b[i], i + 1
                elif op == OP_PUSHDATA2:
                    if i + 2 > len(b):
                        yield OP_INVALIDOPCODE, None
                        return
                    n, i = struct.unpack("<H", b[i:i + 2])[0], i + 2
                else:
                    if i + 4 > len(b):
                        yield OP_INVALIDOPCODE, None
                        return
                    n, i = struct.unpack("<I", b[i:i + 4])[0], i + 4
                if i + n > len(b):
                    yield OP_INVALIDOPCODE, None
                    return
                yield op, b[i:i + n]
                i += n
            else:
                yield op, None

    def sigop_count(self, accurate: bool = False) -> int:
        n, last = 0, OP_INVALIDOPCODE
        for op, _ in self.ops():
            if op == OP_INVALIDOPCODE and _ is None and last is not None:
                pass
            if op in (OP_CHECKSIG, OP_CHECKSIGVERIFY):
                n += 1
            elif op in (OP_CHECKMULTISIG, OP_CHECKMULTISIGVERIFY):
                n += (last - OP_1 + 1) if accurate and OP_1 <= last <= OP_16 else 20
            last = op
        return n


def p2pkh_script(pubkey_hash: bytes) -> CScript:
    return CScript([OP_DUP, OP_HASH160, pubkey_hash, OP_EQUALVERIFY, OP_CHECKSIG])


def p2sh_script(redeem: bytes) -> CScript:
    return CScript([OP_HASH160, hash160(redeem), OP_EQUAL])


def p2pk_script(pubkey: bytes) -> CScript:
    return CScript([pubkey, OP_CHECKSIG])


def signature_hash_forkid(script_code: bytes, tx: CTransaction, n_in: int, hashtype: int, amount: int) -> bytes:
    """BIP143-style digest used with SIGHASH_FORKID (fork value 0)."""
    base = hashtype & 0x1F
    anyone = hashtype & SIGHASH_ANYONECANPAY
    prevouts = sequences = outputs = bytes(32)
    if not anyone:
        prevouts = hash256(b"".join(i.prevout.serialize() for i in tx.vin))
        if base not in (SIGHASH_SINGLE, SIGHASH_NONE):
            sequences = hash256(b"".join(struct.pack("<I", i.nSequence) for i in tx.vin))
    if base not in (SIGHASH_SINGLE, SIGHASH_NONE):
        outputs = hash256(b"".join(o.serialize() for o in tx.vout))
    elif base == SIGHASH_SINGLE and n_in < len(tx.vout):
        outputs = hash256(tx.vout[n_in].serialize())
    pre = (struct.pack("<i", tx.nVersion) + prevouts + sequences + tx.vin[n_in].prevout.serialize() +
           ser_string(bytes(script_code)) + struct.pack("<q", amount) + struct.pack("<I", tx.vin[n_in].nSequence) +
           outputs + struct.pack("<I", tx.nLockTime) + struct.pack("<I", hashtype))
    return hash256(pre)


def signature_hash_legacy(script_code: bytes, tx: CTransaction, n_in: int, hashtype: int) -> bytes:
    """Original digest (pre-fork blocks accept non-FORKID signatures)."""
    one = (1).to_bytes(32, "little")
    if n_in >= len(tx.vin):
        return one
    t = CTransaction(tx)
    code = bytes(b for b in script_code)  # OP_CODESEPARATOR removal is not needed by these tests
    for i, txin in enumerate(t.vin):
        txin.scriptSig = code if i == n_in else b""
    base = hashtype & 0x1F
    if base == SIGHASH_NONE:
        t.vout = []
        for i, txin in enumerate(t.vin):
            if i != n_in:
                txin.nSequence = 0
    elif base == SIGHASH_SINGLE:
        if n_in >= len(t.vout):
            return one
        from .messages import CTxOut
        t.vout = [CTxOut(-1, b"") for _ in range(n_in)] + [t.vout[n_in]]
        for i, txin in enumerate(t.vin):
            if i != n_in:
                txin.nSequence = 0
    if hashtype & SIGHASH_ANYONECANPAY:
        t.vin = [t.vin[n_in]]
    return hash256(t.serialize() + struct.pack("<I", hashtype))


class Key:
    """secp256k1 key backed by the node's signer (RFC6979, low-S DER)."""

    def __init__(self, secret: bytes, compressed: bool = True):
        from bitcoincashplus_amd import native
        self._native = native
        self.secret = secret
        self.compressed = compressed
        self.pubkey = native.ec_pubkey_create(secret, compressed)

    def sign(self, digest: bytes) -> bytes:
        # the digest bytes are the uint256 as the node holds it (sighash bytes as hashed)
        return self._native.ec_sign(self.secret, digest)

    def sign_input(self, tx: CTransaction, n_in: int, script_code: bytes, amount: int,
                   hashtype: int = SIGHASH_ALL | SIGHASH_FORKID) -> bytes:
        if hashtype & SIGHASH_FORKID:
            h = signature_hash_forkid(script_code, tx, n_in, hashtype, amount)
        else:
            h = signature_hash_legacy(script_code, tx, n_in, hashtype)
        return self.sign(h) + bytes([hashtype & 0xFF])


__all__ = [n for n in dir() if n.startswith(("OP_", "SIGHASH_"))] + [
    "CScript", "push", "script_num", "p2pkh_script", "p2sh_script", "p2pk_script", "signature_hash_forkid",
    "signature_hash_legacy", "Key", "hash160", "sha256", "ser_uint256", "ser_compact_size"]
