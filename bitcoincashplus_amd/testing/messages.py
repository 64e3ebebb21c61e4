"""Wire objects and P2P messages of the BCP protocol, in pure Python.

Parity: reference test/functional/test_framework/mininode.py (message classes,
CBlockHeader with both header formats keyed on BCP_REGTEST_HARDFORK_HEIGHT, :42,566-660)
and the C++ wire format of src/primitives/block.h:30-95, src/protocol.h, src/blockencodings.h
and src/bloom.h. Every object serializes to bytes with ``serialize()`` and parses with
``deserialize(stream)``; block headers take a ``legacy`` flag (80-byte Bitcoin layout with the
low 32 bits of the 256-bit nonce, used for peers below protocol 70016).
"""
from __future__ import annotations

import copy
import hashlib
import io
import random
import struct
import time
from typing import List, Optional

MY_VERSION = 70016            # BCP_HARD_FORK_VERSION: new-format headers on the wire
LEGACY_VERSION = 70014        # SHORT_IDS_BLOCKS_VERSION, below the fork version: 80-byte headers
BCP_HARD_FORK_VERSION = 70016
MY_SUBVERSION = b"/pytest-peer:0.3/"
NODE_NETWORK = 1
NODE_BLOOM = 4
MAX_INV_SZ = 50000
MAX_HEADERS_RESULTS = 2000
COIN = 100_000_000
MAX_BLOCK_SIGOPS_PER_MB = 20000
MAX_TX_SIGOPS_COUNT = 20000
ONE_MEGABYTE = 1_000_000
LEGACY_MAX_BLOCK_SIZE = ONE_MEGABYTE
DEFAULT_MAX_BLOCK_SIZE = 8 * ONE_MEGABYTE
MAX_SCRIPT_ELEMENT_SIZE = 520

MSG_TX = 1
MSG_BLOCK = 2
MSG_FILTERED_BLOCK = 3
MSG_CMPCT_BLOCK = 4

REGTEST_MAGIC = bytes([0x46, 0x6D, 0x47, 0xE1])
REGTEST_BCP_HEIGHT = 3000
REGTEST_EQUIHASH = (48, 5)


# ------------------------------------------------------------------ primitives

def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def hash256(b: bytes) -> bytes:
    return sha256(sha256(b))


def ripemd160(msg: bytes) -> bytes:
    """Pure-Python RIPEMD-160 (this image's OpenSSL does not provide it to hashlib)."""
    def rol(x, n):
        return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF

    def f(j, x, y, z):
        if j < 16:
            return x ^ y ^ z
        if j < 32:
            return (x & y) | (~x & z)
        if j < 48:
            return (x | ~y) ^ z
        if j < 64:
            return (x & z) | (y & ~z)
        return x ^ (y | ~z)

    KL = (0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E)
    KR = (0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000)
    RL = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9, 5, 2, 14, 11, 8,
          3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12, 1, 9, 11, 10, 0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2,
          4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13]
    RR = [5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12, 6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8, 12, 4, 9, 1, 2,
          15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13, 8, 6, 4, 1, 3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14,
          12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11]
    SL = [11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8, 7, 6, 8, 13, 11, 9, 7, 15, 7, 12, 15, 9, 11, 7, 13,
          12, 11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5, 11, 12, 14, 15, 14, 15, 9, 8, 9, 14, 5, 6, 8, 6,
          5, 12, 9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6]
    SR = [8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6, 9, 13, 15, 7, 12, 8, 9, 11, 7, 7, 12, 7, 6, 15, 13,
          11, 9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5, 15, 5, 8, 11, 14, 14, 6, 14, 6, 9, 12, 9, 12, 5,
          15, 8, 8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11]
    h = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
    data = msg + b"\x80" + b"\x00" * ((55 - len(msg)) % 64) + struct.pack("<Q", 8 * len(msg))
    for off in range(0, len(data), 64):
        X = struct.unpack("<16I", data[off:off + 64])
        al, bl, cl, dl, el = h
        ar, br, cr, dr, er = h
        for j in range(80):
            t = (rol((al + (f(j, bl, cl, dl) & 0xFFFFFFFF) + X[RL[j]] + KL[j // 16]) & 0xFFFFFFFF, SL[j]) + el) & 0xFFFFFFFF
            al, el, dl, cl, bl = el, dl, rol(cl, 10), bl, t
            t = (rol((ar + (f(79 - j, br, cr, dr) & 0xFFFFFFFF) + X[RR[j]] + KR[j // 16]) & 0xFFFFFFFF, SR[j]) + er) & 0xFFFFFFFF
            ar, er, dr, cr, br = er, dr, rol(cr, 10), br, t
        t = (h[1] + cl + dr) & 0xFFFFFFFF
        h[1] = (h[2] + dl + er) & 0xFFFFFFFF
        h[2] = (h[3] + el + ar) & 0xFFFFFFFF
        h[3] = (h[4] + al + br) & 0xFFFFFFFF
        h[4] = (h[0] + bl + cr) & 0xFFFFFFFF
        h[0] = t
    return struct.pack("<5I", *h)


def hash160(b: bytes) -> bytes:
    return ripemd160(sha256(b))


def ser_compact_size(n: int) -> bytes:
    if n < 253:
        return bytes([n])
    if n < 0x10000:
        return b"\xfd" + struct.pack("<H", n)
    if n < 0x100000000:
        return b"\xfe" + struct.pack("<I", n)
    return b"\xff" + struct.pack("<Q", n)


def deser_compact_size(f) -> int:
    n = f.read(1)[0]
    if n == 253:
        return struct.unpack("<H", f.read(2))[0]
    if n == 254:
        return struct.unpack("<I", f.read(4))[0]
    if n == 255:
        return struct.unpack("<Q", f.read(8))[0]
    return n


def ser_string(b: bytes) -> bytes:
    return ser_compact_size(len(b)) + b


def deser_string(f) -> bytes:
    return f.read(deser_compact_size(f))


def ser_uint256(u: int) -> bytes:
    return u.to_bytes(32, "little")


def deser_uint256(f) -> int:
    return int.from_bytes(f.read(32), "little")


def uint256_from_bytes(b: bytes) -> int:
    return int.from_bytes(b[:32], "little")


def uint256_from_compact(c: int) -> int:
    nbytes = (c >> 24) & 0xFF
    return (c & 0x007FFFFF) << (8 * (nbytes - 3)) if nbytes >= 3 else (c & 0x007FFFFF) >> (8 * (3 - nbytes))


def ser_vector(items, **kw) -> bytes:
    return ser_compact_size(len(items)) + b"".join(i.serialize(**kw) for i in items)


def deser_vector(f, cls, **kw) -> list:
    out = []
    for _ in range(deser_compact_size(f)):
        o = cls()
        o.deserialize(f, **kw)
        out.append(o)
    return out


def ser_uint256_vector(v) -> bytes:
    return ser_compact_size(len(v)) + b"".join(ser_uint256(x) for x in v)


def deser_uint256_vector(f) -> list:
    return [deser_uint256(f) for _ in range(deser_compact_size(f))]


def hex_str(b: bytes) -> str:
    return b.hex()


def from_hex(obj, hex_string: str):
    obj.deserialize(io.BytesIO(bytes.fromhex(hex_string)))
    return obj


# ------------------------------------------------------------------ transactions

class COutPoint:
    def __init__(self, hash: int = 0, n: int = 0):
        self.hash = hash
        self.n = n

    def deserialize(self, f):
        self.hash = deser_uint256(f)
        self.n = struct.unpack("<I", f.read(4))[0]

    def serialize(self) -> bytes:
        return ser_uint256(self.hash) + struct.pack("<I", self.n)

    def __repr__(self):
        return f"COutPoint({self.hash:064x}:{self.n})"


class CTxIn:
    def __init__(self, outpoint: Optional[COutPoint] = None, scriptSig: bytes = b"", nSequence: int = 0xFFFFFFFF):
        self.prevout = outpoint or COutPoint()
        self.scriptSig = bytes(scriptSig)
        self.nSequence = nSequence

    def deserialize(self, f):
        self.prevout = COutPoint()
        self.prevout.deserialize(f)
        self.scriptSig = deser_string(f)
        self.nSequence = struct.unpack("<I", f.read(4))[0]

    def serialize(self) -> bytes:
        return self.prevout.serialize() + ser_string(bytes(self.scriptSig)) + struct.pack("<I", self.nSequence)


class CTxOut:
    def __init__(self, nValue: int = 0, scriptPubKey: bytes = b""):
        self.nValue = nValue
        self.scriptPubKey = bytes(scriptPubKey)

    def deserialize(self, f):
        self.nValue = struct.unpack("<q", f.read(8))[0]
        self.scriptPubKey = deser_string(f)

    def serialize(self) -> bytes:
        return struct.pack("<q", self.nValue) + ser_string(bytes(self.scriptPubKey))


class CTransaction:
    def __init__(self, tx: Optional["CTransaction"] = None):
        if tx is None:
            self.nVersion = 1
            self.vin: List[CTxIn] = []
            self.vout: List[CTxOut] = []
            self.nLockTime = 0
            self.sha256 = None
            self.hash = None
        else:
            self.nVersion = tx.nVersion
            self.vin = copy.deepcopy(tx.vin)
            self.vout = copy.deepcopy(tx.vout)
            self.nLockTime = tx.nLockTime
            self.sha256 = tx.sha256
            self.hash = tx.hash

    def deserialize(self, f):
        self.nVersion = struct.unpack("<i", f.read(4))[0]
        self.vin = deser_vector(f, CTxIn)
        self.vout = deser_vector(f, CTxOut)
        self.nLockTime = struct.unpack("<I", f.read(4))[0]
        self.sha256 = None
        self.hash = None

    def serialize(self) -> bytes:
        return (struct.pack("<i", self.nVersion) + ser_vector(self.vin) + ser_vector(self.vout) +
                struct.pack("<I", self.nLockTime))

    def rehash(self) -> str:
        self.sha256 = None
        self.calc_sha256()
        return self.hash

    def calc_sha256(self):
        if self.sha256 is None:
            h = hash256(self.serialize())
            self.sha256 = uint256_from_bytes(h)
            self.hash = h[::-1].hex()
        return self.sha256

    def is_coinbase(self) -> bool:
        return len(self.vin) == 1 and self.vin[0].prevout.hash == 0 and self.vin[0].prevout.n == 0xFFFFFFFF

    def is_valid_amounts(self) -> bool:
        return all(0 <= o.nValue <= 21_000_000 * COIN for o in self.vout)

    def __len__(self):
        return len(self.serialize())

    def __repr__(self):
        return f"CTransaction({self.hash}, {len(self.vin)} in, {len(self.vout)} out)"


# ------------------------------------------------------------------ blocks

class CBlockHeader:
    """BCP header: both serializations. ``bcp_height`` selects the hashing format by the
    header's own nHeight (reference src/primitives/block.cpp:17-28)."""

    def __init__(self, header: Optional["CBlockHeader"] = None, bcp_height: int = REGTEST_BCP_HEIGHT):
        if header is None:
            self.set_null()
            self.bcp_height = bcp_height
        else:
            self.nVersion = header.nVersion
            self.hashPrevBlock = header.hashPrevBlock
            self.hashMerkleRoot = header.hashMerkleRoot
            self.nHeight = header.nHeight
            self.nReserved = list(header.nReserved)
            self.nTime = header.nTime
            self.nBits = header.nBits
            self.nNonce = header.nNonce
            self.nSolution = bytes(header.nSolution)
            self.bcp_height = header.bcp_height
            self.sha256 = header.sha256
            self.hash = header.hash
            self.calc_sha256()

    def set_null(self):
        self.nVersion = 4
        self.hashPrevBlock = 0
        self.hashMerkleRoot = 0
        self.nHeight = 0
        self.nReserved = [0] * 7
        self.nTime = 0
        self.nBits = 0
        self.nNonce = 0
        self.nSolution = b""
        self.sha256 = None
        self.hash = None

    def is_new_format(self) -> bool:
        return self.nHeight >= self.bcp_height

    def deserialize(self, f, legacy: bool = False):
        self.nVersion = struct.unpack("<i", f.read(4))[0]
        self.hashPrevBlock = deser_uint256(f)
        self.hashMerkleRoot = deser_uint256(f)
        if legacy:
            self.nHeight = 0
            self.nReserved = [0] * 7
        else:
            self.nHeight = struct.unpack("<I", f.read(4))[0]
            self.nReserved = list(struct.unpack("<7I", f.read(28)))
        self.nTime = struct.unpack("<I", f.read(4))[0]
        self.nBits = struct.unpack("<I", f.read(4))[0]
        if legacy:
            self.nNonce = struct.unpack("<I", f.read(4))[0]
            self.nSolution = b""
        else:
            self.nNonce = deser_uint256(f)
            self.nSolution = deser_string(f)
        self.sha256 = None
        self.hash = None

    def serialize_header(self, legacy: bool = False) -> bytes:
        r = struct.pack("<i", self.nVersion) + ser_uint256(self.hashPrevBlock) + ser_uint256(self.hashMerkleRoot)
        if legacy:
            return r + struct.pack("<III", self.nTime, self.nBits, self.nNonce & 0xFFFFFFFF)
        r += struct.pack("<I", self.nHeight) + struct.pack("<7I", *self.nReserved)
        return r + struct.pack("<II", self.nTime, self.nBits) + ser_uint256(self.nNonce) + ser_string(self.nSolution)

    def serialize(self, legacy: bool = False) -> bytes:
        return self.serialize_header(legacy)

    def equihash_input(self) -> bytes:
        """CEquihashInput: the first 108 bytes of the new format (no nonce, no solution)."""
        return (struct.pack("<i", self.nVersion) + ser_uint256(self.hashPrevBlock) +
                ser_uint256(self.hashMerkleRoot) + struct.pack("<I", self.nHeight) +
                struct.pack("<7I", *self.nReserved) + struct.pack("<II", self.nTime, self.nBits))

    def calc_sha256(self) -> int:
        if self.sha256 is None:
            h = hash256(self.serialize_header(legacy=not self.is_new_format()))
            self.sha256 = uint256_from_bytes(h)
            self.hash = h[::-1].hex()
        return self.sha256

    def rehash(self) -> int:
        self.sha256 = None
        return self.calc_sha256()

    def __repr__(self):
        return f"CBlockHeader(h={self.nHeight} hash={self.hash} prev={self.hashPrevBlock:064x})"


class CBlock(CBlockHeader):
    def __init__(self, header: Optional[CBlockHeader] = None, bcp_height: int = REGTEST_BCP_HEIGHT):
        super().__init__(header, bcp_height)
        self.vtx: List[CTransaction] = []

    def deserialize(self, f, legacy: bool = False):
        super().deserialize(f, legacy)
        self.vtx = deser_vector(f, CTransaction)

    def serialize(self, legacy: bool = False, tx_count_bytes: Optional[bytes] = None) -> bytes:
        count = tx_count_bytes if tx_count_bytes is not None else ser_compact_size(len(self.vtx))
        return self.serialize_header(legacy) + count + b"".join(t.serialize() for t in self.vtx)

    def consensus_size(self) -> int:
        """Size the node's CheckBlock limits: the legacy layout before the fork, the new one after
        (reference src/validation.cpp:3267-3279)."""
        return len(self.serialize(legacy=not self.is_new_format()))

    def get_merkle_root(self, hashes: List[bytes]) -> int:
        while len(hashes) > 1:
            nxt = []
            for i in range(0, len(hashes), 2):
                j = min(i + 1, len(hashes) - 1)
                nxt.append(hash256(hashes[i] + hashes[j]))
            hashes = nxt
        return uint256_from_bytes(hashes[0]) if hashes else 0

    def calc_merkle_root(self) -> int:
        hashes = []
        for tx in self.vtx:
            tx.calc_sha256()
            hashes.append(ser_uint256(tx.sha256))
        return self.get_merkle_root(hashes)

    def is_valid_merkle(self) -> bool:
        return self.calc_merkle_root() == self.hashMerkleRoot

    def __repr__(self):
        return f"CBlock(h={self.nHeight} hash={self.hash} ntx={len(self.vtx)})"


class CBlockLocator:
    def __init__(self, have: Optional[List[int]] = None):
        self.nVersion = MY_VERSION
        self.vHave = list(have or [])

    def deserialize(self, f):
        self.nVersion = struct.unpack("<i", f.read(4))[0]
        self.vHave = deser_uint256_vector(f)

    def serialize(self) -> bytes:
        return struct.pack("<i", self.nVersion) + ser_uint256_vector(self.vHave)


class CInv:
    TYPES = {0: "Error", MSG_TX: "TX", MSG_BLOCK: "Block", MSG_FILTERED_BLOCK: "FilteredBlock",
             MSG_CMPCT_BLOCK: "CompactBlock"}

    def __init__(self, t: int = 0, h: int = 0):
        self.type = t
        self.hash = h

    def deserialize(self, f):
        self.type = struct.unpack("<i", f.read(4))[0]
        self.hash = deser_uint256(f)

    def serialize(self) -> bytes:
        return struct.pack("<i", self.type) + ser_uint256(self.hash)

    def __repr__(self):
        return f"CInv({self.TYPES.get(self.type, self.type)} {self.hash:064x})"


class CAddress:
    def __init__(self, ip: str = "0.0.0.0", port: int = 0, services: int = NODE_NETWORK):
        self.nTime = int(time.time())
        self.nServices = services
        self.ip = ip
        self.port = port

    def deserialize(self, f, with_time: bool = True):
        if with_time:
            self.nTime = struct.unpack("<I", f.read(4))[0]
        self.nServices = struct.unpack("<Q", f.read(8))[0]
        raw = f.read(16)
        self.ip = ".".join(str(b) for b in raw[12:]) if raw[:12] == b"\0" * 10 + b"\xff\xff" else raw.hex()
        self.port = struct.unpack(">H", f.read(2))[0]

    def serialize(self, with_time: bool = True) -> bytes:
        r = struct.pack("<I", self.nTime) if with_time else b""
        r += struct.pack("<Q", self.nServices)
        r += b"\0" * 10 + b"\xff\xff" + bytes(int(x) for x in self.ip.split("."))
        return r + struct.pack(">H", self.port)


# ------------------------------------------------------------------ BIP152 compact blocks

def siphash24(k0: int, k1: int, data: bytes) -> int:
    """SipHash-2-4 (reference src/hash.cpp CSipHasher) over arbitrary bytes."""
    M = 0xFFFFFFFFFFFFFFFF

    def rotl(x, b):
        return ((x << b) | (x >> (64 - b))) & M

    v0, v1, v2, v3 = k0 ^ 0x736F6D6570736575, k1 ^ 0x646F72616E646F6D, k0 ^ 0x6C7967656E657261, k1 ^ 0x7465646279746573

    def rnd(v0, v1, v2, v3):
        v0 = (v0 + v1) & M; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32)
        v2 = (v2 + v3) & M; v3 = rotl(v3, 16); v3 ^= v2
        v0 = (v0 + v3) & M; v3 = rotl(v3, 21); v3 ^= v0
        v2 = (v2 + v1) & M; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32)
        return v0, v1, v2, v3

    n = len(data)
    tail = data[n - n % 8:]
    for i in range(0, n - n % 8, 8):
        m = struct.unpack("<Q", data[i:i + 8])[0]
        v3 ^= m
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0 ^= m
    b = (n & 0xFF) << 56
    for i, c in enumerate(tail):
        b |= c << (8 * i)
    v3 ^= b
    v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    v0 ^= b
    v2 ^= 0xFF
    for _ in range(4):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    return v0 ^ v1 ^ v2 ^ v3


class PrefilledTransaction:
    def __init__(self, index: int = 0, tx: Optional[CTransaction] = None):
        self.index = index
        self.tx = tx

    def deserialize(self, f):
        self.index = deser_compact_size(f)
        self.tx = CTransaction()
        self.tx.deserialize(f)

    def serialize(self) -> bytes:
        return ser_compact_size(self.index) + self.tx.serialize()


class HeaderAndShortIDs:
    """cmpctblock payload. Prefilled indexes are differentially encoded on the wire; this
    object holds absolute indexes. Short-id keys come from SHA256(new-format header || nonce)
    whatever the peer's header format (src/blockencodings.cpp FillShortTxIDSelector)."""

    def __init__(self):
        self.header = CBlockHeader()
        self.nonce = 0
        self.shortids: List[int] = []
        self.prefilled_txn: List[PrefilledTransaction] = []

    def deserialize(self, f, legacy: bool = False):
        self.header = CBlockHeader()
        self.header.deserialize(f, legacy)
        self.nonce = struct.unpack("<Q", f.read(8))[0]
        n = deser_compact_size(f)
        self.shortids = [int.from_bytes(f.read(6), "little") for _ in range(n)]
        pre = deser_vector(f, PrefilledTransaction)
        last = -1
        for p in pre:
            p.index = last + 1 + p.index
            last = p.index
        self.prefilled_txn = pre

    def serialize(self, legacy: bool = False) -> bytes:
        r = self.header.serialize_header(legacy) + struct.pack("<Q", self.nonce)
        r += ser_compact_size(len(self.shortids)) + b"".join(s.to_bytes(6, "little") for s in self.shortids)
        r += ser_compact_size(len(self.prefilled_txn))
        last = -1
        for p in self.prefilled_txn:
            r += ser_compact_size(p.index - last - 1) + p.tx.serialize()
            last = p.index
        return r

    def keys(self):
        h = sha256(self.header.serialize_header(legacy=False) + struct.pack("<Q", self.nonce))
        return struct.unpack("<QQ", h[:16])

    def short_id(self, txid: int) -> int:
        k0, k1 = self.keys()
        return siphash24(k0, k1, ser_uint256(txid)) & 0xFFFFFFFFFFFF

    def initialize_from_block(self, block: CBlock, nonce: int = 0, prefill_list=(0,)):
        self.header = CBlockHeader(block)
        self.nonce = nonce
        self.prefilled_txn = [PrefilledTransaction(i, block.vtx[i]) for i in prefill_list]
        self.shortids = []
        for i, tx in enumerate(block.vtx):
            if i not in prefill_list:
                self.shortids.append(self.short_id(tx.calc_sha256()))


class BlockTransactionsRequest:
    def __init__(self, blockhash: int = 0, indexes: Optional[List[int]] = None):
        self.blockhash = blockhash
        self.indexes = list(indexes or [])

    def deserialize(self, f):
        self.blockhash = deser_uint256(f)
        n = deser_compact_size(f)
        last = -1
        self.indexes = []
        for _ in range(n):
            last = last + 1 + deser_compact_size(f)
            self.indexes.append(last)

    def serialize(self) -> bytes:
        r = ser_uint256(self.blockhash) + ser_compact_size(len(self.indexes))
        last = -1
        for i in self.indexes:
            r += ser_compact_size(i - last - 1)
            last = i
        return r


class BlockTransactions:
    def __init__(self, blockhash: int = 0, transactions: Optional[List[CTransaction]] = None):
        self.blockhash = blockhash
        self.transactions = list(transactions or [])

    def deserialize(self, f):
        self.blockhash = deser_uint256(f)
        self.transactions = deser_vector(f, CTransaction)

    def serialize(self) -> bytes:
        return ser_uint256(self.blockhash) + ser_vector(self.transactions)


# ------------------------------------------------------------------ BIP37

class CBloomFilter:
    """BIP37 filter (MurmurHash3 seeds nHashNum * 0xFBA4C795 + nTweak)."""

    def __init__(self, nelements: int = 10, fp: float = 0.0001, tweak: int = 0, flags: int = 1):
        import math
        size = int(min(-1 / (math.log(2) ** 2) * nelements * math.log(fp), 36000 * 8) / 8) or 1
        self.data = bytearray(size)
        self.nHashFuncs = int(min(len(self.data) * 8 / nelements * math.log(2), 50)) or 1
        self.nTweak = tweak
        self.nFlags = flags

    @staticmethod
    def murmur3(seed: int, data: bytes) -> int:
        M = 0xFFFFFFFF
        c1, c2 = 0xCC9E2D51, 0x1B873593
        h = seed & M
        n = len(data) // 4 * 4
        for i in range(0, n, 4):
            k = struct.unpack("<I", data[i:i + 4])[0]
            k = (k * c1) & M
            k = ((k << 15) | (k >> 17)) & M
            k = (k * c2) & M
            h ^= k
            h = ((h << 13) | (h >> 19)) & M
            h = (h * 5 + 0xE6546B64) & M
        k = 0
        tail = data[n:]
        for i, c in enumerate(tail):
            k |= c << (8 * i)
        if tail:
            k = (k * c1) & M
            k = ((k << 15) | (k >> 17)) & M
            k = (k * c2) & M
            h ^= k
        h ^= len(data)
        h ^= h >> 16
        h = (h * 0x85EBCA6B) & M
        h ^= h >> 13
        h = (h * 0xC2B2AE35) & M
        h ^= h >> 16
        return h

    def insert(self, key: bytes):
        for i in range(self.nHashFuncs):
            bit = self.murmur3((i * 0xFBA4C795 + self.nTweak) & 0xFFFFFFFF, key) % (len(self.data) * 8)
            self.data[bit >> 3] |= 1 << (bit & 7)

    def serialize(self) -> bytes:
        return ser_string(bytes(self.data)) + struct.pack("<IIB", self.nHashFuncs, self.nTweak, self.nFlags)


class CMerkleBlock:
    def __init__(self):
        self.header = CBlockHeader()
        self.nTransactions = 0
        self.vHash: List[int] = []
        self.vBits: List[bool] = []

    def deserialize(self, f, legacy: bool = False):
        self.header = CBlockHeader()
        self.header.deserialize(f, legacy)
        self.nTransactions = struct.unpack("<I", f.read(4))[0]
        self.vHash = deser_uint256_vector(f)
        raw = deser_string(f)
        self.vBits = [bool(raw[i // 8] >> (i % 8) & 1) for i in range(len(raw) * 8)]

    def matched_txids(self) -> List[int]:
        """Walk the partial merkle tree (reference src/merkleblock.cpp TraverseAndExtract)."""
        height = 0
        while (self.nTransactions + (1 << height) - 1) >> height > 1:
            height += 1
        bits, hashes, out = iter(self.vBits), iter(self.vHash), []

        def width(h):
            return (self.nTransactions + (1 << h) - 1) >> h

        def walk(h, pos):
            parent = next(bits)
            if h == 0 or not parent:
                x = next(hashes)
                if h == 0 and parent:
                    out.append(x)
                return x
            left = walk(h - 1, pos * 2)
            right = walk(h - 1, pos * 2 + 1) if pos * 2 + 1 < width(h - 1) else left
            return uint256_from_bytes(hash256(ser_uint256(left) + ser_uint256(right)))

        walk(height, 0)
        return out


# ------------------------------------------------------------------ messages

class Msg:
    command = b""
    block_format = False  # True: (de)serialization depends on the connection's header format

    def serialize(self, legacy: bool = False) -> bytes:
        return b""

    def deserialize(self, f, legacy: bool = False):
        pass

    def __repr__(self):
        return f"msg_{self.command.decode()}"


class msg_version(Msg):
    command = b"version"

    def __init__(self, version: int = MY_VERSION):
        self.nVersion = version
        self.nServices = NODE_NETWORK
        self.nTime = int(time.time())
        self.addrTo = CAddress()
        self.addrFrom = CAddress()
        self.nNonce = random.getrandbits(64)
        self.strSubVer = MY_SUBVERSION
        self.nStartingHeight = -1
        self.nRelay = 1

    def deserialize(self, f, legacy=False):
        self.nVersion = struct.unpack("<i", f.read(4))[0]
        self.nServices = struct.unpack("<Q", f.read(8))[0]
        self.nTime = struct.unpack("<q", f.read(8))[0]
        self.addrTo = CAddress()
        self.addrTo.deserialize(f, with_time=False)
        self.addrFrom = CAddress()
        self.addrFrom.deserialize(f, with_time=False)
        self.nNonce = struct.unpack("<Q", f.read(8))[0]
        self.strSubVer = deser_string(f)
        self.nStartingHeight = struct.unpack("<i", f.read(4))[0]
        rest = f.read(1)
        self.nRelay = rest[0] if rest else 1

    def serialize(self, legacy=False):
        return (struct.pack("<iQq", self.nVersion, self.nServices, self.nTime) +
                self.addrTo.serialize(with_time=False) + self.addrFrom.serialize(with_time=False) +
                struct.pack("<Q", self.nNonce) + ser_string(self.strSubVer) +
                struct.pack("<iB", self.nStartingHeight, self.nRelay))


class msg_verack(Msg):
    command = b"verack"


class msg_sendheaders(Msg):
    command = b"sendheaders"


class msg_getaddr(Msg):
    command = b"getaddr"


class msg_mempool(Msg):
    command = b"mempool"


class msg_filterclear(Msg):
    command = b"filterclear"


class _nonce_msg(Msg):
    def __init__(self, nonce: int = 0):
        self.nonce = nonce

    def deserialize(self, f, legacy=False):
        self.nonce = struct.unpack("<Q", f.read(8))[0]

    def serialize(self, legacy=False):
        return struct.pack("<Q", self.nonce)


class msg_ping(_nonce_msg):
    command = b"ping"


class msg_pong(_nonce_msg):
    command = b"pong"


class _inv_msg(Msg):
    def __init__(self, inv: Optional[List[CInv]] = None):
        self.inv = list(inv or [])

    def deserialize(self, f, legacy=False):
        self.inv = deser_vector(f, CInv)

    def serialize(self, legacy=False):
        return ser_vector(self.inv)


class msg_inv(_inv_msg):
    command = b"inv"


class msg_getdata(_inv_msg):
    command = b"getdata"


class msg_notfound(_inv_msg):
    command = b"notfound"


class msg_addr(Msg):
    command = b"addr"

    def __init__(self):
        self.addrs: List[CAddress] = []

    def deserialize(self, f, legacy=False):
        self.addrs = deser_vector(f, CAddress)

    def serialize(self, legacy=False):
        return ser_vector(self.addrs)


class _locator_msg(Msg):
    def __init__(self, have: Optional[List[int]] = None, hashstop: int = 0):
        self.locator = CBlockLocator(have)
        self.hashstop = hashstop

    def deserialize(self, f, legacy=False):
        self.locator = CBlockLocator()
        self.locator.deserialize(f)
        self.hashstop = deser_uint256(f)

    def serialize(self, legacy=False):
        return self.locator.serialize() + ser_uint256(self.hashstop)


class msg_getheaders(_locator_msg):
    command = b"getheaders"


class msg_getblocks(_locator_msg):
    command = b"getblocks"


class msg_headers(Msg):
    command = b"headers"
    block_format = True

    def __init__(self, headers: Optional[List[CBlockHeader]] = None):
        self.headers = list(headers or [])

    def deserialize(self, f, legacy=False):
        self.headers = []
        for _ in range(deser_compact_size(f)):
            h = CBlockHeader()
            h.deserialize(f, legacy)
            deser_compact_size(f)  # tx count (0)
            self.headers.append(h)

    def serialize(self, legacy=False):
        return ser_compact_size(len(self.headers)) + b"".join(
            h.serialize_header(legacy) + b"\x00" for h in self.headers)


class msg_block(Msg):
    command = b"block"
    block_format = True

    def __init__(self, block: Optional[CBlock] = None, raw: Optional[bytes] = None):
        self.block = block or CBlock()
        self.raw = raw  # pre-serialized payload (non-canonical encodings)

    def deserialize(self, f, legacy=False):
        self.block = CBlock()
        self.block.deserialize(f, legacy)

    def serialize(self, legacy=False):
        return self.raw if self.raw is not None else self.block.serialize(legacy)


class msg_tx(Msg):
    command = b"tx"

    def __init__(self, tx: Optional[CTransaction] = None):
        self.tx = tx or CTransaction()

    def deserialize(self, f, legacy=False):
        self.tx = CTransaction()
        self.tx.deserialize(f)

    def serialize(self, legacy=False):
        return self.tx.serialize()


class msg_reject(Msg):
    command = b"reject"
    REJECT_MALFORMED = 1
    REJECT_INVALID = 16
    REJECT_OBSOLETE = 17
    REJECT_DUPLICATE = 18
    REJECT_NONSTANDARD = 64
    REJECT_INSUFFICIENTFEE = 66

    def __init__(self, message: bytes = b"", code: int = 0, reason: bytes = b"", data: int = 0):
        self.message = message
        self.code = code
        self.reason = reason
        self.data = data

    def deserialize(self, f, legacy=False):
        self.message = deser_string(f)
        self.code = f.read(1)[0]
        self.reason = deser_string(f)
        rest = f.read(32)
        self.data = uint256_from_bytes(rest) if len(rest) == 32 else 0

    def serialize(self, legacy=False):
        r = ser_string(self.message) + bytes([self.code]) + ser_string(self.reason)
        if self.message in (b"block", b"tx"):
            r += ser_uint256(self.data)
        return r

    def __repr__(self):
        return f"msg_reject({self.message!r}, {self.code}, {self.reason!r}, {self.data:064x})"


class msg_feefilter(Msg):
    command = b"feefilter"

    def __init__(self, feerate: int = 0):
        self.feerate = feerate

    def deserialize(self, f, legacy=False):
        self.feerate = struct.unpack("<q", f.read(8))[0]

    def serialize(self, legacy=False):
        return struct.pack("<q", self.feerate)


class msg_sendcmpct(Msg):
    command = b"sendcmpct"

    def __init__(self, announce: bool = False, version: int = 1):
        self.announce = announce
        self.version = version

    def deserialize(self, f, legacy=False):
        self.announce = bool(f.read(1)[0])
        self.version = struct.unpack("<Q", f.read(8))[0]

    def serialize(self, legacy=False):
        return bytes([1 if self.announce else 0]) + struct.pack("<Q", self.version)


class msg_cmpctblock(Msg):
    command = b"cmpctblock"
    block_format = True

    def __init__(self, header_and_shortids: Optional[HeaderAndShortIDs] = None):
        self.header_and_shortids = header_and_shortids or HeaderAndShortIDs()

    def deserialize(self, f, legacy=False):
        self.header_and_shortids = HeaderAndShortIDs()
        self.header_and_shortids.deserialize(f, legacy)

    def serialize(self, legacy=False):
        return self.header_and_shortids.serialize(legacy)


class msg_getblocktxn(Msg):
    command = b"getblocktxn"

    def __init__(self, req: Optional[BlockTransactionsRequest] = None):
        self.block_txn_request = req or BlockTransactionsRequest()

    def deserialize(self, f, legacy=False):
        self.block_txn_request = BlockTransactionsRequest()
        self.block_txn_request.deserialize(f)

    def serialize(self, legacy=False):
        return self.block_txn_request.serialize()


class msg_blocktxn(Msg):
    command = b"blocktxn"

    def __init__(self, txs: Optional[BlockTransactions] = None):
        self.block_transactions = txs or BlockTransactions()

    def deserialize(self, f, legacy=False):
        self.block_transactions = BlockTransactions()
        self.block_transactions.deserialize(f)

    def serialize(self, legacy=False):
        return self.block_transactions.serialize()


class msg_filterload(Msg):
    command = b"filterload"

    def __init__(self, flt: Optional[CBloomFilter] = None):
        self.filter = flt or CBloomFilter()

    def serialize(self, legacy=False):
        return self.filter.serialize()


class msg_filteradd(Msg):
    command = b"filteradd"

    def __init__(self, data: bytes = b""):
        self.data = data

    def serialize(self, legacy=False):
        return ser_string(self.data)


class msg_merkleblock(Msg):
    command = b"merkleblock"
    block_format = True

    def __init__(self):
        self.merkleblock = CMerkleBlock()

    def deserialize(self, f, legacy=False):
        self.merkleblock = CMerkleBlock()
        self.merkleblock.deserialize(f, legacy)


MESSAGE_MAP = {m.command: m for m in [
    msg_version, msg_verack, msg_sendheaders, msg_getaddr, msg_mempool, msg_filterclear, msg_ping, msg_pong,
    msg_inv, msg_getdata, msg_notfound, msg_addr, msg_getheaders, msg_getblocks, msg_headers, msg_block, msg_tx,
    msg_reject, msg_feefilter, msg_sendcmpct, msg_cmpctblock, msg_getblocktxn, msg_blocktxn, msg_filterload,
    msg_filteradd, msg_merkleblock]}
