"""Pure-Python Equihash oracle (hashlib BLAKE2b) used to cross-check the C++/HIP code.

It follows the reference's byte-level formulation (src/crypto/equihash.cpp):
ExpandArray to CollisionByteLength-wide big-endian digits, collision on the
next CollisionByteLength bytes, lexicographic index-list ordering,
distinct indices and an all-zero final hash.  Deliberately slow and simple.
"""
from __future__ import annotations

import hashlib
import struct
from typing import List


def personal(n: int, k: int) -> bytes:
    return b"ZcashPoW" + struct.pack("<II", n, k)


def hash_output_len(n: int) -> int:
    return (512 // n) * n // 8


def base_hasher(n: int, k: int, data: bytes):
    h = hashlib.blake2b(digest_size=hash_output_len(n), person=personal(n, k))
    h.update(data)
    return h


def generate_hash(base, g: int) -> bytes:
    h = base.copy()
    h.update(struct.pack("<I", g))
    return h.digest()


def expand_array(inp: bytes, bit_len: int, byte_pad: int = 0) -> bytes:
    out_width = (bit_len + 7) // 8 + byte_pad
    bits = int.from_bytes(inp, "big")
    total = len(inp) * 8
    groups = total // bit_len
    out = bytearray()
    for g in range(groups):
        v = (bits >> (total - (g + 1) * bit_len)) & ((1 << bit_len) - 1)
        out += bytes(byte_pad) + v.to_bytes(out_width - byte_pad, "big")
    return bytes(out)


def indices_from_minimal(minimal: bytes, cbl: int) -> List[int]:
    nb = cbl + 1
    v = int.from_bytes(minimal, "big")
    total = len(minimal) * 8
    cnt = total // nb
    return [(v >> (total - (i + 1) * nb)) & ((1 << nb) - 1) for i in range(cnt)]


def minimal_from_indices(indices: List[int], cbl: int) -> bytes:
    nb = cbl + 1
    v = 0
    for i in indices:
        v = (v << nb) | i
    return v.to_bytes(len(indices) * nb // 8, "big")


def is_valid_solution(n: int, k: int, data: bytes, soln: bytes) -> bool:
    cbl = n // (k + 1)
    cbytes = (cbl + 7) // 8
    iph = 512 // n
    if len(soln) != (1 << k) * (cbl + 1) // 8:
        return False
    base = base_hasher(n, k, data)
    rows = []
    for i in indices_from_minimal(soln, cbl):
        h = generate_hash(base, i // iph)
        sl = h[(i % iph) * n // 8:(i % iph + 1) * n // 8]
        rows.append((expand_array(sl, cbl), [i]))
    while len(rows) > 1:
        nxt = []
        for a, b in zip(rows[0::2], rows[1::2]):
            ha, ia = a
            hb, ib = b
            if ha[:cbytes] != hb[:cbytes]:
                return False
            if ib < ia:  # lexicographic list comparison == reference IndicesBefore
                return False
            if set(ia) & set(ib):
                return False
            nxt.append((bytes(x ^ y for x, y in zip(ha, hb))[cbytes:], ia + ib))
        rows = nxt
    return all(c == 0 for c in rows[0][0])


def solve(n: int, k: int, data: bytes) -> List[bytes]:
    """Full-index-list Wagner solver (reference BasicSolve semantics). Small params only."""
    cbl = n // (k + 1)
    cbytes = (cbl + 7) // 8
    iph = 512 // n
    base = base_hasher(n, k, data)
    init = 1 << (cbl + 1)
    X = []
    g = 0
    while len(X) < init:
        h = generate_hash(base, g)
        for s in range(iph):
            if len(X) >= init:
                break
            X.append((expand_array(h[s * n // 8:(s + 1) * n // 8], cbl), (g * iph + s,)))
        g += 1
    for _ in range(1, k):
        X.sort(key=lambda r: r[0][:cbytes])
        nxt = []
        i = 0
        while i < len(X):
            j = i + 1
            while j < len(X) and X[j][0][:cbytes] == X[i][0][:cbytes]:
                j += 1
            for a in range(i, j):
                for b in range(a + 1, j):
                    ha, ia = X[a]
                    hb, ib = X[b]
                    if set(ia) & set(ib):
                        continue
                    x = bytes(p ^ q for p, q in zip(ha, hb))[cbytes:]
                    nxt.append((x, ia + ib if ia < ib else ib + ia))
            i = j
        X = nxt
    X.sort(key=lambda r: r[0])
    sols = set()
    i = 0
    while i < len(X):
        j = i + 1
        while j < len(X) and X[j][0] == X[i][0]:
            j += 1
        for a in range(i, j):
            for b in range(a + 1, j):
                ia, ib = X[a][1], X[b][1]
                if set(ia) & set(ib):
                    continue
                idx = ia + ib if ia < ib else ib + ia
                sols.add(minimal_from_indices(list(idx), cbl))
        i = j
    return sorted(sols)
