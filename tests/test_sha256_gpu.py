"""SHA-256d kernels (txid batch, 64-byte batch, merkle levels, nonce sweep) vs hashlib."""
import hashlib
import os
import struct

import pytest


def dsha(b):
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


def merkle_ref(leaves):
    """Reference MerkleComputation semantics (src/consensus/merkle.cpp:47-144), constant-space form."""
    if not leaves:
        return bytes(32), False
    mutated = False
    inner = [None] * 32
    count = 0
    for h in leaves:
        count += 1
        level = 0
        while not (count & (1 << level)):
            mutated |= inner[level] == h
            h = dsha(inner[level] + h)
            level += 1
        inner[level] = h
    level = 0
    while not (count & (1 << level)):
        level += 1
    h = inner[level]
    while count != (1 << level):
        h = dsha(h + h)
        count += 1 << level
        level += 1
        while not (count & (1 << level)):
            h = dsha(inner[level] + h)
            level += 1
    return h, mutated


@pytest.mark.gpu
def test_sha256d_batch(native):
    msgs = [os.urandom(n) for n in (0, 1, 55, 56, 63, 64, 65, 119, 120, 200, 1000, 5000)]
    out = native.sha256d_batch_gpu(msgs)
    assert [o for o in out] == [dsha(m) for m in msgs]
    blob = os.urandom(64 * 1000)
    got = native.sha256d64_batch_gpu(blob)
    for i in range(0, 1000, 97):
        assert got[32 * i:32 * i + 32] == dsha(blob[64 * i:64 * i + 64])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 100, 1000, 1024, 1025, 2047, 4097, 21001])
def test_merkle_root(native, n):
    leaves = [os.urandom(32) for _ in range(n)]
    root, mut = native.merkle_root_gpu(b"".join(leaves))
    assert (root, mut) == merkle_ref(leaves)


@pytest.mark.gpu
def test_merkle_mutation(native):
    a, b, c = (os.urandom(32) for _ in range(3))
    for leaves in ([a, b, c, c], [a, a], [a, b, a, b, c, c], [a, b, c]):
        assert native.merkle_root_gpu(b"".join(leaves)) == merkle_ref(leaves)
    # the classic CVE-2012-2459 pair has equal roots but only one is flagged
    r1, m1 = native.merkle_root_gpu(b"".join([a, b, c]))
    r2, m2 = native.merkle_root_gpu(b"".join([a, b, c, c]))
    assert r1 == r2 and not m1 and m2
    # the same in a tree deep enough to go through the wide levels and the one-workgroup tail
    big = [os.urandom(32) for _ in range(3001)]
    for leaves in (big, big + [big[-1]], big[:2048] + big[:2048]):
        assert native.merkle_root_gpu(b"".join(leaves)) == merkle_ref(leaves)


@pytest.mark.gpu
def test_nonce_scan(native):
    header = bytearray(os.urandom(80))
    target = (1 << 248) - 1  # easy: ~1/256 hashes qualify
    tgt_le = target.to_bytes(32, "little")
    nonce = native.sha256d_scan_nonces_gpu(bytes(header), tgt_le, 1000, 1 << 16)
    assert nonce >= 1000

    def h_of(n):
        header[76:80] = struct.pack("<I", n)
        return int.from_bytes(dsha(bytes(header)), "little")

    assert h_of(nonce) <= target
    for n in range(1000, nonce):
        assert h_of(n) > target
    assert native.sha256d_scan_nonces_gpu(bytes(header), bytes(32), 0, 4096) == -1
