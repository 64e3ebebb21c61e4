"""Batched ECDSA verification (CPU pool and MI355X kernel csrc/kernels/secp256k1.hip)
against CPubKey::Verify semantics (reference src/pubkey.cpp:170-193): valid, wrong
message, wrong key, high-S (normalised -> valid), malformed DER, invalid pubkeys,
uncompressed/hybrid keys, edge r values."""
import hashlib
import random

import pytest

from bitcoincashplus_amd.utils import secp256k1_ref as ref


def make_items(native, n, seed=7):
    rng = random.Random(seed)
    items, expect = [], []
    for i in range(n):
        sec = rng.randbytes(32)
        msg = hashlib.sha256(rng.randbytes(8)).digest()
        comp = (i % 5) != 0
        pub = native.ec_pubkey_create(sec, comp)
        sig = native.ec_sign(sec, msg)
        kind = i % 11
        if kind == 1:  # wrong message
            msg = bytes([msg[0] ^ 0x80]) + msg[1:]
            ok = False
        elif kind == 2:  # wrong key
            pub = native.ec_pubkey_create(rng.randbytes(32), True)
            ok = False
        elif kind == 3:  # high-S: CPubKey::Verify normalises -> valid
            r = int.from_bytes(sig[4:4 + sig[3]], "big")
            off = 4 + sig[3]
            s = int.from_bytes(sig[off + 2:off + 2 + sig[off + 1]], "big")
            sig = ref.der_encode(r, ref.N - s)
            ok = True
        elif kind == 4:  # garbage signature
            sig = b"\x30\x02\x01\x01"
            ok = False
        elif kind == 5:  # x not on curve
            pub = b"\x02" + b"\x05" * 32 if ref.parse_pubkey(b"\x02" + b"\x05" * 32) is None else b"\x03" + b"\xff" * 32
            ok = False
        elif kind == 6 and not comp:  # hybrid encoding of an uncompressed key
            pub = bytes([6 + (pub[64] & 1)]) + pub[1:]
            ok = True
        else:
            ok = True
        items.append((pub, sig, msg))
        expect.append(ok)
    return items, expect


PATHS = {"fused": (1 << 40, None), "split8": (0, 0), "split10": (0, 2), "split10h": (0, 3)}


def pin_path(native, name):
    """Pins one GPU path: the fused latency kernel (every batch size) or the prep + verify
    throughput kernels (never fused) with the 8 x 32, the one-lane 10 x 26 or the half-lane
    10 x 26 verify kernel. Returns the previous settings for unpin_path."""
    old = (native.ecdsa_fused_max(), native.ecdsa_split_kernel())
    fmax, sk = PATHS[name]
    native.ecdsa_set_fused_max(fmax)
    if sk is not None:
        native.ecdsa_set_split_kernel(sk)
    return old


def unpin_path(native, old):
    native.ecdsa_set_fused_max(old[0])
    native.ecdsa_set_split_kernel(old[1])


@pytest.fixture(params=list(PATHS))
def ecdsa_path(request, native):
    old = pin_path(native, request.param)
    yield request.param
    unpin_path(native, old)


def test_cpu_batch(native):
    items, expect = make_items(native, 64)
    res, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    assert res == expect


@pytest.mark.gpu
def test_gpu_batch_matches_cpu(native, ecdsa_path):
    items, expect = make_items(native, 300)
    res, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    cpu, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    assert cpu == expect
    assert res == expect


@pytest.mark.gpu
def test_gpu_batch_edge_scalars(native, ecdsa_path):
    # small private keys / messages exercise short wNAF and sparse comb windows
    items = []
    for k in (1, 2, 3, 255, 256, 2**64 + 1):
        sec = k.to_bytes(32, "big")
        for m in (b"\x00" * 31 + b"\x01", b"\xff" * 32, hashlib.sha256(bytes([k % 256])).digest()):
            items.append((native.ec_pubkey_create(sec, True), native.ec_sign(sec, m), m))
    res, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    assert all(res)


def _edge_scalar_items(native):
    """DER signatures whose r or s sit on the scalar-range boundaries (0, 1, n-1, n, n+1,
    2^256-1) plus message hashes >= n. The lax-DER parse on the host and the range checks and
    z reduction in ecdsa_prep_kernel must agree with CPubKey::Verify on every one."""
    n = ref.N
    sec = (0x1234567 * 0x9E3779B97F4A7C15).to_bytes(32, "big")
    pub = native.ec_pubkey_create(sec, True)
    msgs = [b"\xff" * 32, n.to_bytes(32, "big"), (n + 5).to_bytes(32, "big"), b"\x00" * 32,
            hashlib.sha256(b"edge").digest()]
    edges = [0, 1, n - 1, n, n + 1, 2**256 - 1]
    items = []
    for m in msgs:
        good = native.ec_sign(sec, m)
        items.append((pub, good, m))  # valid, with z >= n for the first three messages
        rlen = good[3]
        r_good = int.from_bytes(good[4:4 + rlen], "big")
        off = 4 + rlen
        s_good = int.from_bytes(good[off + 2:off + 2 + good[off + 1]], "big")
        for e in edges:
            items.append((pub, ref.der_encode(e, s_good), m))
            items.append((pub, ref.der_encode(r_good, e), m))
        items.append((pub, ref.der_encode(r_good, n - s_good), m))  # high-S twin: normalised, valid
        if r_good + n < 2**256:
            items.append((pub, ref.der_encode(r_good + n, s_good), m))  # x(R)+n form of r: out of range
    return items


def test_cpu_edge_scalars(native):
    items = _edge_scalar_items(native)
    res, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    # the valid signature and its high-S twin verify for every message; nothing else does
    assert sum(res) == 2 * 5


@pytest.mark.gpu
def test_gpu_edge_scalars_match_cpu(native, ecdsa_path):
    items = _edge_scalar_items(native)
    cpu, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    gpu, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    assert gpu == cpu


def _cancelling_items(native):
    """Signatures whose R = u1*G + u2*Q is the point at infinity or whose partial sums cancel:
    with Q = G (secret 1) and z = n - r, u1 + u2 = (z + r)/s = 0 (mod n). They must verify false
    on every path (the GPU's final additions hit H = 0 with R != 0 and return infinity)."""
    n = ref.N
    pub = native.ec_pubkey_create((1).to_bytes(32, "big"), True)
    rng = random.Random(11)
    items = []
    for _ in range(6):
        r = rng.randrange(1, n)
        s = rng.randrange(1, n // 2)
        items.append((pub, ref.der_encode(r, s), (n - r).to_bytes(32, "big")))
    # and a valid signature by the same key, so the batch is not all-false
    m = hashlib.sha256(b"cancel").digest()
    items.append((pub, native.ec_sign((1).to_bytes(32, "big"), m), m))
    return items


def test_cpu_cancelling(native):
    res, _ = native.ecdsa_verify_batch(_cancelling_items(native), use_gpu=False)
    assert res == [False] * 6 + [True]


@pytest.mark.gpu
def test_gpu_cancelling_match_cpu(native, ecdsa_path):
    items = _cancelling_items(native)
    gpu, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    assert gpu == [False] * 6 + [True]


@pytest.mark.gpu
def test_gpu_fused_partial_workgroups(native):
    """The fused kernel runs 64 signatures per workgroup, the verify kernels 128: batch sizes
    around those boundaries (and a multi-workgroup batch) on every path against the expected
    verdicts."""
    items, expect = make_items(native, 1100, seed=3)
    for n in (1, 63, 64, 65, 127, 129, 1100):
        for name in PATHS:
            old = pin_path(native, name)
            try:
                got, _ = native.ecdsa_verify_batch(items[:n], use_gpu=True)
            finally:
                unpin_path(native, old)
            assert got == expect[:n], (n, name)


@pytest.mark.gpu
def test_gpu_split10_rounds_and_tail(native):
    """The 10 x 26 split path gives whole device rounds (one wave per SIMD: CUs x 256
    signatures) to the one-lane kernel and a last round at most half full to the half-lane
    kernel: a batch of one round plus 1000 takes both kernels (on 256 CUs), and every path
    agrees with the expected verdicts."""
    items, expect = make_items(native, 1100, seed=5)
    n = 65536 + 1000
    reps = n // len(items) + 1
    big, want = (items * reps)[:n], (expect * reps)[:n]
    for name, sk in (("auto", 1), ("split8", 0)):
        old = (native.ecdsa_fused_max(), native.ecdsa_split_kernel())
        native.ecdsa_set_fused_max(0)
        native.ecdsa_set_split_kernel(sk)
        try:
            got, _ = native.ecdsa_verify_batch(big, use_gpu=True, threads=16)
        finally:
            unpin_path(native, old)
        bad = [i for i in range(n) if got[i] != want[i]]
        assert not bad, (name, bad[:10])
