"""Device FORKID signature hashes (K7) and the fused digest -> verify batch.

The recipe (csrc/script/sighash_recipe.cpp) and the kernel (csrc/kernels/sighash_device.h) must
give exactly the digest of SignatureHash (reference src/script/interpreter.cpp:1354-1404) for
every hash type: ALL / NONE / SINGLE with and without ANYONECANPAY, SINGLE past the last output,
legacy (non-FORKID) digests, and script codes whose length prefix takes 1, 3 and 5 bytes. The
transactions are the reference's sighash.json vectors (vendored), re-used with FORKID hash types.
A digest mismatch would be a consensus split, so every comparison is exact.
"""
import json
import os
import random

import pytest

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "vectors", "sighash.json")
FORKID_TYPES = [0x41, 0x42, 0x43, 0xC1, 0xC2, 0xC3, 0x40, 0x44, 0x5F, 0xE1]


def _vectors():
    with open(DATA) as f:
        return [v for v in json.load(f) if len(v) == 5]


def _items(n_long=True, seed=11):
    rng = random.Random(seed)
    items = []
    for raw, script, n_in, ht, _ in _vectors()[:400]:
        tx = bytes.fromhex(raw)
        code = bytes.fromhex(script)
        h = rng.choice(FORKID_TYPES) if rng.random() < 0.85 else ht & 0xFF  # some legacy digests
        items.append((code, tx, n_in, h, rng.randrange(0, 21_000_000 * 10**8)))
    if n_long:
        raw, _, n_in, _, _ = _vectors()[5]
        tx = bytes.fromhex(raw)
        for ln in (31, 32, 252, 253, 300, 65535, 65536, 70000):
            items.append((bytes(rng.randrange(256) for _ in range(ln)), tx, n_in, 0x41, 5000))
    return items


def _expected(native, items):
    return [native.signature_hash(c, tx, i, h, a) for c, tx, i, h, a in items]


def test_recipe_cpu_matches_signature_hash(native):
    items = _items()
    got = native.sighash_recipes(items, use_gpu=False)
    exp = _expected(native, items)
    assert [g[0] for g in got] == exp
    used = [g[1] for g in got]
    # the recipe covers the FORKID digests except SIGHASH_SINGLE with a matching output
    assert sum(used) > len(items) // 2 and not all(used)


@pytest.mark.gpu
def test_recipe_gpu_matches_signature_hash(native):
    items = _items()
    got = native.sighash_recipes(items, use_gpu=True)
    assert [g[0] for g in got] == _expected(native, items)


def _signed_checks(native, n, seed=5):
    """(pubkey, sig||hashtype, script_code, tx, n_in, amount) checks with known validity."""
    rng = random.Random(seed)
    vec = _vectors()
    checks, expect = [], []
    for k in range(n):
        raw, _, n_in, _, _ = vec[k % 300]
        tx = bytes.fromhex(raw)
        sec = rng.randbytes(32)
        pub = native.ec_pubkey_create(sec, k % 4 != 0)
        code = b"\x76\xa9\x14" + rng.randbytes(20) + b"\x88\xac"  # P2PKH script code (25 bytes)
        if k % 7 == 3:
            code = rng.randbytes(40)  # too long for a recipe: digest computed on the CPU
        ht = rng.choice([0x41, 0x42, 0x43, 0xC1, 0xC3])
        amount = rng.randrange(1, 10**12)
        digest = native.signature_hash(code, tx, n_in, ht, amount)
        sig = native.ec_sign(sec, digest) + bytes([ht])
        ok = True
        kind = k % 5
        if kind == 1:
            amount += 1  # signs a different amount
            ok = False
        elif kind == 2:
            pub = native.ec_pubkey_create(rng.randbytes(32), True)
            ok = False
        checks.append((pub, sig, code, tx, n_in, amount))
        expect.append(ok)
    return checks, expect


def test_deferred_recipes_cpu(native):
    checks, expect = _signed_checks(native, 120)
    res, dig, rec = native.verify_sig_recipes(checks, use_gpu=False, recipes=True)
    assert list(res) == expect
    assert any(rec) and not all(rec)
    for (pub, sig, code, tx, n_in, amount), d in zip(checks, dig):
        assert d == native.signature_hash(code, tx, n_in, sig[-1], amount)
    # recipes off: identical verdicts and digests, no recipe checks
    res2, dig2, rec2 = native.verify_sig_recipes(checks, use_gpu=False, recipes=False)
    assert list(res2) == expect and list(dig2) == list(dig) and not any(rec2)


@pytest.mark.gpu
def test_fused_sighash_verify_gpu(native):
    checks, expect = _signed_checks(native, 1500)
    res, dig, rec = native.verify_sig_recipes(checks, use_gpu=True, recipes=True)
    assert list(res) == expect
    assert any(rec) and not all(rec)  # mixed batch: recipe and PRECOMPUTED jobs
    cres, cdig, _ = native.verify_sig_recipes(checks, use_gpu=False, recipes=True)
    assert list(dig) == list(cdig) and list(res) == list(cres)
