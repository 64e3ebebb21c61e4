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


def test_cpu_batch(native):
    items, expect = make_items(native, 64)
    res, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    assert res == expect


@pytest.mark.gpu
def test_gpu_batch_matches_cpu(native):
    items, expect = make_items(native, 300)
    res, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    cpu, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    assert cpu == expect
    assert res == expect


@pytest.mark.gpu
def test_gpu_batch_edge_scalars(native):
    # small private keys / messages exercise short wNAF and sparse comb windows
    items = []
    for k in (1, 2, 3, 255, 256, 2**64 + 1):
        sec = k.to_bytes(32, "big")
        for m in (b"\x00" * 31 + b"\x01", b"\xff" * 32, hashlib.sha256(bytes([k % 256])).digest()):
            items.append((native.ec_pubkey_create(sec, True), native.ec_sign(sec, m), m))
    res, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    assert all(res)
