"""Device-side lax DER parsing (csrc/kernels/secp256k1.hip der_lax_parse, the block path's
GpuVerifyDeferred) against the CPU verifier on the same encodings.

Parity: reference src/pubkey.cpp ecdsa_signature_parse_der_lax + CPubKey::Verify (low-S
normalisation before verifying). Every variant below goes through native.ecdsa_verify_batch with
use_gpu=True and use_gpu=False and must give the same verdict; the expected verdicts pin the
lax rules themselves (long-form lengths and leading zeros accepted, oversized integers and
values >= n rejected, trailing bytes ignored).
"""
import hashlib
import random

import pytest

from bitcoincashplus_amd.utils import secp256k1_ref as ref

pytestmark = pytest.mark.gpu


def _int_bytes(v):
    b = v.to_bytes(32, "big").lstrip(b"\x00") or b"\x00"
    return b"\x00" + b if b[0] & 0x80 else b


def _der(rb, sb, total_long=False, r_long=False):
    r_part = b"\x02" + (b"\x81" + bytes([len(rb)]) if r_long else bytes([len(rb)])) + rb
    s_part = b"\x02" + bytes([len(sb)]) + sb
    body = r_part + s_part
    head = b"\x30" + (b"\x81" + bytes([len(body)]) if total_long else bytes([len(body)]))
    return head + body


def _raw(v):
    """minimal big-endian bytes without the DER sign pad (the lax parser does not need it)"""
    return v.to_bytes(32, "big").lstrip(b"\x00") or b"\x00"


def _variants(r, s):
    """(label, der, expected valid?) for a valid (r, s) with low s; every encoding fits the
    72 bytes a deferred check carries."""
    rb, sb = _int_bytes(r), _int_bytes(s)
    ru, su = _raw(r), _raw(s)
    yield "plain", _der(rb, sb), True
    yield "high_s", _der(rb, _int_bytes(ref.N - s)), True
    yield "no_sign_pad", _der(ru, su), True
    yield "long_total_len", _der(ru, su, total_long=True), True
    yield "long_r_len", _der(ru, su, r_long=True), True
    yield "extra_zero", _der(b"\x00" + ru, su), True
    yield "trailing", _der(ru, su) + b"\x01\x02", True
    yield "truncated", _der(ru, su)[:-1], False
    yield "bad_tag", b"\x31" + _der(ru, su)[1:], False
    yield "r_33_bytes", _der(b"\x01" + r.to_bytes(32, "big"), su[:30]), False
    yield "r_is_n", _der(_raw(ref.N), su), False
    yield "r_zero", _der(b"\x00", su), False
    yield "s_zero", _der(ru, b"\x00"), False
    yield "empty", b"", False
    yield "huge_len", b"\x30\x06\x02\x88" + b"\x01" * 8 + b"\x02\x01\x01", False


@pytest.mark.parametrize("path", ["fused", "split8", "split10", "split10h"])
def test_device_der_parse_matches_cpu(native, path):
    from test_ecdsa_batch import pin_path, unpin_path
    old = pin_path(native, path)
    try:
        _check_der_variants(native)
    finally:
        unpin_path(native, old)


def _check_der_variants(native):
    rng = random.Random(21)
    items, labels, expect = [], [], []
    # enough signatures for the GPU path (the batch threshold does not apply to this entry point)
    for i in range(120):
        sec = rng.randbytes(32)
        msg = hashlib.sha256(rng.randbytes(8)).digest()
        pub = native.ec_pubkey_create(sec, i % 3 != 0)
        der = native.ec_sign(sec, msg)
        r = int.from_bytes(der[4:4 + der[3]], "big")
        off = 4 + der[3]
        s = int.from_bytes(der[off + 2:off + 2 + der[off + 1]], "big")
        for label, sig, ok in _variants(r, s):
            items.append((pub, sig, msg))
            labels.append(label)
            expect.append(ok)
    gpu, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    cpu, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    bad = [(labels[i], gpu[i], cpu[i], expect[i]) for i in range(len(items)) if not (gpu[i] == cpu[i] == expect[i])]
    assert not bad, bad[:10]
