"""Device-resident ops (bitcoincashplus_amd.ops with torch tensors on the MI355X): the kernels read
and write the tensors' device memory on the current torch stream, with no host staging.

Each op is checked against a plain CPU reference of the same computation: hashlib SHA-256d per
64-byte node, the host short-id path, and the host ECDSA path / expected validity. Reference
semantics: SHA256d nodes (src/consensus/merkle.cpp), BIP152 short ids
(src/blockencodings.cpp:37-42), CPubKey::Verify (src/pubkey.cpp:170-193).
"""
import hashlib
import random

import pytest

torch = pytest.importorskip("torch")

from bitcoincashplus_amd import ops  # noqa: E402
from bitcoincashplus_amd.utils import secp256k1_ref as ref  # noqa: E402

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    return torch.device("cuda", 0)


def test_sha256d64_device_resident():
    d = _dev()
    rng = random.Random(3)
    raw = rng.randbytes(64 * 1000)
    x = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(d)
    s = torch.cuda.Stream(d)
    with torch.cuda.stream(s):  # runs on a non-default stream, ordered after the copy there
        x2 = x.clone()
        out = ops.sha256d64(x2)
    s.synchronize()
    assert out.is_cuda and out.shape == (1000, 32)
    got = bytes(out.cpu().numpy().tobytes())
    want = b"".join(hashlib.sha256(hashlib.sha256(raw[64 * i:64 * i + 64]).digest()).digest() for i in range(1000))
    assert got == want


def test_short_txids_device_matches_host():
    d = _dev()
    rng = random.Random(5)
    n = 4096
    raw = rng.randbytes(32 * n + 8)
    k0, k1 = rng.getrandbits(64), rng.getrandbits(64)
    host = ops.short_txids(k0, k1, raw[8:])
    big = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(d)
    dev = ops.short_txids(k0, k1, big[8:])  # 8-byte offset: the op realigns it
    torch.cuda.synchronize()
    assert dev.is_cuda and dev.dtype == torch.int64
    assert [int(v) for v in dev.cpu().tolist()] == list(host)


def test_ecdsa_verify_compact_device(native):
    d = _dev()
    rng = random.Random(11)
    msgs, sigs, pubs, expect = [], [], [], []
    for i in range(700):
        sec = rng.randbytes(32)
        msg = hashlib.sha256(rng.randbytes(8)).digest()
        der = native.ec_sign(sec, msg)
        r = int.from_bytes(der[4:4 + der[3]], "big")
        off = 4 + der[3]
        s = int.from_bytes(der[off + 2:off + 2 + der[off + 1]], "big")
        if s > ref.N // 2:
            s = ref.N - s
        ok = True
        if i % 11 == 7:  # the malleated twin n - s: rejected, as libsecp256k1's verify does
            s = ref.N - s
            ok = False
        if i % 7 == 3:  # wrong message
            msg = bytes([msg[0] ^ 1]) + msg[1:]
            ok = False
        if i % 13 == 5:  # another key
            sec = rng.randbytes(32)
            ok = False
        msgs.append(msg)
        sigs.append(r.to_bytes(32, "big") + s.to_bytes(32, "big"))
        pubs.append(native.ec_pubkey_create(sec, True))
        expect.append(ok)
    m, sg, pb = (torch.frombuffer(bytearray(b"".join(v)), dtype=torch.uint8).to(d) for v in (msgs, sigs, pubs))
    res = ops.ecdsa_verify_compact(m.view(-1, 32), sg.view(-1, 64), pb.view(-1, 33))
    torch.cuda.synchronize()
    assert res.is_cuda and res.shape == (700,)
    assert [bool(v) for v in res.cpu().tolist()] == expect
    # the host path of the same op agrees
    assert list(ops.ecdsa_verify_compact(b"".join(msgs), b"".join(sigs), b"".join(pubs))) == expect
