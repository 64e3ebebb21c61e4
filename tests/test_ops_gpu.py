"""GPU front-ends (bitcoincashplus_amd.ops / models / parallel) on the MI355X, checked
against hashlib / the native CPU implementations."""
import hashlib

import pytest

pytestmark = pytest.mark.gpu


def test_sha256d64_tensor_and_bytes():
    import torch
    from bitcoincashplus_amd import ops
    data = bytes((i * 7 + 3) & 0xFF for i in range(64 * 300))
    ref = b"".join(hashlib.sha256(hashlib.sha256(data[i:i + 64]).digest()).digest() for i in range(0, len(data), 64))
    assert ops.sha256d64(data) == ref
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).view(-1, 64)
    out = ops.sha256d64(t)
    assert out.shape == (300, 32) and bytes(out.flatten().tolist()) == ref


def test_merkle_root_matches_cpu():
    from bitcoincashplus_amd import native, ops
    leaves = [hashlib.sha256(b"%d" % i).digest() for i in range(1000)]
    root, mutated = ops.merkle_root(leaves)
    cref = native.merkle_root(leaves)
    assert root == (cref[0] if isinstance(cref, tuple) else cref) and not mutated


def test_ecdsa_ops_gpu_matches_cpu():
    from bitcoincashplus_amd import native, ops
    items = []
    for i in range(512):
        sk = hashlib.sha256(b"k%d" % i).digest()
        msg = hashlib.sha256(b"m%d" % i).digest()
        sig = native.ec_sign(sk, msg)
        if i % 7 == 0:
            msg = hashlib.sha256(b"x%d" % i).digest()
        items.append((native.ec_pubkey_create(sk), sig, msg))
    g, _ = ops.ecdsa_verify(items, use_gpu=True)
    c, _ = ops.ecdsa_verify(items, use_gpu=False)
    assert g == c and g == [i % 7 != 0 for i in range(512)]


def test_gpu_miner_single_rank():
    from bitcoincashplus_amd import models, parallel
    m = parallel.DistributedEquihashMiner(48, 5, b"\x33" * 108, batch=4, backend="gpu")
    win = m.mine(lambda nonce, sol: True, max_steps=4)
    assert win is not None
    st = models.EquihashModel(48, 5).state(b"\x33" * 108 + win[0])
    assert models.EquihashModel(48, 5).verify(st, win[1])
