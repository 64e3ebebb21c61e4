"""BIP152 short transaction ids on the GPU (K9, csrc/kernels/relay.hip) against the CPU
SipHashUint256 (reference src/hash.cpp:181-300, src/blockencodings.cpp:37-42): 48-bit ids of
random txids under random keys, including all-zero / all-ones txids and keys, must be identical."""
import random

import pytest

MASK = (1 << 48) - 1


@pytest.mark.gpu
def test_short_ids_match_cpu(native):
    rng = random.Random(3)
    for n, (k0, k1) in [(1, (0, 0)), (257, (2**64 - 1, 2**64 - 1)), (100_000, (rng.getrandbits(64), rng.getrandbits(64)))]:
        txids = [bytes(32), b"\xff" * 32] + [rng.randbytes(32) for _ in range(max(0, n - 2))]
        txids = txids[:n]
        got = native.short_txid_batch_gpu(k0, k1, b"".join(txids))
        assert len(got) == n
        for t, g in zip(txids, got):
            assert g == native.siphash_uint256(k0, k1, t) & MASK


@pytest.mark.gpu
def test_short_ids_reject_ragged_input(native):
    with pytest.raises(Exception):
        native.short_txid_batch_gpu(1, 2, b"\x00" * 33)


@pytest.mark.gpu
def test_ops_facade_short_ids(native):
    from bitcoincashplus_amd import ops
    rng = random.Random(9)
    txids = [rng.randbytes(32) for _ in range(64)]
    assert ops.short_txids(5, 6, txids) == [native.siphash_uint256(5, 6, t) & MASK for t in txids]
