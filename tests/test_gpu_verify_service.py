"""GPU verification service (csrc/node/gpuverify.{h,cpp}): node validation batches sharded
across the validation GPUs, one high-priority stream + service thread per lane.

Parity: reference src/checkqueue.h:27-164 / src/validation.cpp:2011-2127 (CCheckQueue splits a
block's checks over -par threads and AND-reduces). Here the sharded path runs with the same
device listed twice (two lanes, two streams on one GPU) so a one-GPU box exercises it, and its
verdicts must equal the CPU's item by item. The randomized differential tests feed >= 10k
mutated ECDSA triples and >= 10k mutated Equihash solutions through the GPU and the CPU
consensus code: any disagreement would be a chain split.
"""
import hashlib
import random
import struct

import pytest

from bitcoincashplus_amd import native as N
from bitcoincashplus_amd.utils import secp256k1_ref as ref

from test_ecdsa_batch import make_items


def test_service_without_gpu_fails_loudly(native):
    if native.gpu_available():
        pytest.skip("GPU visible")
    assert native.gpu_verify_devices() == []
    with pytest.raises(RuntimeError, match="no validation GPU"):
        native.gpu_verify_ecdsa_packed(b"\0" * 32, b"\0" * 64, b"\2" + b"\0" * 32)
    # the node-level batch verifier falls back to the CPU pool when the device path throws
    items, expect = make_items(native, 600)
    old = native.get_gpu_sig_threshold()
    native.set_gpu_sig_threshold(1)
    try:
        assert native.sig_batch_verify(items, use_gpu=True) == all(expect)
    finally:
        native.set_gpu_sig_threshold(old)


@pytest.fixture
def two_lanes(native):
    native.gpu_verify_set_devices([0, 0])
    native.gpu_verify_set_min_shard(64, 8)
    yield
    native.gpu_verify_set_min_shard(65536, 2048)  # the service defaults
    native.gpu_verify_set_devices([])


@pytest.mark.gpu
def test_sharded_ecdsa_matches_cpu(native, two_lanes):
    items, expect = make_items(native, 3001, seed=11)
    cpu, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    assert cpu == expect
    before = native.gpu_verify_stats()["sharded_batches"]
    gpu, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    assert gpu == cpu
    st = native.gpu_verify_stats()
    assert st["sharded_batches"] == before + 1
    lanes = st["lanes"]
    assert [l["device"] for l in lanes] == [0, 0]
    assert all(l["items"] > 0 for l in lanes)
    assert sum(l["items"] for l in lanes) >= 3001
    # both lanes run at the device's greatest (numerically lowest) stream priority
    assert lanes[0]["priority"] == lanes[1]["priority"] <= 0


@pytest.mark.gpu
def test_sharded_equihash_headers_match_cpu(native, two_lanes):
    """HEADERS-style batch: valid (48,5) and (200,9) solutions mixed with corrupted ones."""
    for n, k, nonces in [(48, 5, 48), (200, 9, 8)]:
        solver = native.EquihashGpuSolver(n, k, nonces)
        states = []
        for i in range(nonces):
            st = native.EquihashState(n, k)
            st.update(b"svc" + bytes(105) + struct.pack("<I", i) + bytes(28))
            states.append(st)
        sts, sols = [], []
        for st, ss in zip(states, solver.solve(states)):
            for s in ss:
                sts.append(st)
                sols.append(s)
                bad = bytearray(s)
                bad[len(bad) // 2] ^= 0x10
                sts.append(st)
                sols.append(bytes(bad))
        assert len(sols) >= 16
        got = native.gpu_verify_equihash(n, k, sts, sols)
        want = [native.eh_is_valid_solution(n, k, st, s)[0] for st, s in zip(sts, sols)]
        assert got == want and any(want) and not all(want)
    assert all(l["items"] > 0 for l in native.gpu_verify_stats()["lanes"])


@pytest.mark.gpu
def test_raw_header_batches_match_cpu(native, two_lanes):
    """Header batches through CheckEquihashSolutions' GPU path: the device builds each header's
    BLAKE2b base state from the raw 140 bytes (eh_state_kernel), the lanes fill their shards on
    their own workers. Valid regtest (48,5) and mainnet (200,9) headers, plus corrupted ones
    (a header field, the nonce, a solution byte, a short solution), against the CPU verdicts."""
    from test_equihash import header_input

    def compact(n):
        return bytes([n]) if n < 253 else b"\xfd" + struct.pack("<H", n)

    for n, k, chain, nonces in [(48, 5, "regtest", 40), (200, 9, "main", 6)]:
        solver = native.EquihashGpuSolver(n, k, nonces)
        datas, states = [], []
        for i in range(nonces):
            data = header_input(i, b"rawhdr%d" % n)
            st = native.EquihashState(n, k)
            st.update(data)
            datas.append(data)
            states.append(st)
        batch = []
        for data, ss in zip(datas, solver.solve(states)):
            for s in ss[:2]:
                batch.append(data + compact(len(s)) + s)
        assert len(batch) >= 8
        rng = random.Random(n)
        for h in list(batch[:6]):
            b = bytearray(h)
            which = rng.randrange(4)
            if which == 0:
                b[rng.randrange(4, 108)] ^= 1 << rng.randrange(8)   # a header field
            elif which == 1:
                b[rng.randrange(108, 140)] ^= 1 << rng.randrange(8)  # the nonce
            elif which == 2:
                b[-1 - rng.randrange(20)] ^= 1 << rng.randrange(8)   # the solution
            else:
                ln = len(h) - 140 - len(compact(len(h)))
                b = bytearray(h[:140] + compact(ln - 1) + h[-(ln - 1):])  # one byte short
            batch.append(bytes(b))
        cpu = native.check_equihash_headers(batch, chain, False)
        gpu = native.check_equihash_headers(batch, chain, True)
        assert gpu == cpu and any(cpu) and not all(cpu)
    assert all(l["items"] > 0 for l in native.gpu_verify_stats()["lanes"])


# ------------------------------------------------------------------ randomized differential

def _mutate_sig(rng, pub, sig, msg):
    kind = rng.randrange(12)
    if kind == 0:
        return pub, sig, msg
    if kind == 1:
        m = bytearray(msg)
        m[rng.randrange(32)] ^= 1 << rng.randrange(8)
        return pub, sig, bytes(m)
    if kind == 2:  # flip a bit anywhere in the DER signature (structure, r, s)
        s = bytearray(sig)
        s[rng.randrange(len(s))] ^= 1 << rng.randrange(8)
        return pub, bytes(s), msg
    if kind == 3:  # flip a bit of the key (off-curve points, wrong prefixes)
        p = bytearray(pub)
        p[rng.randrange(len(p))] ^= 1 << rng.randrange(8)
        return bytes(p), sig, msg
    if kind == 4:  # high-S twin (lax parse + normalisation: still valid)
        r, s = ref.der_decode(sig)
        return pub, ref.der_encode(r, ref.N - s), msg
    if kind == 5:  # r or s out of range / zero
        r, s = ref.der_decode(sig)
        choice = rng.randrange(4)
        r2, s2 = [(0, s), (r, 0), (r + ref.N, s), (r, s + ref.N)][choice]
        return pub, ref.der_encode(r2, s2), msg
    if kind == 6:  # truncated signature
        return pub, sig[:rng.randrange(len(sig))], msg
    if kind == 7:  # trailing garbage after the DER (lax parser behaviour)
        return pub, sig + bytes([rng.randrange(256)]), msg
    if kind == 8:  # key of another signer
        return N.ec_pubkey_create(rng.randbytes(32), rng.random() < 0.5), sig, msg
    if kind == 9 and len(pub) == 65:  # hybrid encoding
        return bytes([6 + (pub[64] & 1)]) + pub[1:], sig, msg
    if kind == 10:  # r := x of the key (a value in range, wrong)
        r, s = ref.der_decode(sig)
        return pub, ref.der_encode(int.from_bytes(pub[1:33], "big") % ref.N or 1, s), msg
    return pub, sig, msg


@pytest.mark.gpu
def test_differential_ecdsa_10k(native, two_lanes):
    rng = random.Random(20261017)
    base = []
    for i in range(400):
        sec = rng.randbytes(32)
        msg = hashlib.sha256(b"d%d" % i).digest()
        base.append((native.ec_pubkey_create(sec, i % 3 != 0), native.ec_sign(sec, msg), msg))
    items = []
    for j in range(10240):
        pub, sig, msg = base[j % len(base)]
        pub, sig, msg = _mutate_sig(rng, pub, sig, msg)
        items.append((pub[:65], sig[:72], msg))
    cpu, _ = native.ecdsa_verify_batch(items, use_gpu=False)
    gpu, _ = native.ecdsa_verify_batch(items, use_gpu=True)
    diff = [i for i, (a, b) in enumerate(zip(cpu, gpu)) if a != b]
    assert not diff, [items[i] for i in diff[:3]]
    assert 0.1 < sum(cpu) / len(cpu) < 0.9


def _mutate_solution(rng, sol, cbl):
    kind = rng.randrange(9)
    idx = N.eh_indices_from_minimal(sol, cbl)
    if kind == 0:
        return sol
    if kind == 1:  # flip one bit of the packed solution
        b = bytearray(sol)
        b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        return bytes(b)
    if kind == 2:  # swap two sibling subtrees (ordering rule)
        w = 1 << rng.randrange(len(idx).bit_length() - 1)
        j = rng.randrange(len(idx) // (2 * w)) * 2 * w
        idx = idx[:j] + idx[j + w:j + 2 * w] + idx[j:j + w] + idx[j + 2 * w:]
    elif kind == 3:  # duplicate an index
        a, b = rng.randrange(len(idx)), rng.randrange(len(idx))
        idx[a] = idx[b]
    elif kind == 4:  # replace an index with a random one
        idx[rng.randrange(len(idx))] = rng.randrange(1 << (cbl + 1))
    elif kind == 5:  # wrong length
        return sol[:-1] if rng.random() < 0.5 else sol + b"\0"
    elif kind == 6:  # all zero
        return bytes(len(sol))
    elif kind == 7:  # two adjacent indices swapped (leaf order)
        a = rng.randrange(len(idx) - 1)
        idx[a], idx[a + 1] = idx[a + 1], idx[a]
    else:  # index +- 1
        a = rng.randrange(len(idx))
        idx[a] = (idx[a] + rng.choice((-1, 1))) % (1 << (cbl + 1))
    return N.eh_minimal_from_indices(idx, cbl)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,total", [(48, 5, 12000), (200, 9, 10000)])
def test_differential_equihash_10k(native, two_lanes, n, k, total):
    rng = random.Random(n * 1000 + k)
    cbl = n // (k + 1)
    solver = native.EquihashGpuSolver(n, k, 16)
    pool = []
    nonce = 0
    while len(pool) < 24:
        states = []
        for _ in range(16):
            st = native.EquihashState(n, k)
            st.update(b"diff" + bytes(104) + struct.pack("<I", nonce) + bytes(28))
            nonce += 1
            states.append(st)
        for st, ss in zip(states, solver.solve(states)):
            pool += [(st, s) for s in ss]
    sts, sols = [], []
    for j in range(total):
        st, s = pool[j % len(pool)]
        sts.append(st)
        sols.append(_mutate_solution(rng, s, cbl))
    gpu = native.gpu_verify_equihash(n, k, sts, sols)
    cpu = [native.eh_is_valid_solution(n, k, st, s)[0] for st, s in zip(sts, sols)]
    diff = [i for i, (a, b) in enumerate(zip(cpu, gpu)) if a != b]
    assert not diff, diff[:5]
    assert 0.05 < sum(cpu) / len(cpu) < 0.6


def test_plan_shards_at_block_scale(native):
    """PlanShards at the 8 MB block's 199,680 signatures (pure, no GPU): four lanes on ONE
    device take three shards (each >= the 65,536 per-lane floor); eight devices with two lanes
    each take one shard per device first (>= 4,096 per device)."""
    n = 199_680
    plan = native.plan_shards(n, [0, 0, 0, 0], 4096, 65536)
    assert [(lane, hi - lo) for lane, lo, hi in plan] == [(0, 66560), (1, 66560), (2, 66560)]
    assert plan[0][1] == 0 and plan[-1][2] == n and all(a[2] == b[1] for a, b in zip(plan, plan[1:]))
    devs = [d for d in range(8) for _ in range(2)]
    plan8 = native.plan_shards(n, devs, 4096, 65536)
    assert sorted({devs[lane] for lane, _, _ in plan8}) == list(range(8))
    assert sum(hi - lo for _, lo, hi in plan8) == n and len(plan8) == 8


@pytest.fixture
def four_lanes(native):
    native.gpu_verify_set_devices([0, 0, 0, 0])
    yield
    native.gpu_verify_set_devices([])


@pytest.mark.gpu
def test_four_lanes_block_scale_ecdsa_matches_cpu(native, four_lanes):
    """The node's verify service with four lanes on device 0 at the 199,680-signature shape of an
    8 MB block (service defaults: 65,536 per extra lane on one device): the batch splits into the
    planned three shards, each lane that got a shard did its items, and every verdict equals the
    CPU consensus verifier's. 4,096 distinct signatures (valid, wrong message/key, high-S,
    garbage DER, ...) are tiled to the full size."""
    n = 199_680
    plan = native.gpu_verify_plan(n)
    assert [hi - lo for _, lo, hi in plan] == [66560, 66560, 66560]
    uniq, expect = make_items(native, 4096, seed=23)
    cpu, _ = native.ecdsa_verify_batch(uniq, use_gpu=False)
    assert cpu == expect
    items = (uniq * (n // len(uniq) + 1))[:n]
    want = (cpu * (n // len(cpu) + 1))[:n]
    before = native.gpu_verify_stats()
    gpu, _ = native.ecdsa_verify_batch(items, use_gpu=True)  # the node's deferred batch -> the service
    assert gpu == want
    st = native.gpu_verify_stats()
    assert st["sharded_batches"] == before["sharded_batches"] + 1
    got = [l["items"] for l in st["lanes"]]
    assert [l["device"] for l in st["lanes"]] == [0, 0, 0, 0]
    assert sorted(got, reverse=True)[:3] == [66560, 66560, 66560] and sum(got) == n
