"""Multi-process scale-out (bitcoincashplus_amd.parallel) on gloo, world_size 2:
sharded batch verification returns identical full verdicts on every rank, and the
nonce-space miner sums counts and agrees on one winner. The same code runs on RCCL
(backend "nccl") with one process per MI355X."""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp

from bitcoincashplus_amd import models, parallel


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _items(n):
    from bitcoincashplus_amd import native
    out = []
    for i in range(n):
        sk = hashlib.sha256(b"k%d" % i).digest()
        msg = hashlib.sha256(b"m%d" % i).digest()
        sig = native.ec_sign(sk, msg)
        pub = native.ec_pubkey_create(sk)
        if i % 5 == 3:  # corrupt every fifth message
            msg = hashlib.sha256(b"bad%d" % i).digest()
        out.append((pub, sig, msg))
    return out


def _worker(rank, size, port, q):
    try:
        _run(rank, size, port, q)
    except BaseException as e:  # surface the failure instead of a queue timeout
        q.put((rank, repr(e), None, None))
        raise


def _run(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size))
    import torch.distributed as dist
    from bitcoincashplus_amd import ops
    parallel.init_from_env("gloo")
    items = _items(23)
    res = parallel.sharded_verify(items, lambda shard: ops.ecdsa_verify(shard, use_gpu=False)[0])
    miner = parallel.DistributedEquihashMiner(48, 5, b"\x11" * 108, batch=2, backend="cpu")
    total = miner.step_count()
    win = miner.mine(lambda nonce, sol: True, max_steps=5)
    q.put((rank, res, total, win))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover():
    for n in (0, 1, 7, 23, 64):
        for size in (1, 2, 3, 8):
            spans = [parallel.shard_bounds(n, r, size) for r in range(size)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_models_describe_pow():
    m = models.MODELS["equihash_200_9"]
    assert (m.collision_bits, m.indices_per_solution, m.solution_bytes) == (20, 512, 1344)
    rt = models.chain("regtest")
    assert rt.equihash == models.EquihashModel(48, 5)
    assert rt.pow_for_height(2999) == "sha256d" and rt.pow_for_height(3000) == "equihash"
    assert rt.header_size(3000) == 140
    st = rt.equihash.state(b"\x22" * 140)
    for s in rt.equihash.solve_cpu(st):
        assert len(s) == rt.equihash.solution_bytes and rt.equihash.verify(st, s)


@pytest.mark.timeout(300)
def test_gloo_world2_verify_and_mine():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, res, total, win = q.get(timeout=240)
        assert not isinstance(res, str), res
        out[rank] = (res, total, win)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect = [i % 5 != 3 for i in range(23)]
    assert out[0][0] == expect and out[1][0] == expect
    assert out[0][1] == out[1][1]
    assert out[0][2] is not None and out[0][2] == out[1][2]
    nonce, sol = out[0][2]
    st = models.EquihashModel(48, 5).state(b"\x11" * 108 + nonce)
    assert models.EquihashModel(48, 5).verify(st, sol)
