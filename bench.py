#!/usr/bin/env python3
"""Headline benchmark: Equihash(200,9) solver throughput (solutions/s) on MI355X.

BASELINE.md names Equihash(200,9) Sol/s per GPU and per 8-GPU node as the
metric to establish (the reference publishes no number; its only solver is the
CPU BasicSolve, reference src/crypto/equihash.cpp:332, driven by
src/rpc/mining.cpp:161-199).  A "step" is one solver batch: BATCH nonces per
GPU, each fully solved (BLAKE2b generation, 9 collision rounds, index-tree
recovery, canonical ordering + duplicate rejection).  Per-GPU work is fixed,
so scaling is weak; ranks take disjoint nonce ranges (nonce-space data
parallelism) and the solution counts are summed with an RCCL all-reduce.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import collections
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BCP_EH_BATCH", "32")))
    ap.add_argument("--verify", type=int, default=1, help="GPU-verify every solution after timing")
    ap.add_argument("--solvers", type=int, default=int(os.environ.get("BCP_EH_SOLVERS", "2")),
                    help="solvers in flight per GPU (each its own stream and buffers)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from bitcoincashplus_amd import native, require_gpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    require_gpu("bench.py")
    # one rank per GPU over RCCL ("nccl"); BCP_DIST_BACKEND=gloo + ranks sharing a GPU is the
    # rehearsal mode for the multi-rank path on a 1-GPU box (CPU-side reductions)
    backend = os.environ.get("BCP_DIST_BACKEND", "nccl")
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # several solvers in flight (default two, double-buffered): while the GPU runs batch s, the
    # host decodes batch s-1, and one solver's kernels fill the other's tails
    nsolv = max(1, args.solvers)
    solvers = [native.EquihashGpuSolver(200, 9, args.batch, device) for _ in range(nsolv)]
    solver = solvers[0]
    # Template: CEquihashInput of a mainnet-shaped header (108 B), random-ish but fixed.
    header = bytes((i * 37 + 11) & 0xFF for i in range(108))

    def states_for(step):
        sts = []
        for b in range(args.batch):
            # nonce lanes: rank in the top bytes, step/batch counters in the low bytes
            nonce = struct.pack("<QQQQ", step * args.batch + b, 0, 0, rank)
            st = native.EquihashState(200, 9)
            st.update(header + nonce)
            sts.append(st)
        return sts

    for w in range(args.warmup):
        solvers[w % nsolv].solve(states_for(1_000_000 + w))
    for sv in solvers:
        sv.reset_stats()
    all_states = [states_for(s) for s in range(args.steps)]
    sols_kept = []

    barrier()
    t0 = time.perf_counter()
    nsol = 0
    pending = collections.deque()  # (step, solver) launched but not yet collected

    def collect():
        nonlocal nsol
        ps, psolver = pending.popleft()
        for b, sols in enumerate(psolver.collect()):
            nsol += len(sols)
            if ps < 2:
                sols_kept.extend((all_states[ps][b], x) for x in sols)

    for s in range(args.steps):
        if len(pending) == nsolv:  # this step's solver still holds an older batch
            collect()
        solvers[s % nsolv].launch(all_states[s])
        pending.append((s, solvers[s % nsolv]))
    while pending:
        collect()
    barrier()
    dt = time.perf_counter() - t0

    t = torch.tensor([float(nsol), dt], dtype=torch.float64, device=red_dev)
    if world > 1:
        tot = t.clone()
        dist.all_reduce(tot[:1], op=dist.ReduceOp.SUM)
        mx = t.clone()
        dist.all_reduce(mx[1:], op=dist.ReduceOp.MAX)
        total_sols, max_dt = float(tot[0]), float(mx[1])
    else:
        total_sols, max_dt = nsol, dt

    verified = None
    if args.verify and sols_kept:
        ok = native.eh_verify_batch_gpu(200, 9, [a for a, _ in sols_kept], [b for _, b in sols_kept], device)
        verified = bool(all(ok))
        if not verified:
            raise SystemExit("bench: GPU verifier rejected solver output")

    st = solvers[0].stats()
    if rank == 0:
        value = total_sols / max_dt
        nonces = args.steps * args.batch * world
        out = {
            "metric": "equihash_200_9_solutions_per_sec",
            "value": round(value, 2),
            "unit": "Sol/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * max_dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint32",
            "data": "synthetic",
            "config": {
                "model": "Equihash(200,9) mainnet PoW solver (BLAKE2b, K=9 collision rounds)",
                "global_batch": args.batch * world,
                "seq_len": 2097152,
                "parallelism": f"dp{world} (nonce-space)",
                "solvers_in_flight": nsolv,
                "nonces_per_sec": round(nonces / max_dt, 2),
                "solutions_per_nonce": round(total_sols / max(nonces, 1), 3),
                "verified": verified,
                "rank0_dropped_rows_sampled": st["dropped_rows_sampled"],
            },
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
