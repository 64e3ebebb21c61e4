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

`--gpus N` always drives N GPUs, one process per GPU over RCCL:
* launched by torchrun (WORLD_SIZE set): WORLD_SIZE must equal N;
* launched directly with N > 1: this process counts the visible devices (without
  initialising HIP), refuses N > visible, and starts
  `python -m torch.distributed.run --nproc-per-node N ...` as a child, exiting
  with its status (the parent never touches the GPU).

After timing, every solution of every timed step is re-checked by the GPU batch
verifier; a solution it rejects is re-checked by the CPU verifier, and one that both reject fails
the run (a GPU-only rejection is counted and reported). The mean solutions per nonce must be
>= 1.85 (Equihash(200,9) yields ~1.88 per nonce; a lower figure means the solver
lost rows).
"""
import argparse
import collections
import json
import os
import socket
import struct
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MIN_SOLUTIONS_PER_NONCE = 1.85


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpus() -> int:
    """Device count without initialising the HIP runtime (torch's count is a sysfs/env
    probe on this image), so a launcher parent may still spawn children safely."""
    import torch
    return int(torch.cuda.device_count())


def launch_ranks(argv, gpus: int, launcher=None) -> int:
    """Start one rank per GPU under torch.distributed.run; returns the child's status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return (launcher or subprocess.call)(cmd, env=env)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    # 96 nonces per solver batch: +2.1% Sol/s over 48 in a 10-rep interleaved A/B on the final
    # round-6 solver (88-112 all within 0.3% of it; profiles/equihash_r6.md); two solvers of 96
    # hold ~100 GiB of the GPU's 288 GB
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BCP_EH_BATCH", "96")))
    ap.add_argument("--verify", type=int, default=1, help="GPU-verify every solution after timing")
    ap.add_argument("--solvers", type=int, default=int(os.environ.get("BCP_EH_SOLVERS", "2")),
                    help="solvers in flight per GPU (each its own stream and buffers)")
    ap.add_argument("--pipeline", type=int, default=int(os.environ.get("BCP_EH_PIPELINE", "0")),
                    help="pipeline each batch behind the previous one (generation beside the rounds)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the launcher: ranks rendezvous over gloo, all-reduce, "
                         "report n_gpus; no GPU work and no metric")
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    world = int(os.environ.get("WORLD_SIZE", "0"))
    rehearsal = os.environ.get("BCP_DIST_BACKEND", "nccl") != "nccl"
    if world == 0:
        # not under torchrun: this process is the launcher for N > 1
        nvis = visible_gpus()
        if args.gpus > nvis and not (rehearsal or args.dry_run):
            raise SystemExit(f"bench: --gpus {args.gpus} but only {nvis} GPU(s) visible")
        if args.gpus > 1:
            sys.exit(launch_ranks(argv, args.gpus))
        world = 1
    elif world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        dry_run(world)
    else:
        run(args, world)


def aggregate(nsol, dt, nbad, world, red_dev):
    """Whole-job totals of the timed region: solutions and rejects summed over ranks, the
    slowest rank's time (the job takes as long as its slowest rank)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(nsol), dt, float(nbad)], dtype=torch.float64, device=red_dev)
    if world == 1:
        return float(nsol), dt, float(nbad)
    tot = t.clone()
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    return float(tot[0]), float(mx[1]), float(tot[2])


def dry_run(world):
    """CPU rehearsal of the multi-rank path: the launcher, the gloo rendezvous, the barriers
    around a timed region and the same whole-job aggregation as a real run (each rank reports a
    synthetic solution count and time)."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))  # ranks finish at different times
    nsol = 100 + rank
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    total_sols, max_dt, total_bad = aggregate(nsol, dt, 0, world, "cpu")
    t = torch.tensor([1.0, float(rank)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": int(t[0]), "rank_sum": int(t[1]),
                          "total_solutions": total_sols, "max_rank_seconds": max_dt, "rank0_seconds": dt,
                          "value": total_sols / max_dt}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run(args, world):
    import torch
    import torch.distributed as dist
    from bitcoincashplus_amd import native, require_gpu

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    require_gpu("bench.py")
    # one rank per GPU over RCCL ("nccl"); BCP_DIST_BACKEND=gloo + ranks sharing a GPU is the
    # rehearsal mode for the multi-rank path on a 1-GPU box (CPU-side reductions)
    backend = os.environ.get("BCP_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and local_rank >= ndev:
        raise SystemExit(f"bench: rank {rank} (local {local_rank}) has no GPU of its own ({ndev} visible)")
    device = local_rank % max(1, ndev)
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
    free0 = torch.cuda.mem_get_info(device)[0]
    solvers = [native.EquihashGpuSolver(200, 9, args.batch, device) for _ in range(nsolv)]
    torch.cuda.synchronize()
    # device memory the solvers took (ranks sharing a GPU in the rehearsal overlap here)
    solver_gib = (free0 - torch.cuda.mem_get_info(device)[0]) / 2**30
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
    sols_kept = []  # (state, solution) for EVERY solution of every timed step

    barrier()
    t0 = time.perf_counter()
    nsol = 0
    pending = collections.deque()  # (step, solver) launched but not yet collected

    def collect():
        nonlocal nsol
        ps, psolver = pending.popleft()
        for b, sols in enumerate(psolver.collect()):
            nsol += len(sols)
            sols_kept.extend((all_states[ps][b], x) for x in sols)

    for s in range(args.steps):
        if len(pending) == nsolv:  # this step's solver still holds an older batch
            collect()
        # pipelined behind the previous step's solver: this batch's generation overlaps that
        # batch's collision rounds (solver.launch(states, after=prev))
        prev = solvers[(s - 1) % nsolv] if (args.pipeline and s > 0 and nsolv > 1) else None
        solvers[s % nsolv].launch(all_states[s], prev)
        pending.append((s, solvers[s % nsolv]))
    while pending:
        collect()
    barrier()
    dt = time.perf_counter() - t0

    # verification happens after the timed region: every solution found in every step
    verified = None
    nbad = 0
    gpu_cpu_disagree = 0
    if args.verify and sols_kept:
        ok = native.eh_verify_batch_gpu(200, 9, [a for a, _ in sols_kept], [b for _, b in sols_kept], device)
        # a GPU rejection is re-checked by the CPU verifier (reference IsValidSolution): a
        # solution only counts as bad when both reject it; a disagreement is reported
        for (st_, sol), v in zip(sols_kept, ok):
            if v:
                continue
            if native.eh_is_valid_solution(200, 9, st_, sol):
                gpu_cpu_disagree += 1
            else:
                nbad += 1
        if gpu_cpu_disagree:
            print(f"bench: WARNING: GPU verifier rejected {gpu_cpu_disagree} solution(s) the CPU verifier accepts",
                  file=sys.stderr, flush=True)
        verified = nbad == 0

    # candidate losses over EVERY nonce of the timed steps (device counters, all solvers): rows past a
    # round's capacity, pairs past a round's pair list, final candidates past the per-nonce list
    rows_lost = sum(sum(sv.stats()["stage_dropped_all"] or [0]) for sv in solvers)
    pairs_lost = sum(sum(sv.stats()["pair_dropped_all"] or [0]) for sv in solvers)
    cands_lost = sum(sv.stats()["cand_dropped"] for sv in solvers)
    total_sols, max_dt, total_bad = aggregate(nsol, dt, nbad, world, red_dev)
    per_rank = None
    if world > 1:
        # each rank's nonce lane (the rank id in the nonce's top word, states_for) and its
        # solution count: the lanes must be disjoint and the counts sum to the job total
        # row: [nonce top word, first and last low word timed, solutions]
        mine = torch.tensor([float(rank), 0.0, float(args.steps * args.batch - 1), float(nsol)],
                            dtype=torch.float64, device=red_dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[int(x) for x in t.tolist()] for t in allr]
        if len({r[0] for r in per_rank}) != world:
            raise SystemExit(f"bench: nonce lanes overlap across ranks: {per_rank}")
        lost = torch.tensor([rows_lost, pairs_lost, cands_lost], dtype=torch.float64, device=red_dev)
        dist.all_reduce(lost, op=dist.ReduceOp.SUM)
        rows_lost, pairs_lost, cands_lost = (int(x) for x in lost.tolist())
    if total_bad:
        raise SystemExit(f"bench: GPU and CPU verifiers rejected {int(total_bad)} solver solution(s)")
    nonces = args.steps * args.batch * world
    per_nonce = total_sols / max(nonces, 1)
    if per_nonce < MIN_SOLUTIONS_PER_NONCE:
        raise SystemExit(f"bench: solver recall too low: {per_nonce:.3f} solutions/nonce "
                         f"< {MIN_SOLUTIONS_PER_NONCE}")

    if rank == 0:
        value = total_sols / max_dt
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
                "solutions_per_nonce": round(per_nonce, 3),
                "verified": verified,
                "verified_solutions": int(total_sols) if verified else 0,
                "gpu_cpu_verifier_disagreements": gpu_cpu_disagree,
                "per_rank_nonce_lane_range_solutions": per_rank,
                "solver_device_gib_per_rank": round(solver_gib, 2),
                "rows_dropped_all_nonces": int(rows_lost),
                "pairs_dropped_all_nonces": int(pairs_lost),
                "candidates_dropped_all_nonces": int(cands_lost),
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
