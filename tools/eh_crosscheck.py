#!/usr/bin/env python3
"""Cross-check the GPU Equihash solver against the CPU reference solver, nonce by nonce.

python tools/eh_crosscheck.py [--n 200 --k 9] [--nonces 8] [--reps 2] [--batch 2]
Prints per nonce: CPU solution count, GPU counts per repetition, missing/extra solutions.
"""
import argparse
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--k", type=int, default=9)
    ap.add_argument("--nonces", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=2)
    args = ap.parse_args()
    from bitcoincashplus_amd import native

    def st(i):
        s = native.EquihashState(args.n, args.k)
        s.update(bytes(b"main" + bytes(104)) + struct.pack("<I", i) + bytes(28))
        return s

    states = [st(i) for i in range(args.nonces)]
    cpu = [set(native.eh_solve_cpu(args.n, args.k, s)[0]) for s in states]
    solver = native.EquihashGpuSolver(args.n, args.k, args.batch)
    solver.set_debug(True)
    tot_cpu = sum(len(c) for c in cpu)
    for rep in range(args.reps):
        solver.reset_stats()  # the *_all counters below cover this repetition's nonces
        got = []
        for b0 in range(0, args.nonces, args.batch):
            got += solver.solve(states[b0:b0 + args.batch])
        miss = sum(len(c - set(g)) for c, g in zip(cpu, got))
        extra = sum(len(set(g) - c) for c, g in zip(cpu, got))
        print(json.dumps({"rep": rep, "cpu_total": tot_cpu, "gpu_total": sum(len(g) for g in got),
                          "missing": miss, "extra": extra,
                          "per_nonce": [[len(c), len(g)] for c, g in zip(cpu, got)],
                          "dropped": solver.stats()["stage_dropped"], "top": solver.stats()["stage_top"][6:],
                          "pair_dropped": solver.stats()["pair_dropped"],
                          # every nonce of the repetition: rows past a round's capacity, pairs lost
                          # to a full list or the per-row partner cap, candidates past MAXCAND
                          "stage_dropped_all": solver.stats()["stage_dropped_all"],
                          "pair_dropped_all": solver.stats()["pair_dropped_all"],
                          "cand_dropped": solver.stats()["cand_dropped"]}), flush=True)


if __name__ == "__main__":
    main()
