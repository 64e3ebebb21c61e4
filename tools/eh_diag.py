#!/usr/bin/env python3
"""Equihash GPU solver diagnostics: per-stage bucket fill/drops, yield, batch-size sweep.

python tools/eh_diag.py [--n 200 --k 9] [--nonces 32] [--batches 1,2,4,8]
"""
import argparse
import json
import os
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--k", type=int, default=9)
    ap.add_argument("--nonces", type=int, default=32)
    ap.add_argument("--batches", default="1,2,4,8")
    args = ap.parse_args()
    from bitcoincashplus_amd import native

    header = bytes((i * 37 + 11) & 0xFF for i in range(108))

    def st(i):
        s = native.EquihashState(args.n, args.k)
        s.update(header + struct.pack("<QQQQ", i, 0, 0, 7))
        return s

    # yield + stage stats with batch 1
    solver = native.EquihashGpuSolver(args.n, args.k, 1)
    solver.set_debug(True)
    tot = 0
    drops = None
    for i in range(args.nonces):
        r = solver.solve([st(i)])
        tot += len(r[0])
        s = solver.stats()
        d = s["stage_dropped"]
        drops = d if drops is None else [a + b for a, b in zip(drops, d)]
    s = solver.stats()
    print(json.dumps({"yield_sol_per_nonce": tot / args.nonces, "stage_rows_last": s["stage_rows"],
                      "stage_maxfill_last": s["stage_maxfill"], "stage_dropped_total": drops,
                      "candidates": s["candidates"], "duplicates": s["duplicates"]}))
    for b in [int(x) for x in args.batches.split(",")]:
        solver = native.EquihashGpuSolver(args.n, args.k, b)
        states = [st(1000 + i) for i in range(b)]
        solver.solve(states)
        reps = max(2, 64 // b)
        t = time.perf_counter()
        n = 0
        for r in range(reps):
            res = solver.solve(states)
            n += sum(len(x) for x in res)
        dt = time.perf_counter() - t
        print(json.dumps({"batch": b, "nonces_per_s": reps * b / dt, "ms_per_batch": 1000 * dt / reps,
                          "gpu_ms_per_batch": solver.stats()["gpu_ms"] / (reps + 1),
                          "sol_per_s_est": n / dt}))


def phases():
    """Per-phase cycle breakdown of the round kernels (diagnostic stamp build)."""
    from bitcoincashplus_amd import native
    s = native.EquihashGpuSolver(200, 9, 4)
    s.set_stamp_mode(True)
    header = bytes(108)
    sts = []
    for i in range(4):
        st = native.EquihashState(200, 9)
        st.update(header + struct.pack("<QQQQ", i, 0, 0, 9))
        sts.append(st)
    s.solve(sts)
    s.solve(sts)
    names = ["total", "commit", "issue", "chain", "pairs", "claim_sort", "emit", "pairs_list", "pairs_filter"]
    for stage, ph in enumerate(s.phase_cycles(4)):
        print(json.dumps({"round": stage + 1, **{n: round(v) for n, v in zip(names, ph)}}))


if __name__ == "__main__":
    phases() if os.environ.get("EH_PHASES") else main()
