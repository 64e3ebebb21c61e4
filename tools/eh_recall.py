#!/usr/bin/env python3
"""GPU-vs-CPU solution recall of the Equihash solver over many nonces.

python tools/eh_recall.py --n 200 --k 9 --nonces 32 --threads 8 [--salt main]
Solves every nonce with the CPU reference solver (thread pool; the binding releases
the GIL) and with the GPU solver, then prints per-nonce counts, the total recall
ratio, any GPU solution the CPU does not have (must be none), and the GPU's
per-stage drop counters for the first batch (debug mode).
"""
import argparse
import concurrent.futures as cf
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def header_input(nonce: int, salt: bytes) -> bytes:
    body = (salt + bytes(108))[:108]
    return body + struct.pack("<I", nonce) + bytes(28)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--k", type=int, default=9)
    ap.add_argument("--nonces", type=int, default=32)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--salt", default="main")
    ap.add_argument("--repeat", type=int, default=0)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    from bitcoincashplus_amd import native
    n, k = args.n, args.k
    states = []
    for i in range(args.nonces):
        st = native.EquihashState(n, k)
        st.update(header_input(i, args.salt.encode()))
        states.append(st)
    with cf.ThreadPoolExecutor(args.threads) as ex:
        cpu = list(ex.map(lambda st: set(native.eh_solve_cpu(n, k, st)[0]), states))
    solver = native.EquihashGpuSolver(n, k, args.batch)
    solver.set_debug(True)
    gpu = []
    dbg = None
    for b0 in range(0, args.nonces, args.batch):
        gpu += [set(x) for x in solver.solve(states[b0:b0 + args.batch])]
        if dbg is None:
            s = solver.stats()
            dbg = {key: s[key] for key in ("stage_dropped", "pair_dropped", "stage_maxfill", "cand_max", "cand_dropped") if key in s}
    extra = sum(len(g - c) for g, c in zip(gpu, cpu))
    tc, tg = sum(map(len, cpu)), sum(len(g & c) for g, c in zip(gpu, cpu))
    for i, (c, g) in enumerate(zip(cpu, gpu)):
        if len(g & c) != len(c):
            print(f"nonce {i}: cpu {len(c)} gpu {len(g & c)} missing {len(c - g)}")
    st = solver.stats()
    res = {"n": n, "k": k, "nonces": args.nonces, "cpu_solutions": tc, "gpu_found": tg,
           "recall": round(tg / max(tc, 1), 4), "gpu_not_in_cpu": extra, "debug_first_batch": dbg,
           "cand_max": st.get("cand_max"), "cand_dropped": st.get("cand_dropped")}
    # the solver is not deterministic (row order inside a bucket follows the atomics): solve the
    # same nonces again and report what each repeat found
    reps, drops = [], []
    for _ in range(args.repeat):
        g2 = []
        for b0 in range(0, args.nonces, args.batch):
            g2 += [set(x) for x in solver.solve(states[b0:b0 + args.batch])]
        reps.append(sum(len(g & c) for g, c in zip(g2, cpu)))
        drops.append(list(solver.stats().get("stage_dropped_all") or []))
    if reps:
        st = solver.stats()
        res.update(repeat_found=reps, repeat_stage_dropped_cum=drops, cand_max=st.get("cand_max"), cand_dropped=st.get("cand_dropped"))
    st = solver.stats()
    res.update(stage_dropped_all=st.get("stage_dropped_all"), stage_maxfill_all=st.get("stage_maxfill_all"),
               overflow_fills=[(f >> 32, f & 0xffffffff) for f in (st.get("overflow_fills") or [])][:64])
    print(json.dumps(res))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
