#!/usr/bin/env python3
"""Locate where the GPU solver loses a solution the CPU reference finds (small params).

python tools/eh_missing.py --n 48 --k 5 --nonce 10
For every CPU solution missing from the GPU output: is its index list among the GPU's final
candidates (then expand/validation dropped it), and which tree levels' nodes have equal rows.
"""
import argparse
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


GEOM = {(48, 5): (8, 512), (96, 5): (128, 1280), (200, 9): (512, int(os.environ.get('BCP_EH_AREA', 6016)))}  # (NB, AREA)


def trace_missing(dump, n, k, idx):
    """Follow one missing solution up the GPU's tree: at each stage, find the slot holding each of
    its subtrees (by parent-slot pairs) and report the first stage where one is absent.
    dump: K arrays of ROWS slots: stage-0 leaf indices, then the parent triples
    (bucket << 32 | j << 16 | i) of stages 1..K-1; never-written slots are all-ones."""
    import numpy as np
    nb, area = GEOM[(n, k)]
    rows = nb * area
    d = np.asarray(dump, dtype=np.uint64)
    F = [d[s * rows:(s + 1) * rows] for s in range(k)]
    f0 = F[0]
    valid = f0 != 0xFFFFFFFF
    leaf_slot = {int(v): int(sl) for sl, v in zip(np.nonzero(valid)[0], f0[valid])}
    cur = [leaf_slot.get(i) for i in idx]
    if any(c is None for c in cur):
        print("    stage 0: leaf missing")
        return
    for s in range(1, k):
        f = F[s]
        g = np.nonzero(f != np.uint64(0xFFFFFFFFFFFFFFFF))[0]
        fv = f[g]
        dd = (fv >> np.uint64(32)).astype(np.int64)
        fi = (fv & np.uint64(0xFFFF)).astype(np.int64)
        fj = ((fv >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64)
        p1, p2 = dd * area + fi, dd * area + fj
        lo, hi = np.minimum(p1, p2).astype(np.uint64), np.maximum(p1, p2).astype(np.uint64)
        keys = (lo << np.uint64(32)) | hi
        order = np.argsort(keys)
        sk = keys[order]
        nxt = []
        for a, b in zip(cur[0::2], cur[1::2]):
            q = (min(a, b) << 32) | max(a, b)
            pos = int(np.searchsorted(sk, np.uint64(q)))
            if pos < len(sk) and int(sk[pos]) == q:
                nxt.append(int(g[order[pos]]))
            else:
                print(f"    stage {s}: pair of stage-{s - 1} slots ({a}, {b}) never collided "
                      f"(buckets {a // area}, {b // area})")
                return
        cur = nxt
    print(f"    all {k - 1} stages present; final pair slots {cur} (buckets {[c // area for c in cur]})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--nonces", default="10,25")
    ap.add_argument("--salt", default="main")
    ap.add_argument("--scan", type=int, default=0, help="scan nonces 0..SCAN-1 and trace every miss")
    args = ap.parse_args()
    from bitcoincashplus_amd import native
    from bitcoincashplus_amd.utils import equihash_ref as R
    cbl = args.n // (args.k + 1)
    nonces = range(args.scan) if args.scan else [int(x) for x in args.nonces.split(",")]
    for nonce in nonces:
        d = (args.salt.encode() + bytes(108))[:108] + struct.pack("<I", nonce) + bytes(28)
        st = native.EquihashState(args.n, args.k)
        st.update(d)
        cpu = native.eh_solve_cpu(args.n, args.k, st)[0]
        solver = native.EquihashGpuSolver(args.n, args.k, 1)
        solver.set_debug(True)
        gpu = solver.solve([st])[0]
        cands = [tuple(c) for c in solver.stats()["debug_cands"]]
        if args.scan and set(cpu) <= set(gpu):
            continue
        print(f"nonce {nonce}: cpu {len(cpu)} gpu {len(gpu)} candidates {len(cands)} "
              f"pair_dropped {solver.stats()['pair_dropped']} dropped {solver.stats()['stage_dropped']}")
        sets = None
        for sol in cpu:
            if sol in gpu:
                continue
            idx = tuple(R.indices_from_minimal(sol, cbl))
            incand = idx in cands or any(sorted(c) == sorted(idx) for c in cands)
            print("  missing solution; among candidates:", incand, "first indices", idx[:8])
            trace_missing(solver.debug_dump(), args.n, args.k, idx)


if __name__ == "__main__":
    main()
