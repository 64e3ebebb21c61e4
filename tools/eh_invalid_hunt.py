#!/usr/bin/env python3
"""Hunt for invalid GPU solver outputs: solve many nonces of Equihash(200,9), re-check every
solution with the CPU verifier (reference IsValidSolution semantics), and for each rejected one
name the first failing rule from an independent hashlib.blake2b recomputation of the tree:
collision bits, subtree ordering or index distinctness at the level where it breaks.

python tools/eh_invalid_hunt.py [--batches 64] [--batch 32] [--json out.json]
"""
import argparse
import hashlib
import json
import os
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

N, K = 200, 9
CBL = N // (K + 1)


def header(i):
    return bytes((j * 37 + 11) & 0xFF for j in range(108)) + struct.pack("<QQQQ", i, 7, 0, 0)


def leaf(hdr, idx):
    g = idx // 2
    h = hashlib.blake2b(hdr + struct.pack("<I", g), digest_size=50,
                        person=b"ZcashPoW" + struct.pack("<II", N, K)).digest()
    chunk = h[(idx % 2) * 25:(idx % 2) * 25 + 25]
    return int.from_bytes(chunk, "big")  # 200 bits, big-endian as the digest's bit order


def diagnose(hdr, idx):
    """First failing rule of IsValidSolution for index list idx, or None."""
    level = [(leaf(hdr, i), [i]) for i in idx]
    for lv in range(1, K + 1):
        nxt = []
        for a in range(0, len(level), 2):
            (va, ia), (vb, ib) = level[a], level[a + 1]
            x = va ^ vb
            bits = CBL * lv if lv < K else N
            if x >> (N - bits):
                return {"level": lv, "pair": a // 2, "rule": "collision", "bits": bits}
            if not ia[0] < ib[0]:
                return {"level": lv, "pair": a // 2, "rule": "ordering"}
            if set(ia) & set(ib):
                return {"level": lv, "pair": a // 2, "rule": "distinct"}
            nxt.append((x, ia + ib))
        level = nxt
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--json", default="")
    ap.add_argument("--selfcheck", type=int, default=20, help="valid solutions also run through diagnose()")
    ap.add_argument("--solvers", type=int, default=2, help="solvers in flight (launch/collect as bench.py)")
    a = ap.parse_args()
    from bitcoincashplus_amd import native
    solvers = [native.EquihashGpuSolver(N, K, a.batch) for _ in range(max(1, a.solvers))]
    total = bad = 0
    found = []
    t0 = time.time()
    pending = []

    def batch_states(b):
        hdrs = [header(b * a.batch + i) for i in range(a.batch)]
        sts = []
        for h in hdrs:
            s = native.EquihashState(N, K)
            s.update(h)
            sts.append(s)
        return hdrs, sts

    gpu_disagree = 0

    def check(b, hdrs, sts, res):
        nonlocal total, bad, gpu_disagree
        flat = [(sts[i], sol) for i, sols in enumerate(res) for sol in sols]
        if flat:  # the GPU batch verifier's verdicts against the CPU verifier's
            gv = native.eh_verify_batch_gpu(N, K, [x for x, _ in flat], [y for _, y in flat], 0)
            for (st_, sol), v in zip(flat, gv):
                if bool(v) != bool(native.eh_is_valid_solution(N, K, st_, sol)):
                    gpu_disagree += 1
                    print(json.dumps({"batch": b, "gpu_verifier": bool(v), "cpu_verifier": not bool(v)}), flush=True)
        for i, sols in enumerate(res):
            for sol in sols:
                total += 1
                if native.eh_is_valid_solution(N, K, sts[i], sol):
                    if a.selfcheck > 0:  # the independent model must accept what the verifier accepts
                        a.selfcheck -= 1
                        d = diagnose(hdrs[i], native.eh_indices_from_minimal(sol, CBL))
                        assert d is None, d
                    continue
                bad += 1
                idx = native.eh_indices_from_minimal(sol, CBL)
                d = diagnose(hdrs[i], idx)
                found.append({"batch": b, "nonce": i, "diag": d, "dup_indices": len(idx) - len(set(idx))})
                print(json.dumps(found[-1]), flush=True)

    # launch/collect with several solvers in flight, as bench.py does
    for b in range(a.batches):
        sv = solvers[b % len(solvers)]
        if len(pending) == len(solvers):
            pb, phdrs, psts, psv = pending.pop(0)
            check(pb, phdrs, psts, psv.collect())
        hdrs, sts = batch_states(b)
        sv.launch(sts)
        pending.append((b, hdrs, sts, sv))
        if b % 16 == 15:
            print(json.dumps({"batches": b + 1, "solutions": total, "invalid": bad,
                              "seconds": round(time.time() - t0, 1)}), flush=True)
    while pending:
        pb, phdrs, psts, psv = pending.pop(0)
        check(pb, phdrs, psts, psv.collect())
    out = {"nonces": a.batches * a.batch, "solutions": total, "invalid": bad, "gpu_verifier_disagreements": gpu_disagree,
           "found": found}
    print(json.dumps({k: v for k, v in out.items() if k != "found"}))
    if a.json:
        json.dump(out, open(a.json, "w"))


if __name__ == "__main__":
    main()
