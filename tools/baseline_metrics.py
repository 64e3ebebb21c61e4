#!/usr/bin/env python3
"""The MI355X numbers BASELINE.md asks for beyond the headline Sol/s (one JSON line each).

python tools/baseline_metrics.py [--quick]

  eh48_solve_latency   Equihash(48,5) (regtest) solve latency: GPU solver, one nonce per launch,
                       vs the CPU solver (reference BasicSolve, src/crypto/equihash.cpp:332)
  eh200_verify         Equihash(200,9) header verification in 2000-header batches (one `headers`
                       message, reference src/validation.h:101): GPU batch verifier vs the CPU
                       IsValidSolution (reference src/crypto/equihash.cpp:725)
  eh200_solve          Equihash(200,9) nonces/s and Sol/s at several batch sizes (single solver)

SHA-256d, merkle and the 8 MB block connect are measured by bin/bench_bcp
(GPU_SHA256d64_1M, GPU_MerkleRoot_*, ConnectBlock8MB_{CPU,GPU}).
"""
import argparse
import json
import os
import statistics
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HEADER = bytes((i * 37 + 11) & 0xFF for i in range(108))


def state(native, n, k, i, salt=0):
    st = native.EquihashState(n, k)
    st.update(HEADER + struct.pack("<QQQQ", i, salt, 0, 5))
    return st


def emit(d):
    print(json.dumps(d), flush=True)


def eh48(native, quick):
    nn = 16 if quick else 64
    solver = native.EquihashGpuSolver(48, 5, 1)
    solver.solve([state(native, 48, 5, 0)])  # warm-up (module load, first launch)
    lat, sols = [], 0
    for i in range(nn):
        st = state(native, 48, 5, i)
        t = time.perf_counter()
        r = solver.solve([st])
        lat.append(time.perf_counter() - t)
        sols += len(r[0])
    cpu = []
    for i in range(min(nn, 16)):
        st = state(native, 48, 5, i)
        t = time.perf_counter()
        native.eh_solve_cpu(48, 5, st)
        cpu.append(time.perf_counter() - t)
    emit({"metric": "eh48_solve_latency", "gpu_ms_median": round(1e3 * statistics.median(lat), 3),
          "gpu_ms_p90": round(1e3 * sorted(lat)[int(0.9 * len(lat))], 3),
          "cpu_ms_median": round(1e3 * statistics.median(cpu), 3), "nonces": nn, "solutions": sols})


def eh200_verify(native, quick):
    solver = native.EquihashGpuSolver(200, 9, 32)
    pairs = []
    for b in range(1 if quick else 2):
        sts = [state(native, 200, 9, 32 * b + i, 77) for i in range(32)]
        for st, sols in zip(sts, solver.solve(sts)):
            pairs += [(st, s) for s in sols]
    if not pairs:
        raise SystemExit("no (200,9) solutions to verify")
    batch = [pairs[i % len(pairs)] for i in range(2000)]
    sts, sols = [p[0] for p in batch], [p[1] for p in batch]
    ok = native.eh_verify_batch_gpu(200, 9, sts, sols)
    assert all(ok), "GPU verifier rejected solver output"
    # negative control: one corrupted solution in the batch is caught
    bad = list(sols)
    bad[7] = bytes([bad[7][0] ^ 1]) + bad[7][1:]
    assert native.eh_verify_batch_gpu(200, 9, sts, bad)[7] is False
    reps = 5 if quick else 20
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        native.eh_verify_batch_gpu(200, 9, sts, sols)
        ts.append(time.perf_counter() - t)
    cpu = []
    for st, s in batch[:50]:
        t = time.perf_counter()
        assert native.eh_is_valid_solution(200, 9, st, s)[0]
        cpu.append(time.perf_counter() - t)
    med = statistics.median(ts)
    emit({"metric": "eh200_verify_2000_headers", "gpu_ms_per_batch": round(1e3 * med, 3),
          "gpu_headers_per_s": round(2000 / med, 1), "cpu_us_per_header": round(1e6 * statistics.median(cpu), 1),
          "cpu_headers_per_s_1thread": round(1 / statistics.median(cpu), 1),
          "distinct_solutions": len(pairs)})


def eh200_solve(native, quick):
    for b in ([8, 32] if quick else [8, 16, 32, 64]):
        solver = native.EquihashGpuSolver(200, 9, b)
        sts = [state(native, 200, 9, 1000 + i, 3) for i in range(b)]
        solver.solve(sts)
        reps = max(2, 128 // b)
        t = time.perf_counter()
        n = 0
        for _ in range(reps):
            n += sum(len(x) for x in solver.solve(sts))
        dt = time.perf_counter() - t
        emit({"metric": "eh200_solve_single_solver", "batch": b, "nonces_per_s": round(reps * b / dt, 1),
              "sol_per_s": round(n / dt, 1), "ms_per_batch": round(1e3 * dt / reps, 3),
              "device_gib": round(solver.device_bytes / 2**30, 2)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="eh48,eh200_verify,eh200_solve")
    a = ap.parse_args()
    from bitcoincashplus_amd import native, require_gpu
    require_gpu("baseline_metrics")
    emit({"device": native.gpu_device_name(0)})
    for name in a.only.split(","):
        {"eh48": eh48, "eh200_verify": eh200_verify, "eh200_solve": eh200_solve}[name](native, a.quick)


if __name__ == "__main__":
    main()
