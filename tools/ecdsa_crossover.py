"""CPU-pool vs MI355X crossover for batched ECDSA verification (sets -gpusigthreshold).

Block validation sends a batch to the GPU only when it has at least -gpusigthreshold
signatures (csrc/node/sigverify.h DEFAULT_GPU_SIG_THRESHOLD). This measures both paths
end to end (host DER parse + upload + kernels + readback for the GPU; the 16-thread
worker pool, the reference's MAX_SCRIPTCHECK_THREADS, for the CPU) at batch sizes from
64 to 64k and prints one JSON line with the per-size timings and the crossover.
Usage: python tools/ecdsa_crossover.py [threads]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bitcoincashplus_amd as b  # noqa: E402

threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
nat = b.native
base = []
for i in range(1024):
    k = os.urandom(32)
    m = os.urandom(32)
    base.append((nat.ec_pubkey_create(k, True), nat.ec_sign(k, m), m))
items = (base * 64)[:65536]
print(f"{len(base)} unique signatures, {threads} CPU threads", flush=True)


def best_ms(n, use_gpu, reps):
    best = 1e30
    for _ in range(reps):
        r, ms = nat.ecdsa_verify_batch(items[:n], use_gpu=use_gpu, threads=threads)
        assert all(r)
        best = min(best, ms)
    return best


if b.gpu_available():
    nat.ecdsa_verify_batch(items[:4096], use_gpu=True, threads=threads)  # table upload, code load
rows = []
crossover = None
default_fused = nat.ecdsa_fused_max()


def path_ms(n, fused_max, reps):
    nat.ecdsa_set_fused_max(fused_max)
    try:
        return best_ms(n, True, reps)
    finally:
        nat.ecdsa_set_fused_max(default_fused)


for n in (64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536):
    reps = 5 if n <= 4096 else 3
    cpu = best_ms(n, False, reps)
    gpu = best_ms(n, True, reps) if b.gpu_available() else None
    row = {"n": n, "cpu_ms": round(cpu, 3), "gpu_ms": None if gpu is None else round(gpu, 3),
           "cpu_sig_per_s": round(n / cpu * 1e3), "gpu_sig_per_s": None if gpu is None else round(n / gpu * 1e3)}
    if b.gpu_available():  # both GPU paths pinned (default: fused up to ecdsa_fused_max())
        row["gpu_fused_ms"] = round(path_ms(n, 1 << 40, reps), 3)
        row["gpu_split_ms"] = round(path_ms(n, 0, reps), 3)
    rows.append(row)
    print(json.dumps(rows[-1]), flush=True)
    if gpu is not None and crossover is None and gpu < cpu:
        crossover = n
print(json.dumps({"threads": threads, "fused_max": default_fused, "crossover_n": crossover, "rows": rows}))
