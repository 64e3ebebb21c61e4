"""Batched ECDSA verification throughput: CPU pool vs MI355X kernel.
Usage: python tools/ecdsa_bench.py [n_sigs]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bitcoincashplus_amd as b  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
nat = b.native
t = time.time()
base = []
for i in range(512):
    k = os.urandom(32)
    m = os.urandom(32)
    base.append((nat.ec_pubkey_create(k, True), nat.ec_sign(k, m), m))
items = (base * (4 * n // len(base) + 1))[:4 * n]
print(f"generated {len(base)} unique sigs in {time.time()-t:.1f}s", flush=True)
out = {"n": n}
r, ms = nat.ecdsa_verify_batch(items[:2000], use_gpu=False, threads=os.cpu_count() or 8)
out["cpu_sig_per_s"] = 2000 / ms * 1e3
assert all(r)
if b.gpu_available():
    nat.ecdsa_verify_batch(items[:256], use_gpu=True)  # warm-up (table upload, code load)
    for size in (1024, 8192, n, 4 * n):
        r, ms = nat.ecdsa_verify_batch(items[:size], use_gpu=True, threads=min(16, os.cpu_count() or 8))
        assert all(r), "GPU rejected a valid signature"
        out[f"gpu_sig_per_s_{size}"] = size / ms * 1e3
print(json.dumps(out))
