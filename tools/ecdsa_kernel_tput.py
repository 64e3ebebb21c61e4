"""Device-only ECDSA verify throughput: the kernels of ops.ecdsa_verify_compact on tensors that
already sit on the GPU (no host parse, no copies), timed with HIP events, best of REPS.

For each batch size it times the three device paths:
  fused    ecdsa_fused_kernel (ecdsa_set_fused_max(huge))
  split8   ecdsa_prep_kernel + ecdsa_verify_kernel (8 x 32 field)
  split10  ecdsa_prep_kernel + ecdsa_verify10_kernel (10 x 26 field, global-z table) for whole
           rounds of the device and ecdsa_verify10h_kernel (one GLV half per lane) for the rest
  split10-1lane  the one-lane kernel for the whole batch
and checks that every signature verified. One JSON line per (n, path), then a summary line.
Usage: python tools/ecdsa_kernel_tput.py [n ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bitcoincashplus_amd as b  # noqa: E402
from bitcoincashplus_amd.utils import secp256k1_ref as ref  # noqa: E402

nat = b.native
sizes = [int(a) for a in sys.argv[1:]] or [4096, 32768, 65536, 131072, 199680, 262144, 1048576]
REPS = 3


def compact(der):
    rlen = der[3]
    r = int.from_bytes(der[4:4 + rlen], "big")
    off = 4 + rlen
    s = int.from_bytes(der[off + 2:off + 2 + der[off + 1]], "big")
    if s > ref.N // 2:
        s = ref.N - s
    return r.to_bytes(32, "big") + s.to_bytes(32, "big")


base_m, base_s, base_p = [], [], []
for i in range(1024):
    k = os.urandom(32)
    m = os.urandom(32)
    base_m.append(m)
    base_s.append(compact(nat.ec_sign(k, m)))
    base_p.append(nat.ec_pubkey_create(k, True))
nmax = max(sizes)
rep = nmax // 1024 + 1
dev = torch.device("cuda:0")
M = torch.frombuffer(bytearray(b"".join(base_m) * rep), dtype=torch.uint8)[: nmax * 32].to(dev)
S = torch.frombuffer(bytearray(b"".join(base_s) * rep), dtype=torch.uint8)[: nmax * 64].to(dev)
P = torch.frombuffer(bytearray(b"".join(base_p) * rep), dtype=torch.uint8)[: nmax * 33].to(dev)
jobs = torch.empty(nmax * nat.ecdsa_job_bytes(), dtype=torch.uint8, device=dev)
out = torch.empty(nmax, dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream().cuda_stream
fused0, split0 = nat.ecdsa_fused_max(), nat.ecdsa_split_kernel()
paths = {"fused": (1 << 40, split0), "split8": (0, 0), "split10": (0, 1), "split10-1lane": (0, 2)}
rows = []
try:
    for n in sizes:
        for name, (fmax, sk) in paths.items():
            nat.ecdsa_set_fused_max(fmax)
            nat.ecdsa_set_split_kernel(sk)
            best = 1e30
            for r in range(REPS + 1):
                out.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                nat.ecdsa_verify_device(M.data_ptr(), S.data_ptr(), P.data_ptr(), jobs.data_ptr(), out.data_ptr(), n,
                                        0, stream)
                e1.record()
                torch.cuda.synchronize()
                if r:  # the first run loads code and the generator table
                    best = min(best, e0.elapsed_time(e1))
            good = int(out[:n].sum().item())
            row = {"n": n, "path": name, "ms": round(best, 3), "msig_per_s": round(n / best / 1e3, 2), "valid": good}
            print(json.dumps(row), flush=True)
            assert good == n, row
            rows.append(row)
finally:
    nat.ecdsa_set_fused_max(fused0)
    nat.ecdsa_set_split_kernel(split0)
print(json.dumps({"rows": rows}))
