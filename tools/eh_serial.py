#!/usr/bin/env python3
"""One Equihash(200,9) GPU solver, batches solved back to back (no double buffering), so a
`rocprofv3 --kernel-trace` of it gives each kernel's own time, not time shared with the other
solver of bench.py.

python tools/eh_serial.py [--batch 32] [--iters 10]
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
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from bitcoincashplus_amd import native

    sv = native.EquihashGpuSolver(200, 9, a.batch, 0)
    header = bytes((i * 37 + 11) & 0xFF for i in range(108))

    def states(step):
        out = []
        for b in range(a.batch):
            st = native.EquihashState(200, 9)
            st.update(header + struct.pack("<QQQQ", step * a.batch + b, 0, 0, 7))
            out.append(st)
        return out

    sv.solve(states(10_000))
    batches = [states(i) for i in range(a.iters)]
    t0 = time.perf_counter()
    nsol = 0
    for b in batches:
        nsol += sum(len(x) for x in sv.solve(b))
    dt = time.perf_counter() - t0
    n = a.iters * a.batch
    print(json.dumps({"batch": a.batch, "iters": a.iters, "ms_per_batch": round(1e3 * dt / a.iters, 3),
                      "nonces_per_sec": round(n / dt, 1), "sol_per_sec": round(nsol / dt, 1)}))


if __name__ == "__main__":
    main()
