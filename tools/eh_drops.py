#!/usr/bin/env python3
"""Row and pair losses of the (200,9) GPU solver over many nonces: per round, the rows dropped for
LDS capacity (sampled: nonce 0 of each batch) and the pairs dropped when a bucket's pair list
overflowed (every bucket), the same row losses over every nonce, with candidates, duplicates and solutions per nonce.

python tools/eh_drops.py [--batches 8] [--batch 32]
"""
import argparse
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    from bitcoincashplus_amd import native
    header = bytes((i * 37 + 11) & 0xFF for i in range(108))
    solver = native.EquihashGpuSolver(200, 9, a.batch)
    solver.set_debug(True)
    pair_drop = None
    row_drop = None
    sols = 0
    for b in range(a.batches):
        sts = []
        for i in range(a.batch):
            s = native.EquihashState(200, 9)
            s.update(header + struct.pack("<QQQQ", b * a.batch + i, 0, 0, 11))
            sts.append(s)
        sols += sum(len(x) for x in solver.solve(sts))
        st = solver.stats()
        pd, rd = st["pair_dropped"], st["stage_dropped"]
        pair_drop = pd if pair_drop is None else [x + y for x, y in zip(pair_drop, pd)]
        row_drop = rd if row_drop is None else [x + y for x, y in zip(row_drop, rd)]
    st = solver.stats()
    n = a.batches * a.batch
    print(json.dumps({"nonces": n, "solutions_per_nonce": round(sols / n, 4),
                      "pair_dropped_per_round": pair_drop, "rows_dropped_sampled": row_drop,
                      "candidates": st["candidates"], "duplicates": st["duplicates"],
                      # every nonce (accumulated over the run): rows past a round's capacity,
                      # the buckets that overflowed, and final candidates past the list
                      "rows_dropped_all": st.get("stage_dropped_all"),
                      "overflow_buckets": len(st.get("overflow_fills") or []),
                      "overflow_fills_first": [(f >> 32, f & 0xFFFFFFFF) for f in (st.get("overflow_fills") or [])][:32],
                      "cand_max": st.get("cand_max"), "cand_dropped": st.get("cand_dropped")}))


if __name__ == "__main__":
    main()
