#!/usr/bin/env python3
"""Per-phase cycles of the (200,9) round kernels at the bench's batch (stamp instantiation).

python tools/eh_phases.py [--batch 48]   (BCP_NATIVE_PATH selects a build)
Columns: s_memtime cycles per bucket between the phase stamps of eh_round (see
EquihashGpuSolver::PhaseCycles): total, commit, issue+barrier, key sort, pairs, claim+pair sort,
emit, and the pair phase split into listing and filtering.
"""
import argparse
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=48)
    a = ap.parse_args()
    from bitcoincashplus_amd import native
    s = native.EquihashGpuSolver(200, 9, a.batch)
    s.set_stamp_mode(True)
    header = bytes((i * 37 + 11) & 0xFF for i in range(108))
    sts = []
    for i in range(a.batch):
        st = native.EquihashState(200, 9)
        st.update(header + struct.pack("<QQQQ", i, 0, 0, 9))
        sts.append(st)
    for _ in range(3):
        s.solve(sts)
    names = ["total", "commit", "issue", "keysort", "pairs", "claim_sort", "emit", "pairs_list", "pairs_filter"]
    for stage, ph in enumerate(s.phase_cycles(a.batch)):
        print(json.dumps({"round": stage + 1, **{n: round(v) for n, v in zip(names, ph)}}), flush=True)


if __name__ == "__main__":
    main()
