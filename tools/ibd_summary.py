#!/usr/bin/env python3
"""Median / min / max of the per-run IBD ms/block lines bench_bcp prints (IbdPipelineRun), per
log file and, within an -ibdab log, per configuration (in_place, lookahead)."""
import collections
import glob
import json
import statistics
import sys

for f in sorted(glob.glob(sys.argv[1] + "/ibd_*.log")):
    groups = collections.defaultdict(list)
    for line in open(f):
        if '"IbdPipelineRun"' not in line:
            continue
        r = json.loads(line)
        groups[(r.get("in_place"), r.get("lookahead"))].append(r["ms_per_block"])
    for (inplace, la), v in sorted(groups.items(), key=str):
        print(json.dumps({"file": f.split("/")[-1], "in_place": inplace, "lookahead": la, "runs": len(v),
                          "median": statistics.median(v), "min": min(v), "max": max(v), "values": v}))
