#!/usr/bin/env python3
"""Median / min / max of the per-run IBD ms/block lines bench_bcp prints (IbdPipelineRun)."""
import glob
import json
import statistics
import sys

for f in sorted(glob.glob(sys.argv[1] + "/ibd_*.log")):
    v = [json.loads(l)["ms_per_block"] for l in open(f) if '"IbdPipelineRun"' in l]
    if v:
        print(json.dumps({"file": f.split("/")[-1], "runs": len(v), "median": statistics.median(v), "min": min(v),
                          "max": max(v), "values": v}))
