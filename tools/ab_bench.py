#!/usr/bin/env python3
"""A/B the headline bench between builds of the native extension, interleaved on one GPU.

python tools/ab_bench.py [--reps 3] [--steps 20] A.so B.so ...
Each build is loaded through BCP_NATIVE_PATH (bitcoincashplus_amd/_native.py) in its own
process; runs alternate A, B, A, B, ... so clock/thermal drift hits every build alike.
Prints one JSON line per run and a summary per build: median, min, max and the relative
spread ((max - min) / median), so a difference smaller than the spread is read as noise.
A build may carry environment settings for its runs: path.so@NAME=VALUE,NAME2=VALUE2
(e.g. the same build with BCP_EH_PIPELINE=0 and =1).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("builds", nargs="+")
    a = ap.parse_args()
    res = {b: [] for b in a.builds}
    for r in range(a.reps):
        for b in a.builds:
            path, _, extra = b.partition("@")
            env = dict(os.environ, BCP_NATIVE_PATH=os.path.abspath(path))
            for kv in filter(None, extra.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps),
                                  "--warmup", str(a.warmup)], env=env, capture_output=True, text=True,
                                 timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if out.returncode != 0 or not line:
                print(json.dumps({"build": b, "rep": r, "error": out.stderr[-400:]}), flush=True)
                sys.exit(1)
            v = json.loads(line[-1])
            res[b].append(v["value"])
            print(json.dumps({"build": b, "rep": r, "value": v["value"], "ms_per_step": v["ms_per_step"],
                              "sol_per_nonce": v["config"]["solutions_per_nonce"]}), flush=True)
    summary = {b: {"median": statistics.median(v), "min": min(v), "max": max(v),
                   "spread": (max(v) - min(v)) / statistics.median(v), "n": len(v)} for b, v in res.items()}
    print(json.dumps({"median": {b: s["median"] for b, s in summary.items()}, "summary": summary}))


if __name__ == "__main__":
    main()
