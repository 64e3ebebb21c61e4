#!/usr/bin/env python3
"""Per-kernel HBM bytes and achieved bandwidth from tools/pmc_bw.sh output.

python tools/pmc_bw.py gpurun_out/TAG [> profiles/xxx.md]
FETCH_SIZE / WRITE_SIZE are rocprofv3's derived TCC counters in KiB (bytes the L2 moved to or
from memory); durations come from the counter-free kernel-trace pass.
"""
import collections
import csv
import glob
import re
import sys


def kname(name):
    m = re.search(r"eh_round<[^>]*>, (\d+), (?:false|true)>", name)
    if m:
        return "eh_round<%s>" % m.group(1)
    for k in ("eh_gen_reg", "eh_gen", "eh_expand", "eh_verify"):
        if k in name:
            return k
    return re.sub(r"\(.*", "", name)[:40]


def main():
    d = sys.argv[1]
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{d}/t/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("f", "w"):
        for f in glob.glob(f"{d}/{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                ctr[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | dispatches | avg ms | read MB | write MB | read+write GB/s |")
    print("|---|---|---|---|---|---|")
    tot_b = tot_t = 0.0
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        if not k.startswith("eh_"):
            continue
        t = sum(dur[k]) / len(dur[k])
        rd = ctr[k].get("FETCH_SIZE", [0])
        wr = ctr[k].get("WRITE_SIZE", [0])
        rb = sum(rd) / len(rd) * 1024
        wb = sum(wr) / len(wr) * 1024
        tot_b += rb + wb
        tot_t += t
        print(f"| {k} | {len(dur[k])} | {t * 1e3:.3f} | {rb / 1e6:.0f} | {wb / 1e6:.0f} | {(rb + wb) / t / 1e9:.0f} |")
    if tot_t:
        print(f"\nall solver kernels: {tot_b / 1e9:.2f} GB in {tot_t * 1e3:.2f} ms per batch = {tot_b / tot_t / 1e12:.2f} TB/s")


if __name__ == "__main__":
    main()
