#!/usr/bin/env python3
"""Per-kernel table of the PMC counters collected by tools/pmc_eh.sh.

python tools/pmc_table.py gpurun_out/pmc [> profiles/xxx.md]
Values are summed over the profiled dispatches of each kernel; 'per bucket' columns divide by
the number of (nonce, bucket) work items of a round (batch * NB * dispatches).
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
    for k in ("eh_gen", "eh_expand", "eh_verify"):
        if k in name:
            return k
    return re.sub(r"\(.*", "", name)[:40]


def main():
    d = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/*/*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            agg[kname(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    cols = sorted({c for v in agg.values() for c in v})
    print("| kernel | " + " | ".join(cols) + " |")
    print("|---" * (len(cols) + 1) + "|")
    for k in sorted(agg):
        print(f"| {k} | " + " | ".join("%.3g" % agg[k].get(c, 0) for c in cols) + " |")


if __name__ == "__main__":
    main()
