#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace (.db from rocpd, or kernel_trace.csv) into a per-kernel table.

python tools/prof_summary.py <results.db | kernel_trace.csv> [> profiles/xxx.md]
"""
import collections
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"bcpk::EhCfg<200, 9, [^>]*>", "Eh200_9", name)
    name = re.sub(r"bcpk::EhCfg<(\d+), (\d+), [^>]*>", r"Eh\1_\2", name)
    name = name.replace("void bcpk::", "").replace("bcpk::", "")
    name = re.sub(r"\(.*\)$", "", name)
    return name[:90]


def rows_from_db(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    q = f"select {name_col}, start, end from kernels"
    for name, s, e in c.execute(q):
        yield name, (e - s)


def rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    path = sys.argv[1]
    it = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    agg = collections.defaultdict(lambda: [0, 0])
    for name, ns in it:
        a = agg[short(name)]
        a[0] += 1
        a[1] += ns
    total = sum(v[1] for v in agg.values())
    print(f"| kernel | calls | total ms | avg us | % |")
    print(f"|---|---|---|---|---|")
    for k, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {n} | {ns / 1e6:.3f} | {ns / n / 1e3:.1f} | {100 * ns / total:.1f} |")
    print(f"\ntotal GPU kernel time: {total / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
