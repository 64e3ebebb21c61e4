#!/usr/bin/env python3
"""Per-kernel time table from rocprofv3 rocpd databases (the default `--kernel-trace` output).

python tools/rocpd_stats.py A/k_results.db [B/k_results.db ...]
One column of average microseconds per database, kernels matched by (shortened) name.
"""
import re
import sqlite3
import sys


def short(name):
    """'void bcpk::eh_round<bcpk::EhCfg<200, 9, ...>, 3, true>(...)' -> 'eh_round<200,9><3,true>'."""
    head = name.split("(")[0].replace("void ", "")
    m = re.match(r"(?:\w+::)*(\w+)<(.*)>$", head)
    if not m:
        return head[:60]
    fn, args = m.groups()
    cfg = re.match(r"(?:\w+::)*\w+<(\d+), (\d+)[^>]*>(.*)", args)
    if not cfg:
        return "%s<%s>" % (fn, args[:40])
    rest = cfg.group(3).strip(", ")
    return "%s<%s,%s>%s" % (fn, cfg.group(1), cfg.group(2), "<%s>" % rest.replace(" ", "") if rest else "")


def load(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels").fetchall()
    agg = {}
    for n, d in rows:
        k = short(n)
        s = agg.setdefault(k, [0, 0.0])
        s[0] += 1
        s[1] += d
    return agg


def main():
    dbs = sys.argv[1:]
    aggs = [load(d) for d in dbs]
    keys = sorted(set().union(*aggs), key=lambda k: -max(a.get(k, [0, 0])[1] for a in aggs))
    print("| kernel | " + " | ".join("%s calls / avg us / total ms" % d for d in dbs) + " |")
    print("|---" * (len(dbs) + 1) + "|")
    for k in keys:
        cells = []
        for a in aggs:
            n, t = a.get(k, [0, 0.0])
            cells.append("%d / %.1f / %.2f" % (n, t / n / 1e3 if n else 0, t / 1e6))
        print("| %s | %s |" % (k, " | ".join(cells)))


if __name__ == "__main__":
    main()
