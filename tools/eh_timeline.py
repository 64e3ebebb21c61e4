#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of the Equihash bench: per-kernel busy time, how much of
each kernel class ran concurrently with another stream's kernels, and the wall time of the
traced region. Usage: eh_timeline.py <rocprofv3 output dir>"""
import collections
import csv
import glob
import sys


def main(d, seq=0):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not files:
        print("no kernel_trace.csv under", d)
        return
    ks = []
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            short = name.split("<")[0].split("(")[0].replace("void ", "").split("::")[-1]
            if "eh_round" in name:
                short = "eh_round<" + name.split("EhCfg<")[1].split(">,")[1].split(",")[0].strip() + ">"
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id")), short))
    ks.sort()
    eh = [k for k in ks if k[3].startswith("eh_")]
    if not eh:
        print("no eh_ kernels")
        return
    t0, t1 = eh[0][0], max(k[1] for k in eh)
    busy = collections.defaultdict(float)
    over = collections.defaultdict(float)
    cnt = collections.Counter()
    for i, (s, e, st, nm) in enumerate(eh):
        busy[nm] += (e - s) / 1e6
        cnt[nm] += 1
        # time of this kernel overlapped by kernels of other streams
        ov = 0
        for (s2, e2, st2, nm2) in eh:
            if st2 != st and s2 < e and e2 > s:
                ov += min(e, e2) - max(s, s2)
        over[nm] += min(ov, e - s) / 1e6
    # union of busy intervals
    union, cur_s, cur_e = 0, None, None
    for s, e, _, _ in eh:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    wall = (t1 - t0) / 1e6
    print(f"traced region {wall:.2f} ms, GPU busy (union) {union/1e6:.2f} ms, streams {sorted(set(k[2] for k in eh))}")
    print(f"{'kernel':16s} {'calls':>6s} {'avg ms':>8s} {'total ms':>9s} {'overlapped ms':>14s}")
    for nm in sorted(busy, key=lambda n: (n[:8], n)):
        print(f"{nm:16s} {cnt[nm]:6d} {busy[nm]/cnt[nm]:8.3f} {busy[nm]:9.2f} {over[nm]:14.2f}")
    if seq:
        # the last `seq` solver kernels: start offset, duration, stream (interleaving of the solvers)
        tail = eh[-seq:]
        b = tail[0][0]
        print(f"{'start us':>9s} {'end us':>9s} {'dur us':>8s} stream kernel")
        for s, e, st, nm in tail:
            print(f"{(s - b) / 1e3:9.1f} {(e - b) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {st:>6} {nm}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
