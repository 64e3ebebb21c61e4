"""Summarise a rocprofv3 SQLite output (run_results.db) into a per-kernel table.
Usage: python tools/rocpd_summary.py gpurun_out/prof_x/run_results.db [> profiles/x.md]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(top_kernels)")]
rows = db.execute("select * from top_kernels").fetchall()
print("| " + " | ".join(cols) + " |")
print("|" + "---|" * len(cols))
for r in rows:
    print("| " + " | ".join(f"{v:.4g}" if isinstance(v, float) else str(v) for v in r) + " |")
# per-dispatch duration stats (ns) by kernel name
q = """select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start)
       from kernels group by name order by sum(end-start) desc"""
try:
    print("\n| kernel | calls | total_ms | avg_us | min_us | max_us |\n|---|---|---|---|---|---|")
    for name, n, tot, avg, mn, mx in db.execute(q):
        print(f"| {name[:90]} | {n} | {tot/1e6:.3f} | {avg/1e3:.1f} | {mn/1e3:.1f} | {mx/1e3:.1f} |")
except sqlite3.Error as e:
    print("kernels view:", e)
