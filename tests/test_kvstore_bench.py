"""bench_bcp KVStoreCoins at CI scale: the chainstate store stays inside its memory budget while
the coin set grows, every inserted coin reads back, absent coins read as absent, and a full scan
sees each coin once. (The 50M-coin run is recorded in profiles/kvstore_r3.md.)"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "bench_bcp")


def test_kvstore_coins_bounded_memory():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-C", ROOT, "-j8", "tools"])
    p = subprocess.run([BIN, "-filter=KVStoreCoins", "-kvcoins=1500000", "-kvdbcache=64", "-time=0"],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    line = next(l for l in p.stdout.splitlines() if l.startswith("{"))
    r = json.loads(line)
    assert r["hits"] == 1000000 and r["misses_absent"] == 1000000
    assert r["scanned"] == 1500000
    assert r["flushes"] > 3 and r["segments"] >= 1
    assert r["within_budget"], r
