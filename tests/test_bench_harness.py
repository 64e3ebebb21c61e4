"""Native micro-benchmark harness (reference src/bench): every registered bench runs and
reports; DeserializeAndCheckBlockTest parses the reference's block413567.raw (legacy
80-byte header) and passes CheckBlock under mainnet rules."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "bench_bcp")


def test_bench_list_and_run(tmp_path):
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-C", ROOT, "-j8", "tools"])
    names = subprocess.run([BIN, "-list"], capture_output=True, text=True, check=True).stdout.split()
    for want in ["SHA256", "Base58Decode", "DeserializeAndCheckBlockTest", "CoinSelection", "MempoolEviction",
                 "LockedPool", "RollingBloom", "CCheckQueueSpeed", "CCoinsCaching"]:
        assert want in names
    out = subprocess.run([BIN, "-time=0.02", "-filter=(SHA256|Deserialize.*|CoinSelection|LockedPool|MempoolEviction)"],
                         capture_output=True, text=True, check=True, cwd=str(tmp_path), timeout=300).stdout
    rows = [l.split() for l in out.splitlines() if l and not l.startswith("#")]
    got = {r[0]: int(r[1]) for r in rows}
    assert set(got) >= {"SHA256", "DeserializeBlockTest", "DeserializeAndCheckBlockTest", "CoinSelection",
                        "LockedPool", "MempoolEviction"}
    assert all(v > 0 for v in got.values())
