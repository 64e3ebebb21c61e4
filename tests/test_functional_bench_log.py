"""-debug=bench connect timing: every ConnectTip logs its steps with this block's
time and the running total since startup, like the reference's nTimeCheck / nTimeConnect /
nTimeFlush / nTimeChainState / nTimePostConnect / nTimeTotal accumulators
(src/validation.cpp:1690-1700, 2200-2290)."""
import os
import re

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

LINE = re.compile(r"- (Load block from disk|Connect total|Flush|Writing chainstate|Connect postprocess|Connect block|"
                  r"Sanity checks|UTXO pass): ([0-9.]+)ms \[([0-9.]+)s\]")


def test_connect_bench_accumulators(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-debug=bench"])
    n.start()
    try:
        n.rpc.generate(5)
    finally:
        n.stop()
    log = open(os.path.join(n.datadir, "regtest", "debug.log"), errors="replace").read()
    seen = {}
    for what, ms, tot in LINE.findall(log):
        seen.setdefault(what, []).append((float(ms), float(tot)))
    for what in ("Load block from disk", "Connect total", "Flush", "Writing chainstate", "Connect postprocess",
                 "Connect block", "Sanity checks"):
        assert len(seen.get(what, [])) >= 5, what
    blocks = seen["Connect block"]
    totals = [t for _, t in blocks]
    assert totals == sorted(totals)  # running totals never decrease
    # the total grows by each block's own time (rounding of the printed values aside)
    assert abs(totals[-1] - totals[-2] - blocks[-1][0] / 1000.0) < 0.01
