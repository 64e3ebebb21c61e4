"""Compile-time lock discipline: `make thread-safety` runs clang's -Wthread-safety analysis over
every CPU source (reference src/threadsafety.h + configure's -Wthread-safety-analysis). The
chainstate (cs_main: block index, active chain, candidates, dirty sets), the mempool (mapTx,
links, deltas, rolling fee state) and the connection manager (vNodes, one-shots, added nodes,
outbound accounting) carry GUARDED_BY / EXCLUSIVE_LOCKS_REQUIRED annotations; any violation is
an error. The runtime side (TSan/ASan over the node) is tools/sanitize.sh."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG), reason="clang++ not available")
def test_thread_safety_analysis_clean(tmp_path):
    # a private stamp directory so a stale build/tsa cannot hide anything
    shutil.rmtree(os.path.join(ROOT, "build", "tsa"), ignore_errors=True)
    p = subprocess.run(["make", "-C", ROOT, "-k", "-j8", "thread-safety"], capture_output=True, text=True,
                       timeout=900)
    errors = [l for l in p.stderr.splitlines() if "error:" in l or "warning: " in l and "thread-safety" in l]
    assert p.returncode == 0 and not errors, "\n".join(errors[:40])
