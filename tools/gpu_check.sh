#!/bin/bash
# One GPU round-trip: gpu tests, smoke, bench, rocprof kernel stats.
# Usage (from this container): gpurun --timeout 900 -- 'bash tools/gpu_check.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench -- python3 bench.py --steps 5 --warmup 1 > "$OUT/prof.log" 2>&1
echo DONE
