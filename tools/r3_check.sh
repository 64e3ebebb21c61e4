#!/bin/bash
# Round-3 GPU round-trip: gpu tests, smoke, bench (1 GPU and the --gpus launcher path),
# solver recall vs the CPU reference.
# Usage: gpurun --timeout 1100 -- 'bash tools/r3_check.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -3 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
timeout -k 10 300 python -u tools/eh_recall.py --nonces 32 --threads 16 --json "$OUT/recall.json" > "$OUT/recall.log" 2>&1
tail -4 "$OUT/recall.log"
if [ "${2:-}" = "prof" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
  cd "$GRAFT_REPO_ROOT"
  tail -1 "$OUT/prof.log"
fi
echo DONE
