#!/bin/bash
# Kernel timeline of the double-buffered Equihash(200,9) bench on one MI355X: which kernels of
# the two solvers overlap. Usage: gpurun --timeout 600 -- 'bash tools/r3_eh_trace.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ehtrace}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 6 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
cd "$GRAFT_REPO_ROOT" && python3 tools/eh_timeline.py "$OUT/prof" | tee "$OUT/timeline.txt"
echo DONE
