#!/bin/bash
# Round-3 GPU regression pass on one MI355X: the GPU test tier, smoke, the headline bench, and
# the hashing/merkle micro-benches (CPU SHA-NI vs GPU). Usage: gpurun -- 'bash tools/r3_gpu_check.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-gpucheck}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 300 ./bin/bench_bcp -filter='MerkleRoot|SHA256d64|^SHA256$' -time=1 > "$OUT/hash.log" 2>&1
cat "$OUT/hash.log"
echo DONE
