#!/bin/bash
# BASELINE.md secondary metrics on one GPU: Equihash (48,5) latency, (200,9) verify and solve,
# bench_bcp GPU/CPU batches (SHA256d, merkle, 8 MB block connect). Usage: bash tools/baseline_check.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
timeout -k 10 300 python -u tools/baseline_metrics.py > "$O/metrics.log" 2>&1
grep '^{' "$O/metrics.log" | cut -c1-220
timeout -k 10 300 bin/bench_bcp -filter="ConnectBlock8MB.*|GPU_.*|CPU_MerkleRoot.*|CPU_SHA256d64.*" -time=3 > "$O/bench_bcp.log" 2>&1
tail -n 20 "$O/bench_bcp.log"
