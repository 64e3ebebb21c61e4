#!/bin/bash
# 8 MB connect benches on one MI355X plus a kernel-time profile of the 160k-sigop GPU connect.
# Usage: gpurun --timeout 900 -- 'bash tools/r3_connect_prof.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-connprof}
mkdir -p "$OUT"
timeout -k 10 300 ./bin/bench_bcp -filter='ConnectBlock8MB_(160kSigops_)?GPU|ConnectBlock8MB_Multisig_GPU' -time=3 > "$OUT/connect.log" 2> "$OUT/connect.err"
cat "$OUT/connect.log"; grep '^#' "$OUT/connect.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- "$GRAFT_REPO_ROOT/bin/bench_bcp" -filter='ConnectBlock8MB_160kSigops_GPU' -time=2 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
find "$GRAFT_REPO_ROOT/$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
echo DONE
