#!/bin/bash
# Block-connect GPU path on one MI355X: 8 MB connects (P2PKH, 160k-sigop worst case, 2-of-3
# multisig) CPU vs GPU, and the IBD pipeline (consecutive 7.5 MB blocks, one at a time vs
# pipelined). Usage: gpurun --timeout 1100 -- 'bash tools/r3_connect.sh TAG [IBDBLOCKS]'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-connect}
mkdir -p "$OUT"
N=${2:-50}
timeout -k 10 420 ./bin/bench_bcp -filter='ConnectBlock8MB.*' -time=4 > "$OUT/connect.log" 2> "$OUT/connect.err"
cat "$OUT/connect.log"; grep '^#' "$OUT/connect.err" | tail -12
timeout -k 10 600 ./bin/bench_bcp -filter='IbdPipeline_(Seq|Pipe)_GPU' -ibdblocks=$N -time=0 > "$OUT/ibd.log" 2> "$OUT/ibd.err"
cat "$OUT/ibd.log"; tail -3 "$OUT/ibd.err"
echo DONE
