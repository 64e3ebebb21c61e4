#!/bin/bash
# CPU ECDSA (GLV ecmult, addition-chain field inverse/sqrt, Jacobian x check) on the GPU box's
# quiet CPUs, and the CPU-pool vs MI355X batch crossover. Usage: gpurun -- 'bash tools/r3_ecdsa_cpu.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ecdsacpu}
mkdir -p "$OUT"
timeout -k 10 120 ./bin/bench_bcp -filter='ECDSAVerify_CPU|Ecmult_CPU.*' -time=3 > "$OUT/cpu.log" 2>&1
cat "$OUT/cpu.log"
timeout -k 10 300 python tools/ecdsa_crossover.py 16 > "$OUT/crossover.log" 2>&1
tail -3 "$OUT/crossover.log"
timeout -k 10 300 ./bin/bench_bcp -filter='ConnectBlock8MB_CPU' -time=3 > "$OUT/connect_cpu.log" 2> "$OUT/connect_cpu.err"
cat "$OUT/connect_cpu.log"; grep '^#' "$OUT/connect_cpu.err" | tail -2
echo DONE
