#!/bin/bash
# Pipelined-launch A/B (round 5): the same builds with BCP_EH_PIPELINE=0/1, interleaved, plus a
# kernel timeline of each build with pipelined launches (tools/eh_pipe_trace.sh). Run on the GPU box: bash tools/eh_pipe_ab.sh TAG REPS
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
TAG=${1:-pipe}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 > "$O/smoke_bench.log" 2>&1
tail -n 1 "$O/smoke_bench.log" | cut -c1-200
B=""
for b in $(ls ab); do B="$B ab/$b/$EXT@BCP_EH_PIPELINE=1"; done
B="$B ab/base/$EXT@BCP_EH_PIPELINE=0"
timeout -k 10 900 python -u tools/ab_bench.py --reps "${2:-6}" $B > "$O/ab.log" 2>&1
tail -n 1 "$O/ab.log"
bash tools/eh_pipe_trace.sh "$TAG/trace"
