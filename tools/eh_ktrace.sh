#!/bin/bash
# Per-kernel durations of each solver build under ab/ (serial solver, rocprofv3 --kernel-trace --stats).
# Usage (gpurun): bash tools/eh_ktrace.sh TAG   ->  gpurun_out/TAG/<build>/k_kernel_stats.csv
set -e
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  (cd /tmp && BCP_NATIVE_PATH=$GRAFT_REPO_ROOT/ab/$b/$EXT timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/$b" -o k -- python3 "$GRAFT_REPO_ROOT/tools/eh_serial.py" --iters 5 > "$O/$b.log" 2>&1)
  echo "$b $(tail -n 1 "$O/$b.log")"
done
