#!/bin/bash
# Interleaved A/B of the Equihash solver builds under ab/*/ on one GPU: serial per-batch timing
# (tools/eh_serial.py) and the headline bench (tools/ab_bench.py, REPS interleaved runs each).
# Usage (gpurun): bash tools/eh_ab.sh TAG [REPS]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
REPS=${2:-3}
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  BCP_NATIVE_PATH=$PWD/ab/$b/$EXT timeout -k 10 100 python3 tools/eh_serial.py > "$O/ser_$b.log" 2>&1
  echo "$b $(tail -n 1 "$O/ser_$b.log")"
done
timeout -k 10 600 python -u tools/ab_bench.py --reps "$REPS" ab/*/$EXT > "$O/ab.log" 2>&1
tail -n 1 "$O/ab.log"
