#!/bin/bash
# Generation and rounds on disjoint CU sets (BCP_EH_GEN_CUS): per-kernel times of the serial
# solver with the split, then the headline with and without pipelined launches per split.
#   bash tools/eh_cusplit.sh TAG "0 64" "0 48 64 80 96"
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cusplit}
mkdir -p "$O"
export TMPDIR=/tmp
for G in ${2:-0 64}; do
  (cd /tmp && BCP_EH_GEN_CUS=$G timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/ser_$G" -o k -- \
    python3 "$R/tools/eh_serial.py" --iters 5 > "$O/ser_$G.log" 2>&1)
  echo "serial G=$G $(grep ms_per_batch "$O/ser_$G.log" | tail -n 1)"
done
cd "$R"
for G in ${3:-0 48 64 80 96}; do
  for P in 0 1; do
    BCP_EH_GEN_CUS=$G timeout -k 10 150 python3 bench.py --pipeline $P --steps 20 --warmup 3 > "$O/b_${G}_p$P.log" 2>&1
    echo "G=$G pipeline=$P $(tail -n 1 "$O/b_${G}_p$P.log" | grep -o '"value": [0-9.]*')"
  done
done
