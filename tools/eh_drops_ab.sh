#!/bin/bash
# Pair/row losses (tools/eh_drops.py) of each ab/ build, then the interleaved headline A/B.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-drops}
mkdir -p "$O"
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 200 python3 -u tools/eh_drops.py --batches "${2:-16}" > "$O/drops_$b.log" 2>&1
  echo "drops $b $(tail -n 1 "$O/drops_$b.log")"
done
AB="$(ls ab)" bash tools/eh_r5_combo.sh "${1:-drops}" 0 "${3:-8}"
