#!/bin/bash
# Run tools/eh_invalid_hunt.py over every ab/ build (GPU box): bash tools/eh_hunt.sh TAG BATCHES
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-hunt}
mkdir -p "$O"
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  BCP_NATIVE_PATH=$GRAFT_REPO_ROOT/ab/$b/$EXT timeout -k 10 280 python3 -u tools/eh_invalid_hunt.py --batches "${2:-64}" \
    --json "$O/$b.json" > "$O/$b.log" 2>&1
  echo "$b $(tail -n 1 "$O/$b.log")"
done
echo DONE
