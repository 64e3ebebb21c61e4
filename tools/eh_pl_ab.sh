#!/bin/bash
# Payload-light rounds (BCP_EH_PL_FROM): per ab/ build named in $PL, the Equihash GPU tests and
# the recall against the CPU solver (32 nonces), then the drops and the interleaved headline A/B of
# every ab/ build.   PL="pl1 pl5" bash tools/eh_pl_ab.sh TAG REPS
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-plab}
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $PL; do
  BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 300 python -u -m pytest tests/test_equihash.py -q -m gpu --timeout 200 \
    --timeout-method thread > "$O/t_$b.log" 2>&1 || true
  echo "tests $b $(tail -n 1 "$O/t_$b.log")"
  BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 300 python3 -u tools/eh_recall.py --nonces 32 --threads 16 \
    --json "$O/recall_$b.json" > "$O/recall_$b.log" 2>&1
  echo "recall $b $(grep -o '"recall": [0-9.]*, "gpu_not_in_cpu": [0-9]*' "$O/recall_$b.log" | tail -n 1)"
done
bash tools/eh_drops_ab.sh "${1:-plab}" 16 "${2:-8}"
