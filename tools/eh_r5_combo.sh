#!/bin/bash
# Round-5 combined GPU call: invalid-solution hunt (2 solvers in flight) over the ab/ builds named
# in $HUNT, then the interleaved headline A/B of the builds named in $AB (BCP_EH_PIPELINE=0).
#   HUNT="np7 np9" AB="base np9 np9r0" bash tools/eh_r5_combo.sh TAG BATCHES REPS
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-combo}
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $HUNT; do
  BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 280 python3 -u tools/eh_invalid_hunt.py --batches "${2:-300}" --solvers 2 \
    --json "$O/hunt_$b.json" > "$O/hunt_$b.log" 2>&1
  echo "hunt $b $(tail -n 1 "$O/hunt_$b.log")"
done
B=""
for b in $AB; do B="$B ab/$b/$EXT@BCP_EH_PIPELINE=0"; done
if [ -n "$B" ]; then
  timeout -k 10 900 python -u tools/ab_bench.py --reps "${3:-8}" $B > "$O/ab.log" 2>&1 || { tail -n 3 "$O/ab.log"; exit 1; }
  python3 - "$O/ab.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"median'):
        for k, v in json.loads(l)["summary"].items():
            print(k.split("/")[1], round(v["median"], 1), round(v["min"], 1), round(v["max"], 1))
PY
fi
echo DONE
