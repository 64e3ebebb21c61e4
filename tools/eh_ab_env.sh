#!/bin/bash
# Interleaved headline A/B of every ab/ build (tools/ab_bench.py), each build run with the
# environment given as $3 (e.g. BCP_EH_PIPELINE=0), plus the per-build serial solver timing
# and solutions per nonce (tools/eh_serial.py). Usage on the GPU box:
#   bash tools/eh_ab_env.sh TAG REPS [ENV]
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
TAG=${1:-abenv}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 100 python3 tools/eh_serial.py > "$O/ser_$b.log" 2>&1
  echo "$b $(tail -n 1 "$O/ser_$b.log")"
done
B=""
for b in $(ls ab); do B="$B ab/$b/$EXT@${3:-BCP_EH_PIPELINE=0}"; done
timeout -k 10 900 python -u tools/ab_bench.py --reps "${2:-6}" $B > "$O/ab.log" 2>&1
python3 - "$O/ab.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"median'):
        for k, v in json.loads(l)["summary"].items():
            print(k.split("/")[1], round(v["median"], 1), round(v["min"], 1), round(v["max"], 1))
PY
echo DONE
