#!/bin/bash
# Final-round capacity (round 5): recall repeats of each ab/ build on the same 32 nonces (with the
# buckets that overflowed), then an interleaved headline A/B. Run on the GPU box:
#   bash tools/eh_capf_ab.sh TAG REPS
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-capf}
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 300 python -u tools/eh_recall.py --nonces 32 --threads 16 --repeat 4 \
    --json "$O/recall_$b.json" > "$O/recall_$b.log" 2>&1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['gpu_found'], d['repeat_found'], d['stage_dropped_all'], d['overflow_fills'][:12])" "$O/recall_$b.json" "$b"
done
B=""
for b in $(ls ab); do B="$B ab/$b/$EXT"; done
timeout -k 10 900 python -u tools/ab_bench.py --reps "${2:-4}" $B > "$O/ab.log" 2>&1
tail -n 1 "$O/ab.log"
