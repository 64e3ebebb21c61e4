#!/bin/bash
# Pipelined generation that starts after round R of the other batch (BCP_EH_PIPE_ROUND=R), with a
# persistent one-workgroup-per-CU generation (ab/gp1h1, ab/gp1h2), against the default launch
# order (ab/base). Run on the GPU box: bash tools/eh_piperound_ab.sh TAG REPS
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
TAG=${1:-pr}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
B="ab/base/$EXT"
for b in gp1h1 gp1h2; do for r in 2 3; do B="$B ab/$b/$EXT@BCP_EH_PIPELINE=1,BCP_EH_PIPE_ROUND=$r"; done; done
timeout -k 10 900 python -u tools/ab_bench.py --reps "${2:-4}" $B > "$O/ab.log" 2>&1
tail -n 1 "$O/ab.log"
for b in gp1h1 gp1h2; do
  (cd /tmp && BCP_EH_PIPELINE=1 BCP_EH_PIPE_ROUND=2 BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 200 rocprofv3 --kernel-trace \
    --output-format csv -d "$O/$b" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 > "$O/$b.log" 2>&1)
  python3 tools/eh_timeline.py "$O/$b" 48 > "$O/$b.txt"
done
echo DONE
