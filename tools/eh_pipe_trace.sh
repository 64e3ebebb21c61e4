#!/bin/bash
# Kernel timelines of every ab/ build with pipelined launches (BCP_EH_PIPELINE=1): shows whether
# one batch's generation runs beside the other batch's rounds. Run on the GPU box:
#   bash tools/eh_pipe_trace.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ptrace}
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  (cd /tmp && BCP_EH_PIPELINE=1 BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
    -d "$O/$b" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 > "$O/$b.log" 2>&1)
  python3 tools/eh_timeline.py "$O/$b" 48 > "$O/$b.txt"
  head -n 14 "$O/$b.txt"
done
echo DONE
