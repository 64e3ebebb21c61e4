#!/bin/bash
# Serial rocprof kernel trace and per-phase stamps of every build in ab/ (timing experiments
# that produce no valid solutions are fine here). Usage (GPU box): bash tools/eh_prof_builds.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
    (cd /tmp && BCP_NATIVE_PATH=$GRAFT_REPO_ROOT/ab/$b/$EXT timeout -k 10 120 rocprofv3 --kernel-trace \
        -d "$GRAFT_REPO_ROOT/$O/p_$b" -o k -- python3 "$GRAFT_REPO_ROOT/tools/eh_serial.py" > "$GRAFT_REPO_ROOT/$O/prof_$b.log" 2>&1)
    BCP_NATIVE_PATH=$PWD/ab/$b/$EXT EH_PHASES=1 timeout -k 10 120 python -u tools/eh_diag.py > "$O/phases_$b.log" 2>&1
    echo "== $b"; grep '"round"' "$O/phases_$b.log" | head -n 9
done
