#!/bin/bash
# Per-phase cycle stamps of the round kernels for every build under ab/ (tools/eh_diag.py).
# Usage (gpurun): bash tools/eh_phases.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
for b in $(ls ab); do
  BCP_NATIVE_PATH=$PWD/ab/$b/_bcpnative.cpython-310-x86_64-linux-gnu.so EH_PHASES=1 timeout -k 10 120 python -u tools/eh_diag.py > "$O/ph_$b.log" 2>&1
  echo "== $b"; grep '"round"' "$O/ph_$b.log"
done
