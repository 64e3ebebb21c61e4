#!/bin/bash
# Headline sweep over (batch, solvers in flight); 640 nonces timed per point. Usage: bash tools/eh_sweep.sh TAG "B:S B:S ..."
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
for p in $2; do
    B=${p%:*}; S=${p#*:}
    timeout -k 10 150 python3 bench.py --batch $B --solvers $S --steps $((640 / B)) --warmup $((S + 1)) > "$O/b${B}_s${S}.log" 2>&1
    echo "batch $B solvers $S $(tail -n 1 "$O/b${B}_s${S}.log" | grep -o '"value": [0-9.]*')"
done
