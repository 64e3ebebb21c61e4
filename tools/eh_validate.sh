#!/bin/bash
# Correctness gate for a solver change (in-tree build): the Equihash GPU tests and a CPU-solver
# cross-check of (200,9), then the interleaved A/B of the builds under ab/ (tools/eh_ab.sh).
# Usage (gpurun): bash tools/eh_validate.sh TAG [REPS]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_equihash.py -x -q -m gpu --timeout 200 --timeout-method thread > "$O/t.log" 2>&1 || { tail -n 30 "$O/t.log"; exit 1; }
tail -n 1 "$O/t.log"
timeout -k 10 240 python -u tools/eh_crosscheck.py --nonces 8 > "$O/x200.log" 2>&1
tail -n 2 "$O/x200.log"
bash tools/eh_ab.sh "$1" "${2:-3}"
