#!/bin/bash
# Slim Equihash A/B of two solver builds (ab/base, ab/new): (200,9) cross-check of the new build
# against the CPU solver, serial batch timing of both, interleaved bench medians.
# Usage: gpurun -- 'bash tools/r3_eh_ab.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ehab}
mkdir -p "$O"
NEW=$PWD/ab/new/_bcpnative.cpython-310-x86_64-linux-gnu.so
BCP_NATIVE_PATH=$NEW timeout -k 10 240 python -u tools/eh_crosscheck.py --nonces 8 > "$O/x200.log" 2>&1
BCP_NATIVE_PATH=$NEW timeout -k 10 120 python -u tools/eh_crosscheck.py --n 96 --k 5 --nonces 16 > "$O/x96.log" 2>&1
grep -h -o '"cpu_total": [0-9]*, "gpu_total": [0-9]*, "missing": [0-9]*, "extra": [0-9]*' "$O"/x*.log
for b in base new; do BCP_NATIVE_PATH=$PWD/ab/$b/_bcpnative.cpython-310-x86_64-linux-gnu.so timeout -k 10 100 python3 tools/eh_serial.py > "$O/ser_$b.log" 2>&1; echo "$b: $(tail -n 1 "$O/ser_$b.log")"; done
timeout -k 10 400 python -u tools/ab_bench.py --reps 3 ab/base/_bcpnative.cpython-310-x86_64-linux-gnu.so ab/new/_bcpnative.cpython-310-x86_64-linux-gnu.so > "$O/ab.log" 2>&1
tail -n 2 "$O/ab.log"
echo DONE
