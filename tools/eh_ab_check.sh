#!/bin/bash
# A/B check of two solver builds (ab/base, ab/new): GPU tests, CPU cross-checks, serial
# timing, rocprof kernel traces, interleaved bench, phase stamps. Usage: bash tools/eh_ab_check.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 250 python -u -m pytest tests/test_equihash.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/t.log 2>&1
tail -n 1 $O/t.log
timeout -k 10 120 python -u tools/eh_crosscheck.py --n 96 --k 5 --nonces 16 > $O/x96.log 2>&1
timeout -k 10 120 python -u tools/eh_crosscheck.py --n 48 --k 5 --nonces 16 > $O/x48.log 2>&1
timeout -k 10 240 python -u tools/eh_crosscheck.py --nonces 8 > $O/x200.log 2>&1
grep -h -o '"cpu_total": [0-9]*, "gpu_total": [0-9]*, "missing": [0-9]*, "extra": [0-9]*' $O/x*.log
for b in $(ls ab); do BCP_NATIVE_PATH=$PWD/ab/$b/_bcpnative.cpython-310-x86_64-linux-gnu.so timeout -k 10 100 python3 tools/eh_serial.py > $O/ser_$b.log 2>&1; tail -n 1 $O/ser_$b.log; done
cd /tmp
for b in $(ls ab); do BCP_NATIVE_PATH=$GRAFT_REPO_ROOT/ab/$b/_bcpnative.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/p_$b -o k -- python3 $GRAFT_REPO_ROOT/tools/eh_serial.py > $GRAFT_REPO_ROOT/$O/prof_$b.log 2>&1; done
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/ab_bench.py --reps 3 ab/*/_bcpnative.cpython-310-x86_64-linux-gnu.so > $O/ab.log 2>&1
tail -n 1 $O/ab.log
BCP_NATIVE_PATH=$PWD/ab/new/_bcpnative.cpython-310-x86_64-linux-gnu.so EH_PHASES=1 timeout -k 10 120 python -u tools/eh_diag.py > $O/phases_new.log 2>&1
tail -n 3 $O/phases_new.log
