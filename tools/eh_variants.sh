#!/bin/bash
# Compare solver builds ab/*/ on one GPU: per build a CPU cross-check of (200,9) and (96,5)
# solutions, serial batch timing and a rocprof kernel trace of the serial run; then an
# interleaved headline A/B over all builds. Usage (on the GPU box): bash tools/eh_variants.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
if [ -x bin/valu_rates ]; then timeout -k 10 60 bin/valu_rates > "$O/valu_rates.log" 2>&1; fi
for b in $(ls ab); do
    export BCP_NATIVE_PATH=$PWD/ab/$b/$EXT
    timeout -k 10 200 python -u tools/eh_crosscheck.py --nonces 2 > "$O/x200_$b.log" 2>&1
    timeout -k 10 100 python -u tools/eh_crosscheck.py --n 96 --k 5 --nonces 16 > "$O/x96_$b.log" 2>&1
    timeout -k 10 100 python -u tools/eh_crosscheck.py --n 48 --k 5 --nonces 32 > "$O/x48_$b.log" 2>&1
    echo "$b $(grep -h -o '"missing": [0-9]*, "extra": [0-9]*'  "$O/x200_$b.log" "$O/x96_$b.log" "$O/x48_$b.log" | tr '\n' ' ')"
    timeout -k 10 100 python3 tools/eh_serial.py > "$O/ser_$b.log" 2>&1
    echo "$b serial $(tail -n 1 "$O/ser_$b.log")"
done
cd /tmp
for b in $(ls "$GRAFT_REPO_ROOT/ab"); do
    BCP_NATIVE_PATH=$GRAFT_REPO_ROOT/ab/$b/$EXT timeout -k 10 120 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/p_$b" \
        -o k -- python3 "$GRAFT_REPO_ROOT/tools/eh_serial.py" > "$GRAFT_REPO_ROOT/$O/prof_$b.log" 2>&1
done
cd "$GRAFT_REPO_ROOT"
unset BCP_NATIVE_PATH
timeout -k 10 500 python -u tools/ab_bench.py --reps ${REPS:-3} ab/*/$EXT > "$O/ab.log" 2>&1
tail -n 6 "$O/ab.log"
# PMC pass over the serial run of the first build (generation + rounds)
if [ -n "$PMC_BUILD" ]; then
    cd /tmp
    BCP_NATIVE_PATH=$GRAFT_REPO_ROOT/ab/$PMC_BUILD/$EXT timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv \
        -d "$GRAFT_REPO_ROOT/$O/pmc_a" -o a --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -- python3 "$GRAFT_REPO_ROOT/tools/eh_serial.py" --iters 2 \
        > "$GRAFT_REPO_ROOT/$O/pmc_a.log" 2>&1
    echo pmc_done
fi
# headline batch-size sweep of one build
if [ -n "$SWEEP_BUILD" ]; then
    cd "$GRAFT_REPO_ROOT"
    for B in 8 16 32 64; do
        BCP_NATIVE_PATH=$PWD/ab/$SWEEP_BUILD/$EXT timeout -k 10 120 python3 bench.py --batch $B > "$O/sweep_$B.log" 2>&1
        echo "batch $B $(tail -n 1 "$O/sweep_$B.log" | cut -c1-120)"
    done
fi
