#!/bin/bash
# HBM traffic and achieved bandwidth per solver kernel: one plain kernel-trace pass for
# durations, then one counter pass each for FETCH_SIZE and WRITE_SIZE (TCC counters: 3 + 2 of
# the 4 per pass, so they cannot share a pass). Serial solver (tools/eh_serial.py), so kernel
# durations are not shared with a second solver.
# Usage (GPU box): bash tools/pmc_bw.sh TAG   then here: python3 tools/pmc_bw.py gpurun_out/TAG
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
S="$GRAFT_REPO_ROOT/tools/eh_serial.py --iters 3"
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/t -o t -- python3 $S > $O/t.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/f -o f --pmc FETCH_SIZE -- python3 $S > $O/f.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/w -o w --pmc WRITE_SIZE -- python3 $S > $O/w.log 2>&1
echo pmc_bw_done
