#!/bin/bash
# ECDSA batch-verify check on one GPU: VALU rates, CPU/GPU crossover, 262k throughput, rocprof kernel stats.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ec1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ecdsa_batch.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log; export TMPDIR=/tmp
timeout -k 10 60 bin/valu_rates > $O/valu_rates.log 2>&1
timeout -k 10 200 python -u tools/ecdsa_crossover.py 16 > $O/cross.log 2>&1
tail -n 2 $O/cross.log | cut -c1-300
timeout -k 10 200 python -u tools/ecdsa_bench.py 262144 > $O/bench.log 2>&1
tail -n 3 $O/bench.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o ec -- python3 $GRAFT_REPO_ROOT/tools/ecdsa_bench.py 262144 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo done
