set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_ecdsa3
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_ecdsa_batch.py tests/test_node_regtest.py -q -m gpu -x > gpurun_out/pytest_gpu3.log 2>&1 && echo PYTEST_OK
tail -3 gpurun_out/pytest_gpu3.log
timeout -k 10 300 python tools/ecdsa_bench.py 65536 > gpurun_out/ecdsa_bench3.log 2>&1 && cat gpurun_out/ecdsa_bench3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ecdsa3 -o run -- python3 tools/ecdsa_bench.py 65536 > gpurun_out/prof_ecdsa3.log 2>&1 && echo PROF_OK
