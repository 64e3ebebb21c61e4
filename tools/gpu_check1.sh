set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ecdsa_batch.py tests/test_equihash.py tests/test_sha256_gpu.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
timeout -k 10 300 python tools/ecdsa_bench.py 50000 > gpurun_out/ecdsa_bench.log 2>&1 && cat gpurun_out/ecdsa_bench.log
