# GPU round check: full gpu test tier, ECDSA bench, rocprof kernel stats for ECDSA and Equihash bench.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_ecdsa gpurun_out/prof_eh
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
timeout -k 10 300 python tools/ecdsa_bench.py 65536 > gpurun_out/ecdsa_bench.log 2>&1 && cat gpurun_out/ecdsa_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ecdsa -o run -- python3 tools/ecdsa_bench.py 65536 > gpurun_out/prof_ecdsa.log 2>&1 && echo PROF_ECDSA_OK
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_eh -o run -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_eh.log 2>&1 && echo PROF_EH_OK
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && cat gpurun_out/bench.log
