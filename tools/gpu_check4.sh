set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu4.log 2>&1 && echo PYTEST_OK
tail -3 gpurun_out/pytest_gpu4.log
timeout -k 10 300 python bench.py > gpurun_out/bench4.log 2>&1 && cat gpurun_out/bench4.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke4.log 2>&1 && tail -2 gpurun_out/smoke4.log
