#!/bin/bash
# ECDSA kernel A/B: GPU numerics tests on the in-tree build, then per-build kernel times
# (rocprofv3 --kernel-trace of tools/ecdsa_bench.py) for every build under ab/.
# Usage (gpurun): bash tools/ec_ab.sh TAG [N]
set -e
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/$1
N=${2:-262144}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ecdsa_batch.py tests/test_gpu_verify_service.py -x -q -m gpu --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -n 30 "$O/pytest.log"; exit 1; }
tail -n 1 "$O/pytest.log"
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  (cd /tmp && BCP_NATIVE_PATH=$GRAFT_REPO_ROOT/ab/$b/$EXT timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/$b" -o k -- python3 "$GRAFT_REPO_ROOT/tools/ecdsa_bench.py" "$N" > "$O/$b.log" 2>&1)
  echo "$b $(grep '^{' "$O/$b.log" | tail -n 1)"
done
