#!/bin/bash
# 8 MB connect benches on one MI355X plus a kernel-time profile of the 160k-sigop GPU connect,
# and the hashing/merkle micro-benches (CPU SHA-NI vs GPU).
# Usage: gpurun --timeout 900 -- 'bash tools/r3_connect_prof.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-connprof}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify_service.py tests/test_ops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -2 "$OUT/pytest.log"
timeout -k 10 300 ./bin/bench_bcp -filter='ConnectBlock8MB_(160kSigops_)?GPU|ConnectBlock8MB_Multisig_GPU' -time=3 > "$OUT/connect.log" 2> "$OUT/connect.err"
cat "$OUT/connect.log"; grep '^#' "$OUT/connect.err"
timeout -k 10 300 ./bin/bench_bcp -filter='.*MerkleRoot.*|.*SHA256d64.*' -time=1 > "$OUT/hash.log" 2>&1
cat "$OUT/hash.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- "$GRAFT_REPO_ROOT/bin/bench_bcp" -filter='ConnectBlock8MB_160kSigops_GPU' -time=2 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
echo DONE
