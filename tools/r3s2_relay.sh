#!/bin/bash
# K7/K9 on one MI355X: GPU tests of the device sighash recipes, the fused sighash -> verify lane
# and the BIP152 short-id kernel; their micro-benches (CPU vs GPU); 8 MB connects with the FORKID
# digests on the CPU workers (-gpusighash=0) vs fused into the GPU batch (-gpusighash=2); a
# rocprofv3 kernel split of the fused 160k-sigop connect.
# Usage: gpurun --timeout 1100 -- 'bash tools/r3s2_relay.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-relay}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_sighash_recipes.py tests/test_shortid_gpu.py -m gpu -x -v \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -3 "$OUT/pytest.log"
timeout -k 10 120 ./bin/bench_bcp -filter='(CPU|GPU)_(ShortIds|Sighash).*' -time=2 > "$OUT/micro.log" 2>&1
cat "$OUT/micro.log"
for m in 0 2; do
    timeout -k 10 300 ./bin/bench_bcp -filter='ConnectBlock8MB(_160kSigops)?_GPU' -gpusighash=$m -time=3 \
        > "$OUT/connect_sh$m.log" 2> "$OUT/connect_sh$m.err"
    echo "== -gpusighash=$m"; cat "$OUT/connect_sh$m.log"; grep '^#' "$OUT/connect_sh$m.err" | tail -6
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o fused -- \
    "$GRAFT_REPO_ROOT/bin/bench_bcp" -filter='ConnectBlock8MB_160kSigops_GPU' -gpusighash=2 -time=2 \
    > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
find "$GRAFT_REPO_ROOT/$OUT/prof" -name '*kernel_stats.csv' -exec head -12 {} \;
echo DONE
