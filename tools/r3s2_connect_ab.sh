#!/bin/bash
# A/B of the 8 MB GPU connects: the pre-K7 bench_bcp (ab/bench_bcp_pre_k7) vs the current one
# (-gpusighash=0, the default), interleaved 3 times. Usage: gpurun -- 'bash tools/r3s2_connect_ab.sh TAG'
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-connab}
mkdir -p "$OUT"
for rep in 1 2 3; do
    for b in ab/bench_bcp_pre_k7 bin/bench_bcp; do
        timeout -k 10 200 ./$b -filter='ConnectBlock8MB(_160kSigops|_Multisig)?_GPU' -time=2 > "$OUT/$rep_$(basename $b).log" 2>/dev/null
        echo "== rep $rep $b"; grep ConnectBlock "$OUT/$rep_$(basename $b).log"
    done
done
echo DONE
