#!/bin/bash
# Every one-GPU measurement of this repo behind one entry point (run on the GPU box):
#   gpurun --timeout 1100 -- 'bash tools/gpu_check.sh MODE TAG [ARGS]'
# Output lands in gpurun_out/TAG/. Each GPU step has its own time limit and the steps are
# chained by `set -e`, so the first failure (test, fault, timeout) ends the run.
#
# Modes
#   check TAG [prof]     GPU test tier, smoke(), bench.py (20 steps), solver recall vs the CPU
#                        solver; with "prof" also a rocprofv3 --kernel-trace --stats of the bench
#   bench TAG [RUNS]     RUNS (default 5) separate bench.py processes of 20 steps: median, min, max
#   eh-ab TAG [REPS]     solver builds under ab/*/: GPU equihash tests + (200,9)/(96,5) CPU
#                        cross-checks of the in-tree build, serial batch timing per build,
#                        interleaved headline A/B (tools/ab_bench.py, REPS >= 20 recommended)
#   eh-trace TAG         per-kernel durations of each ab/ build (serial solver) and the
#                        two-solver timeline of the bench (tools/eh_timeline.py)
#   eh-phases TAG        per-phase cycle stamps of the round kernels for each ab/ build
#   eh-sweep TAG "B:S.." headline over (nonce batch, solvers in flight)
#   pmc-eh TAG [SO]      PMC passes over the serial solver -> python3 tools/pmc_report.py gpurun_out/TAG
#   pmc-ec TAG [N]       PMC passes over the ECDSA batch kernels (tools/ecdsa_bench.py N)
#   ecdsa TAG [N]        ECDSA GPU tests, per-build kernel times of ab/*/ at N signatures,
#                        the CPU-pool vs GPU crossover sweep
#   ecdsa-cpu TAG        CPU ECDSA / ecmult micro-benches and the CPU 8 MB connect
#   connect TAG [BLOCKS] 8 MB block connects on the GPU path, parallel vs serial UTXO pass, the IBD pipeline, a kernel profile
#                        of the 160k-sigop GPU connect
#   ibd TAG [BLOCKS] [SECS]  IBD runs, plus interleaved A/Bs of -connectlookahead and -connectinplace:
#                            per-run ms/block, median/min/max per configuration, phase split
#   relay TAG            BIP152 short-id kernel: GPU tests and the CPU vs GPU micro-bench
#   lanes TAG            verify-service tests, then a 199k-signature and a 2000-header batch over
#                        lanes [0], [0,0], [0,0,0,0] (sharding overhead) and the host-built-state
#                        header path, with a kernel trace of the 2000-header runs
#   hash TAG             SHA256d64 / merkle micro-benches (CPU SHA-NI vs GPU)
#   baseline TAG         BASELINE.md secondary metrics (tools/baseline_metrics.py + bench_bcp)
#   multirank TAG        bench.py as 2 ranks on one GPU over gloo (the multi-rank launcher path)
#
# Older profiles name the per-session scripts these modes replace: r3_check.sh -> check;
# r3_eh_ab.sh, eh_ab_check.sh, eh_validate.sh, eh_variants.sh -> eh-ab; r3_eh_trace.sh,
# eh_ktrace.sh, eh_prof_builds.sh -> eh-trace; pmc_eh.sh, pmc_bw.sh, pmc_rounds.sh -> pmc-eh;
# ecdsa_check.sh, ec_ab.sh -> ecdsa; r3_ecdsa_cpu.sh -> ecdsa-cpu; r3_connect*.sh -> connect;
# r3s2_relay.sh -> relay (short ids; the device sighash path was removed in round 4); r3_gpu_check.sh -> check + hash; baseline_check.sh -> baseline;
# r3_ab_batch.sh, eh_sweep.sh -> eh-sweep; multirank_rehearsal.sh -> multirank.
set -e
cd "$GRAFT_REPO_ROOT"
MODE=${1:?mode}
TAG=${2:-$MODE}
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
R=$GRAFT_REPO_ROOT
builds() { ls ab 2>/dev/null; }

eh_tests() {
  timeout -k 10 300 python -u -m pytest tests/test_equihash.py -x -q -m gpu --timeout 200 --timeout-method thread \
    > "$O/t.log" 2>&1 || { tail -n 30 "$O/t.log"; exit 1; }
  tail -n 1 "$O/t.log"
  timeout -k 10 240 python -u tools/eh_crosscheck.py --nonces 8 > "$O/x200.log" 2>&1
  timeout -k 10 120 python -u tools/eh_crosscheck.py --n 96 --k 5 --nonces 16 > "$O/x96.log" 2>&1
  grep -h -o '"cpu_total": [0-9]*, "gpu_total": [0-9]*, "missing": [0-9]*, "extra": [0-9]*' "$O"/x*.log
}

case "$MODE" in
check)
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
    || { tail -n 40 "$O/pytest_gpu.log"; exit 1; }
  tail -n 3 "$O/pytest_gpu.log"
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -n 2 "$O/smoke.log"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$O/bench.log" 2>&1
  tail -n 1 "$O/bench.log"
  timeout -k 10 300 python -u tools/eh_recall.py --nonces 32 --threads 16 --json "$O/recall.json" > "$O/recall.log" 2>&1
  tail -n 4 "$O/recall.log"
  if [ "${3:-}" = prof ]; then
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 \
      > "$O/prof.log" 2>&1)
    tail -n 1 "$O/prof.log"
  fi ;;
bench)
  for i in $(seq 1 "${3:-5}"); do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$O/bench_$i.log" 2>&1
  done
  python3 - "$O" <<'EOF'
import glob, json, statistics, sys
v = [json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sorted(glob.glob(sys.argv[1] + "/bench_*.log"))]
print(json.dumps({"runs": len(v), "median": statistics.median(v), "min": min(v), "max": max(v), "values": v}))
EOF
  ;;
eh-ab)
  eh_tests
  for b in $(builds); do
    BCP_NATIVE_PATH=$PWD/ab/$b/$EXT timeout -k 10 100 python3 tools/eh_serial.py > "$O/ser_$b.log" 2>&1
    echo "$b $(tail -n 1 "$O/ser_$b.log")"
  done
  timeout -k 10 900 python -u tools/ab_bench.py --reps "${3:-20}" ab/*/$EXT > "$O/ab.log" 2>&1
  tail -n 3 "$O/ab.log" ;;
eh-trace)
  for b in $(builds); do
    (cd /tmp && BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/$b" -o k -- \
      python3 "$R/tools/eh_serial.py" --iters 5 > "$O/$b.log" 2>&1)
    echo "$b $(tail -n 1 "$O/$b.log")"
  done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/timeline" -o run -- \
    python3 "$R/bench.py" --steps 4 --warmup 2 > "$O/timeline.log" 2>&1)
  python3 tools/eh_timeline.py "$O/timeline" > "$O/timeline.txt" && tail -n 20 "$O/timeline.txt" ;;
eh-phases)
  for b in $(builds); do
    BCP_NATIVE_PATH=$PWD/ab/$b/$EXT EH_PHASES=1 timeout -k 10 120 python -u tools/eh_diag.py > "$O/ph_$b.log" 2>&1
    echo "== $b"; grep '"round"' "$O/ph_$b.log"
  done ;;
eh-sweep)
  for p in ${3:?"B:S list"}; do
    B=${p%:*}; S=${p#*:}
    timeout -k 10 150 python3 bench.py --batch "$B" --solvers "$S" --steps $((640 / B)) --warmup $((S + 1)) > "$O/b${B}_s${S}.log" 2>&1
    echo "batch $B solvers $S $(tail -n 1 "$O/b${B}_s${S}.log" | grep -o '"value": [0-9.]*')"
  done ;;
pmc-eh|pmc-ec)
  if [ "$MODE" = pmc-eh ]; then
    [ -n "${3:-}" ] && export BCP_NATIVE_PATH=$(readlink -f "$3")
    S="python3 $R/tools/eh_serial.py --iters 2"
  else
    S="python3 $R/tools/ecdsa_bench.py ${3:-262144}"
  fi
  cd /tmp
  pass() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$O/$n" -o "$n" --pmc "$@" -- $S > "$O/$n.log" 2>&1; }
  pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
  pass b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM
  pass c FETCH_SIZE GRBM_GUI_ACTIVE
  pass d WRITE_SIZE TCC_HIT_sum
  cd "$R" && python3 tools/pmc_report.py "$O" | tee "$O/report.md" ;;
ecdsa)
  N=${3:-262144}
  timeout -k 10 300 python -u -m pytest tests/test_ecdsa_batch.py tests/test_gpu_verify_service.py -x -q -m gpu --timeout 200 \
    --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -n 30 "$O/pytest.log"; exit 1; }
  tail -n 1 "$O/pytest.log"
  for b in $(builds); do
    (cd /tmp && BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/$b" -o k -- \
      python3 "$R/tools/ecdsa_bench.py" "$N" > "$O/$b.log" 2>&1)
    echo "$b $(grep '^{' "$O/$b.log" | tail -n 1)"
  done
  timeout -k 10 300 python -u tools/ecdsa_crossover.py 16 > "$O/crossover.log" 2>&1
  tail -n 3 "$O/crossover.log" | cut -c1-400 ;;
ecdsa-cpu)
  timeout -k 10 120 ./bin/bench_bcp -filter='ECDSAVerify_CPU|Ecmult_CPU.*' -time=3 > "$O/cpu.log" 2>&1
  cat "$O/cpu.log"
  timeout -k 10 300 ./bin/bench_bcp -filter='ConnectBlock8MB_CPU' -time=3 > "$O/connect_cpu.log" 2> "$O/connect_cpu.err"
  cat "$O/connect_cpu.log" ;;
connect)
  # GPU path, parallel UTXO pass (default) then the serial pass (-parallelutxo=0), >= 20 iterations each
  timeout -k 10 300 ./bin/bench_bcp -filter='ConnectBlock8MB.*_GPU' -time=4 > "$O/connect.log" 2> "$O/connect.err"
  cat "$O/connect.log"; grep '^#' "$O/connect.err" | tail -n 12
  timeout -k 10 300 ./bin/bench_bcp -filter='ConnectBlock8MB.*_GPU' -time=4 -parallelutxo=0 > "$O/connect_serial.log" \
    2> "$O/connect_serial.err"
  cat "$O/connect_serial.log"; grep '^#' "$O/connect_serial.err" | tail -n 12
  timeout -k 10 600 ./bin/bench_bcp -filter='IbdPipeline_Seq_GPU' -ibdblocks="${3:-50}" -time=0 > "$O/ibd.log" 2> "$O/ibd.err"
  cat "$O/ibd.log"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- "$R/bin/bench_bcp" \
    -filter='ConnectBlock8MB_160kSigops_GPU' -time=2 > "$O/prof.log" 2>&1) ;;
ibd)
  # IBD of -ibdblocks big blocks on the GPU path: one fixture, then as many whole runs as fit in
  # -time seconds (default config), then the same with each of the two overlap options alternated
  # on/off run by run; per-run ms/block and the phase split around ConnectTip (stderr '# ibd'
  # lines), summarised as median / min / max per configuration
  timeout -k 10 900 ./bin/bench_bcp -filter="IbdPipeline_Seq_GPU" -ibdblocks="${3:-50}" -time="${4:-12}" \
    > "$O/ibd_default.log" 2> "$O/ibd_default.err"
  for ab in lookahead inplace; do
    timeout -k 10 900 ./bin/bench_bcp -filter="IbdPipeline_Seq_GPU" -ibdblocks="${3:-50}" -time="${4:-12}" -ibdab=$ab \
      > "$O/ibd_ab_$ab.log" 2> "$O/ibd_ab_$ab.err"
  done
  python3 tools/ibd_summary.py "$O"
  grep -h '^# ibd' "$O"/ibd_default.err | tail -n 2 ;;
relay)
  timeout -k 10 300 python -u -m pytest tests/test_shortid_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/pytest.log" 2>&1
  tail -n 3 "$O/pytest.log"
  timeout -k 10 120 ./bin/bench_bcp -filter='(CPU|GPU)_ShortIds.*' -time=2 > "$O/micro.log" 2>&1
  cat "$O/micro.log" ;;
lanes)
  timeout -k 10 400 python -u -m pytest tests/test_gpu_verify_service.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$O/pytest.log" 2>&1 || { tail -n 30 "$O/pytest.log"; exit 1; }
  tail -n 2 "$O/pytest.log"
  timeout -k 10 300 ./bin/bench_bcp -filter='Lanes.*|HeadersHostStates' -time=3 > "$O/lanes.log" 2>&1
  cat "$O/lanes.log"
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof" -o hdr -- "$R/bin/bench_bcp" \
    -filter='Lanes1_Headers2000_GPU|Lanes1_Ecdsa199k_GPU' -time=2 > "$O/prof.log" 2>&1) ;;
hash)
  timeout -k 10 300 ./bin/bench_bcp -filter='MerkleRoot|SHA256d64|^SHA256$' -time=1 > "$O/hash.log" 2>&1
  cat "$O/hash.log" ;;
baseline)
  timeout -k 10 300 python -u tools/baseline_metrics.py > "$O/metrics.log" 2>&1
  grep '^{' "$O/metrics.log" | cut -c1-220
  timeout -k 10 300 bin/bench_bcp -filter="ConnectBlock8MB.*|GPU_.*|CPU_MerkleRoot.*|CPU_SHA256d64.*" -time=3 > "$O/bench_bcp.log" 2>&1
  tail -n 20 "$O/bench_bcp.log" ;;
multirank)
  BCP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --batch 48 > "$O/bench2.log" 2>&1  # two ranks share one GPU: half the default batch each
  tail -n 1 "$O/bench2.log" ;;
*)
  echo "unknown mode $MODE"; exit 2 ;;
esac
echo DONE
