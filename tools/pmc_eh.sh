#!/bin/bash
# Collect PMC counters for the Equihash solver kernels (run on the GPU box from the repo root).
# Usage: bash tools/pmc_eh.sh [OUTDIR]   (one rocprofv3 pass per counter group, each under its own timeout)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --verify 0"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/a -o a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- $B > $OUT/a.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/b -o b --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH -- $B > $OUT/b.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/c -o c --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -- $B > $OUT/c.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/e -o e --pmc FETCH_SIZE -- $B > $OUT/e.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/f -o f --pmc WRITE_SIZE TA_BUSY_avr TA_TA_BUSY_sum -- $B > $OUT/f.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/g -o g --pmc SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY -- $B > $OUT/g.log 2>&1
echo pmc_done
