#!/bin/bash
# LDS / memory counters of the solver kernels over a serial run (one rocprofv3 pass per group),
# plus the per-phase cycle stamps. Usage (GPU box): bash tools/pmc_rounds.sh TAG
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/counters.txt 2>&1 || echo list_failed
S="python3 $GRAFT_REPO_ROOT/tools/eh_serial.py --iters 2"
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/l -o l --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -- $S > $O/l.log 2>&1 || echo pass_l_failed
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/m -o m --pmc SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAVES -- $S > $O/m.log 2>&1 || echo pass_m_failed
cd $GRAFT_REPO_ROOT
EH_PHASES=1 timeout -k 10 120 python -u tools/eh_diag.py > $O/phases.log 2>&1
tail -n 12 $O/phases.log
echo pmc_rounds_done
