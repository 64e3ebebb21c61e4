#!/bin/bash
# PMC counters of the Equihash solver kernels over a serial run (tools/eh_serial.py: one solver,
# no overlap, so every dispatch's counters are its own). One rocprofv3 pass per counter group,
# each within the per-block limits (8 SQ, 4 TCC, 2 GRBM) and under its own kill timeout.
# Usage (GPU box, repo root): bash tools/pmc_eh.sh TAG [NATIVE_SO]
# Table: python3 tools/pmc_table.py gpurun_out/TAG
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc}
mkdir -p "$O"
[ -n "$2" ] && export BCP_NATIVE_PATH=$(readlink -f "$2")
cd /tmp && export TMPDIR=/tmp
[ -f "$O/counters.txt" ] || timeout -s KILL 60 rocprofv3 --list-avail > "$O/counters.txt" 2>&1 || true
S="python3 $GRAFT_REPO_ROOT/tools/eh_serial.py --iters 2"
pass() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$O/$n" -o "$n" --pmc "$@" -- $S > "$O/$n.log" 2>&1; }
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM
pass c FETCH_SIZE GRBM_GUI_ACTIVE
pass d WRITE_SIZE TCC_HIT_sum
echo pmc_done
