#!/bin/bash
# PMC passes over tools/configs_bench.py for one BASELINE config (2, 4 or 5); same counter groups
# and gfx950 slot limits as tools/pmc_bench.sh.  Summaries land in gpurun_out/pmc_cfg<C>_*.txt.
# Usage (GPU box): bash tools/pmc_configs.sh <config> [kernel-substring-for-traffic]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C=$1
K=${2:-}
mkdir -p gpurun_out
pass() {
  local k=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/pmcc${C}_$k -o run -- python3 tools/configs_bench.py --configs $C --reps 1 > gpurun_out/pmcc${C}_$k.log 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
pass sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pass mfma SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 tools/pmc_summary.py gpurun_out/pmcc${C}_sq1 gpurun_out/pmcc${C}_sq2 gpurun_out/pmcc${C}_mfma gpurun_out/pmcc${C}_fetch gpurun_out/pmcc${C}_write > gpurun_out/pmc_cfg${C}_summary.txt
if [ -n "$K" ]; then
  python3 tools/pmc_traffic.py gpurun_out/pmcc${C}_fetch gpurun_out/pmcc${C}_write $K > gpurun_out/pmc_cfg${C}_traffic.json
fi
rm -rf gpurun_out/pmcc${C}_sq1 gpurun_out/pmcc${C}_sq2 gpurun_out/pmcc${C}_mfma gpurun_out/pmcc${C}_fetch gpurun_out/pmcc${C}_write
