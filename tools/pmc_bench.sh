#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc pass per counter group; gfx950 slot
# limits: 8 SQ, 4 TCC (FETCH_SIZE uses 3, WRITE_SIZE 2), 2 GRBM).  Summaries land in gpurun_out/
# (pmc_summary.txt, traffic.json); the databases are deleted (gpurun_out is capped at 64 MiB).
# Usage (GPU box): bash tools/pmc_bench.sh [bench args...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS=${@:-"--steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-latency"}
pass() {
  local k=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$k -o run -- python3 bench.py $ARGS > gpurun_out/pmc_$k.log 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
pass sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pass mfma SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 tools/pmc_summary.py gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 gpurun_out/pmc_mfma gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_summary.txt
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write ${PMC_KERNEL:-k_chain} > gpurun_out/traffic.json
rm -rf gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 gpurun_out/pmc_mfma gpurun_out/pmc_fetch gpurun_out/pmc_write
python3 tools/pmc_exec.py gpurun_out/pmc_summary.txt ${PMC_KERNEL:-k_chain} --units-per-dispatch ${PMC_UNITS:-15872} > gpurun_out/exec_k_chain.json
