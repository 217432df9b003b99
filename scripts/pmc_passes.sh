#!/bin/bash
# rocprofv3 PMC passes over scripts/pmc_run.py (one pass per process; each under its own limit).
# Usage: pmc_passes.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc_${TAG}/p$i -o run -- \
    python3 scripts/pmc_run.py > gpurun_out/pmc_${TAG}_p$i.log 2>&1
  rc=$?
  tail -2 gpurun_out/pmc_${TAG}_p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i ($counters) status $rc: stop"; exit $rc; fi
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU
SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES
LIST
find gpurun_out/pmc_${TAG} -name "*counter_collection*"
