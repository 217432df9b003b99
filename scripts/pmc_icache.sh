#!/bin/bash
# Instruction-fetch counters of the reactor kernel (one rocprofv3 pass per counter group).
# Usage: pmc_icache.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-ic}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc_${TAG}/p$i -o run -- \
    python3 scripts/reactor_once.py 8192 > gpurun_out/pmc_${TAG}_p$i.log 2>&1
  rc=$?
  tail -2 gpurun_out/pmc_${TAG}_p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i ($counters) status $rc: stop"; exit $rc; fi
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH
SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU
LIST
find gpurun_out/pmc_${TAG} -name "*counter_collection*"
