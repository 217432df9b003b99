#!/bin/bash
# MFMA evidence for the batched LU (configs[4] component): kernel trace of scripts/lu_bench.py and
# one PMC pass with the FP64-MFMA counters this GPU exposes.  Usage: lu_pmc.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_avail_$TAG.txt 2>&1
rc=$?
if [ $rc -ne 0 ]; then echo "counter list status $rc: stop"; exit $rc; fi
want=""
for c in SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE; do
  if grep -q "\b$c\b" gpurun_out/counters_avail_$TAG.txt; then want="$want $c"; fi
done
echo "counters:$want"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lu_trace_$TAG -o run -- \
  python3 scripts/lu_bench.py > gpurun_out/lu_trace_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/lu_trace_$TAG.log
if [ $rc -ne 0 ]; then echo "trace status $rc: stop"; exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc $want --output-format csv -d gpurun_out/lu_pmc_$TAG -o run -- \
  python3 scripts/lu_bench.py > gpurun_out/lu_pmc_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/lu_pmc_$TAG.log
if [ $rc -ne 0 ]; then echo "pmc status $rc: stop"; exit $rc; fi
find gpurun_out/lu_trace_$TAG gpurun_out/lu_pmc_$TAG -name "*.csv"
