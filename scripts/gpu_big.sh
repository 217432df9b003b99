#!/bin/bash
# Workgroup-kernel (configs[4]) iteration on one GPU: the big-kernel GPU tests on the default library,
# an A/B of library variants on the c5 sample, then per variant one LDS pass and the two HBM-traffic
# passes (FETCH_SIZE, WRITE_SIZE) over 512 configs[4] reactors (scripts/c5_once.py).
# Usage: scripts/gpu_big.sh TAG lib1.so lib2.so ...   (NOTEST=1 skips the tests, NOPMC=1 the passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bigreactor.py tests/test_gpu_configs.py tests/test_gpu_bigmech_ext.py \
    -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_big_$TAG.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_big_$TAG.log
  if [ $rc -ne 0 ]; then echo "pytest status $rc: stop"; exit $rc; fi
fi
NOTEST=1 REPS=${REPS:-2} bash scripts/gpu_ab.sh ${TAG}_c5 "$@" --c5 || exit $?
[ "${NOPMC:-0}" = 1 ] && exit 0
for lib in "$@"; do
  name=$(basename "$lib" .so)
  i=0
  for counters in "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" FETCH_SIZE WRITE_SIZE; do
    i=$((i + 1))
    CKMI_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc_${TAG}_$name/p$i -o run -- \
      python3 scripts/c5_once.py 512 > gpurun_out/pmc_${TAG}_${name}_p$i.log 2>&1
    rc=$?
    tail -1 gpurun_out/pmc_${TAG}_${name}_p$i.log
    if [ $rc -ne 0 ]; then echo "$name pass $i status $rc: stop"; exit $rc; fi
  done
  echo "== $name"
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_$name | tee gpurun_out/pmc_${TAG}_${name}_summary.txt
done
