#!/bin/bash
# Round-4 check: GPU tests, A/B of the reactor kernel variants against round 3, PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04b}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
L=pychemkin_amd/_lib
timeout -k 10 900 python3 scripts/ab_bench.py $L/libckmi_r03.so $L/libckmi_b128.so $L/libckmi.so $L/libckmi.so@CKMI_LANES=0 \
  $L/libckmi_gjb8.so --reps 3 > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -30 gpurun_out/ab_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_passes.sh $TAG
