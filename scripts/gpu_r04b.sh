#!/bin/bash
# Round-4 check: GPU tests on the lane-assigned image, A/B of the reactor kernel against round 3, PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04b}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
timeout -k 10 600 python3 scripts/ab_bench.py pychemkin_amd/_lib/libckmi_r03.so pychemkin_amd/_lib/libckmi.so \
  pychemkin_amd/_lib/libckmi.so@CKMI_LANES=0 --reps 3 > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -25 gpurun_out/ab_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_passes.sh $TAG
