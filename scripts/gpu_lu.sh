#!/bin/bash
# GPU session: GPU tests (unless NOTEST=1), then the LU phase split and an A/B of standalone LU builds.
# Usage: scripts/gpu_lu.sh TAG phase_lib.so lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; PH=$2; shift 2
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -8 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
fi
timeout -k 10 300 python3 scripts/lu_phase.py "$PH" > gpurun_out/lu_phase_$TAG.log 2>&1 || exit $?
cat gpurun_out/lu_phase_$TAG.log
timeout -k 10 300 python3 scripts/lu_ab.py "$@" > gpurun_out/lu_ab_$TAG.log 2>&1; rc=$?
cat gpurun_out/lu_ab_$TAG.log; exit $rc
