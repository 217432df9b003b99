#!/bin/bash
# GPU session: GPU tests (unless NOTEST=1), then an A/B of reactor-kernel library variants.
# Usage: scripts/gpu_ab.sh TAG lib1.so[@ENV=V] lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -6 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
fi
timeout -k 10 900 python3 scripts/ab_bench.py "$@" --reps ${REPS:-3} > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -28 gpurun_out/ab_$TAG.log; exit $rc
