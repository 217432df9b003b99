#!/bin/bash
# Round-3 check: viscosity, KIN, extended specialised-ROP parity; A/B of the LDS-broadcast Newton solve.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_transport.py tests/test_gpu_kin.py tests/test_gpu_rop_jit.py \
  tests/test_cheb_lt.py tests/test_ford.py tests/test_wide_reactions.py tests/test_plog.py -m gpu -x -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r03e.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_r03e.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
timeout -k 10 400 python3 scripts/ab_bench.py pychemkin_amd/_lib/libckmi.so pychemkin_amd/_lib/libckmi_solvelds.so \
  --reps 3 --n 16384 > gpurun_out/ab_solvelds_r03e.log 2>&1
rc2=$?; tail -12 gpurun_out/ab_solvelds_r03e.log
exit $(( rc != 0 ? rc : rc2 ))
