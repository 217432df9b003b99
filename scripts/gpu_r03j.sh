#!/bin/bash
# Round-3: plug flow compiled into the FP64-inverse reactor variants only (FP32 launch skips problem 3,
# a paired FP64 launch runs it): A/B on configs[2] against the previous library, then the reactor tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 scripts/ab_bench.py --n 65536 --reps 3 \
  pychemkin_amd/_lib/libA_head.so pychemkin_amd/_lib/libB_pfsel.so > gpurun_out/ab_pfsel_r03j.log 2>&1
rc=$?; tail -12 gpurun_out/ab_pfsel_r03j.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pfr.py tests/test_gpu_reactor.py tests/test_gpu_kin.py -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r03j.log 2>&1
rc=$?; tail -6 gpurun_out/pytest_gpu_r03j.log; exit $rc
