#!/bin/bash
# Round-3: engine cylinders (problem 4) on the wave kernel -- engine, plug-flow and reactor GPU tests,
# then an A/B of the configs[2] kernel against the previous library (RunCtx / launch-split changes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_pfr.py tests/test_gpu_reactor.py tests/test_gpu_kin.py tests/test_gpu_transport.py -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r03n.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu_r03n.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 scripts/ab_bench.py --n 65536 --reps 3 \
  pychemkin_amd/_lib/libA_r03k.so pychemkin_amd/_lib/libB_engine.so > gpurun_out/ab_engine_r03n.log 2>&1
rc2=$?; tail -12 gpurun_out/ab_engine_r03n.log
exit $(( rc > rc2 ? rc : rc2 ))
