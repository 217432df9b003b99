#!/bin/bash
# Round-3: configs[2] A/B of the engine-capable library against the previous one, and the invalid-problem test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 scripts/ab_bench.py --n 65536 --reps 3 \
  pychemkin_amd/_lib/libA_r03k.so pychemkin_amd/_lib/libB_engine.so > gpurun_out/ab_engine_r03m.log 2>&1
rc=$?; tail -12 gpurun_out/ab_engine_r03m.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_reactor.py -q -k invalid --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu_r03m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r03m.log; exit $rc
