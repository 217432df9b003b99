#!/bin/bash
# Round-3: plug-flow reactors on the GPU, the whole GPU suite, and a c3-only bench (regression check).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu_r03g.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_r03g.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --lines c3 > gpurun_out/bench_c3_r03g.json \
  2> gpurun_out/bench_c3_r03g.err
rc2=$?; head -c 700 gpurun_out/bench_c3_r03g.json; echo; tail -3 gpurun_out/bench_c3_r03g.err
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 200 python3 scripts/c3_stats.py > gpurun_out/c3_stats_r03g.log 2>&1
rc3=$?; tail -2 gpurun_out/c3_stats_r03g.log
exit $(( rc != 0 ? rc : rc3 ))
