#!/bin/bash
# Quick GPU iteration: parity tests, phase profile, short bench.  Usage: gpu_quick.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-dev}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
timeout -k 10 120 python3 scripts/phase_profile.py 4096 > gpurun_out/phase_$TAG.json 2>&1
rc=$?; cat gpurun_out/phase_$TAG.json
if [ $rc -ne 0 ]; then echo "phase profile status $rc: stop"; exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
exit $rc
