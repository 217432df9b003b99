#!/bin/bash
# Round-3: engine cylinders through the KIN ABI and the drop-in; engine / KIN / transport GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_kin.py tests/test_gpu_transport.py -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r03o.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu_r03o.log; exit $rc
