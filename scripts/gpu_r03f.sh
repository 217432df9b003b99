#!/bin/bash
# Round-3: narrow-window reaction order of the specialised ROP kernel, A/B on configs[1] (10M GRI states),
# then its parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=pychemkin_amd/_lib/libckmi.so
timeout -k 10 500 python3 scripts/ab_bench.py --rop --n 10000000 --reps 3 \
  "$L@CKMI_JIT_ORDER=0" "$L@CKMI_JIT_ORDER=1" "$L@CKMI_JIT_ORDER=1@CKMI_JIT_WAVES=3" "$L@CKMI_JIT_ORDER=1@CKMI_JIT_WAVES=4" \
  > gpurun_out/ab_jit_order_r03f.log 2>&1
rc=$?; tail -22 gpurun_out/ab_jit_order_r03f.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rop_jit.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_jit_r03f.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_jit_r03f.log; exit $rc
