#!/bin/bash
# ROP kernel check: GPU ROP tests, A/B of the specialised kernel's wdot accumulators (registers vs
# LDS), HBM traffic of the bench's ROP line in both forms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-rop}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rop_jit.py tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stop"; exit $rc; fi
timeout -k 10 600 python3 scripts/ab_bench.py pychemkin_amd/_lib/libckmi.so@CKMI_JIT_WLDS=0 pychemkin_amd/_lib/libckmi.so@CKMI_JIT_WLDS=1 --rop --reps 3 > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -12 gpurun_out/ab_$TAG.log; [ $rc -eq 0 ] || exit $rc
for w in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    CKMI_JIT_WLDS=$w timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic_${TAG}_w$w/$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --lines rop > gpurun_out/traffic_${TAG}_w${w}_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/traffic_${TAG}_w${w}_$c.log; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/traffic_summary.py gpurun_out/traffic_${TAG}_w$w > gpurun_out/traffic_${TAG}_w$w.json && cat gpurun_out/traffic_${TAG}_w$w.json
done
