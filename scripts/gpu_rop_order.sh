#!/bin/bash
# ROP kernel: A/B of the specialised kernel's reaction order (default sort vs the narrow-window
# order, CKMI_JIT_ORDER=1) and the HBM traffic of the bench's ROP line under each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-roporder}
timeout -k 10 600 python3 scripts/ab_bench.py pychemkin_amd/_lib/libckmi.so@CKMI_JIT_ORDER=0 pychemkin_amd/_lib/libckmi.so@CKMI_JIT_ORDER=1 --rop --reps 3 > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -12 gpurun_out/ab_$TAG.log; [ $rc -eq 0 ] || exit $rc
for o in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    CKMI_JIT_ORDER=$o timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic_${TAG}_o$o/$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --lines rop > gpurun_out/traffic_${TAG}_o${o}_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/traffic_${TAG}_o${o}_$c.log; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/traffic_summary.py gpurun_out/traffic_${TAG}_o$o > gpurun_out/traffic_${TAG}_o$o.json && cat gpurun_out/traffic_${TAG}_o$o.json
done
