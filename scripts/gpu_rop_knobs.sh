#!/bin/bash
# Specialised ROP kernel knobs on the bench's ROP line (10M GRI-3.0 states): states/s (scripts/ab_bench.py)
# and HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE passes) per setting.
# Usage: gpu_rop_knobs.sh TAG "ENV1 ENV2 ..."   (each ENV e.g. CKMI_JIT_WAVES=1,CKMI_JIT_GROUP=16; "-" = defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ropk}
SETS=${2:--}
libs=()
for s in $SETS; do
  if [ "$s" = "-" ]; then libs+=(pychemkin_amd/_lib/libckmi.so); else libs+=("pychemkin_amd/_lib/libckmi.so@${s//,/@}"); fi
done
timeout -k 10 600 python3 scripts/ab_bench.py "${libs[@]}" --rop --reps 3 > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -30 gpurun_out/ab_$TAG.log; [ $rc -eq 0 ] || exit $rc
i=0
for s in $SETS; do
  i=$((i + 1))
  envs=()
  [ "$s" != "-" ] && envs=(${s//,/ })
  for c in FETCH_SIZE WRITE_SIZE; do
    env "${envs[@]}" timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic_${TAG}_$i/$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --lines rop > gpurun_out/traffic_${TAG}_${i}_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/traffic_${TAG}_${i}_$c.log; [ $rc -eq 0 ] || exit $rc
  done
  echo "== $s"
  python3 scripts/traffic_summary.py gpurun_out/traffic_${TAG}_$i > gpurun_out/traffic_${TAG}_$i.json && grep -A2 '"rop_jit"' gpurun_out/traffic_${TAG}_$i.json
done
