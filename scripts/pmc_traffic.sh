#!/bin/bash
# HBM traffic of the bench workload's kernels: one rocprofv3 pass per counter group
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), one reactor launch + one ROP launch.
# Usage: pmc_traffic.sh TAG   -> gpurun_out/traffic_TAG/{fetch,write}
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-dev}
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic_$TAG/$c -o run -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/traffic_${TAG}_$c.log 2>&1
  rc=$?
  tail -1 gpurun_out/traffic_${TAG}_$c.log
  if [ $rc -ne 0 ]; then echo "$c pass status $rc: stop"; exit $rc; fi
done
python3 scripts/traffic_summary.py gpurun_out/traffic_$TAG > gpurun_out/traffic_$TAG.json && cat gpurun_out/traffic_$TAG.json
