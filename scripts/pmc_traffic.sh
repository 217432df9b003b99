#!/bin/bash
# HBM traffic of the bench workload's kernels: one rocprofv3 pass per counter group
# (FETCH_SIZE and WRITE_SIZE cannot share a pass).  Three bench runs, so that every kernel's
# dispatches belong to one line: c3 + rop + lu + rop161, then c4 alone, then c5 alone.
# Usage: pmc_traffic.sh TAG   -> gpurun_out/traffic_TAG{,_c4,_c5}.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-dev}
export TMPDIR=/tmp
run() {  # run NAME LINES SUMMARY-FLAGS BENCH-FLAGS
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic_$1/$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --lines $2 $4 > gpurun_out/traffic_$1_$c.log 2>&1
    rc=$?
    tail -1 gpurun_out/traffic_$1_$c.log
    if [ $rc -ne 0 ]; then echo "$1 $c pass status $rc: stop"; exit $rc; fi
  done
  python3 scripts/traffic_summary.py gpurun_out/traffic_$1 $3 > gpurun_out/traffic_$1.json && cat gpurun_out/traffic_$1.json
}
run $TAG c3,rop,lu,rop161 "" "" && run ${TAG}_c4 c4 --c4 "--reactors 64" && run ${TAG}_c5 c5 "" "--reactors 64"
