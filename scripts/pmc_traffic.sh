#!/bin/bash
# HBM traffic of the bench workload's kernels: one rocprofv3 pass per counter group
# (FETCH_SIZE and WRITE_SIZE cannot share a pass).  One bench run per line group, so that every
# kernel's dispatches belong to one line: c3 + rop + lu + rop161, then c4, c5, pfr and hcci alone;
# then the per-line summaries are merged with profiles/traffic.json (the file bench.py reads) into
# gpurun_out/traffic_merged.json, to be copied into profiles/ with the run's other results.
# Usage: pmc_traffic.sh TAG [GROUPS]   (GROUPS: comma list of c3,c4,c5,pfr,hcci,ropext; default all)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-dev}
GROUPS_=${2:-c3,c4,c5,pfr,hcci,ropext}
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
files=()
for g in ${GROUPS_//,/ }; do
  case $g in
    c3) run $TAG c3,rop,lu,rop161 "" "" || exit $?; files+=(gpurun_out/traffic_$TAG.json) ;;
    c4) run ${TAG}_c4 c4 "--line c4" "--reactors 64" || exit $?; files+=(gpurun_out/traffic_${TAG}_c4.json) ;;
    c5) run ${TAG}_c5 c5 "--line c5" "--reactors 64" || exit $?; files+=(gpurun_out/traffic_${TAG}_c5.json) ;;
    pfr) run ${TAG}_pfr pfr "--line pfr" "--reactors 64" || exit $?; files+=(gpurun_out/traffic_${TAG}_pfr.json) ;;
    hcci) run ${TAG}_hcci hcci "--line hcci" "--reactors 64" || exit $?; files+=(gpurun_out/traffic_${TAG}_hcci.json) ;;
    ropext) run ${TAG}_ropext ropext "--line ropext" "--reactors 64" || exit $?; files+=(gpurun_out/traffic_${TAG}_ropext.json) ;;
  esac
done
python3 - "${files[@]}" <<'PY'
import json, sys
try:
    t = json.load(open("profiles/traffic.json"))
except (OSError, ValueError):
    t = {}
for f in sys.argv[1:]:
    t.update(json.load(open(f)))
json.dump(t, open("gpurun_out/traffic_merged.json", "w"), indent=1)
print("merged", ", ".join(sys.argv[1:]), "-> gpurun_out/traffic_merged.json")
PY
