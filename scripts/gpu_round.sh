#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit.  An ordinary test failure (pytest exit 1) lets the
# session go on to the bench; a crash, abort, fault or time-out (any other non-zero status)
# ends it there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
STEPS=${2:-all}
mkdir -p gpurun_out
export TMPDIR=/tmp

stop_unless_ok() {  # $1 = status, $2 = step name, $3 = allowed non-fatal status
  if [ "$1" -ne 0 ] && [ "$1" -ne "${3:-0}" ]; then
    echo "!! $2 ended with status $1: stopping"
    exit "$1"
  fi
}

if [[ $STEPS == all || $STEPS == *test* ]]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -25 gpurun_out/pytest_gpu_$TAG.log; stop_unless_ok $rc pytest 1
  echo "== smoke"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/smoke_$TAG.log; stop_unless_ok $rc smoke 1
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  echo "== bench"
  timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err; stop_unless_ok $rc bench
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
  rc=$?; cat gpurun_out/bench_prof_$TAG.json; tail -5 gpurun_out/bench_prof_$TAG.err; stop_unless_ok $rc rocprofv3
  find gpurun_out/prof_$TAG -name "*stats*"
fi
if [[ $STEPS == all || $STEPS == *traffic* ]]; then
  echo "== PMC traffic"
  bash scripts/pmc_traffic.sh $TAG; stop_unless_ok $? traffic
fi
echo "== done"
