#!/bin/bash
# Round-3: the plug-flow and HCCI bench lines alone (c3 headline reduced), to size them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py --steps 1 --warmup 0 --reactors 4096 --cpu-sample 0 --lines c3,pfr,hcci \
  > gpurun_out/bench_models_r03p.json 2> gpurun_out/bench_models_r03p.err
rc=$?; python3 -c "
import json; b=json.loads(open('gpurun_out/bench_models_r03p.json').readline())
for k in ('pfr','hcci'):
    v=b[k]; print(k, round(v['value']), v['unit'], 'failed', v['failed'], 'not_ign', v['not_ignited'], 's', round(v['seconds'],3), 'frac', round(v['roofline']['frac'],4), v['solver'])
"; tail -3 gpurun_out/bench_models_r03p.err; exit $rc
