#!/bin/bash
# Round-3: the HCCI sweep with NNEG (no stalled cylinder expected), then the pfr / hcci bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_engine_r03q.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_engine_r03q.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 scripts/hcci_diag.py --nneg > gpurun_out/hcci_diag_c.json 2> gpurun_out/hcci_diag_c.err
rc=$?; cut -c1-300 gpurun_out/hcci_diag_c.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 1 --warmup 0 --reactors 4096 --cpu-sample 0 --lines c3,pfr,hcci \
  > gpurun_out/bench_models_r03q.json 2> gpurun_out/bench_models_r03q.err
rc=$?
python3 - <<'PY'
import json
b = json.loads(open("gpurun_out/bench_models_r03q.json").readline())
for k in ("pfr", "hcci"):
    v = b[k]
    print(k, round(v["value"]), v["unit"], "failed", v["failed"], "s", round(v["seconds"], 3),
          "frac", round(v["roofline"]["frac"], 4), v["solver"])
PY
exit $rc
