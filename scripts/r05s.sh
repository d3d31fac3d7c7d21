#!/bin/bash
# GPU-box: temporal tests (error-flag handling), then the config-3 records
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_temporal.py tests/test_gpu_parity.py -k "temporal or index or correct_alpha or warp" -x -q --timeout 200 --timeout-method thread > gpurun_out/r05s_tests.log 2>&1 || { tail -30 gpurun_out/r05s_tests.log; exit 1; }
tail -2 gpurun_out/r05s_tests.log
timeout -k 10 200 python bench.py --only temporal --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r05s_t.log 2>&1 || { tail -5 gpurun_out/r05s_t.log; exit 1; }
python3 - gpurun_out/r05s_t.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for r in d["record"]:
    print(r["dtype"], r["workload"][40:60], r["ms_per_pair"], r["device_ms"],
          {k: round(v["frac"], 3) for k, v in r["roofline"].items()})
PY
