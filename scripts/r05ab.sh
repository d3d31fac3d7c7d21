#!/bin/bash
# GPU-box: vectorised forward BN — parity (kernels, goldens, training steps), then the config-5 step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_small_train.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ab_tests.log 2>&1 || { tail -40 gpurun_out/r05ab_tests.log; exit 1; }
tail -2 gpurun_out/r05ab_tests.log
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --only train --steps 40 --warmup 5 --no-cpu-baseline --option bn_vec_fwd=$v > gpurun_out/r05ab_v${v}_$i.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r05ab_v${v}_$i.log; exit 1; }
    python3 - "$v" "gpurun_out/r05ab_v${v}_$i.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["record"]
print("bn_vec_fwd", sys.argv[1], r["ms_per_step"], r["device_ms"])
PY
  done
done
