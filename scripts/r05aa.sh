#!/bin/bash
# GPU-box: vectorised BN backward — parity (kernel + training-step gradients), then the config-5 step A/B (bn_vec 0/1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_small_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05aa_tests.log 2>&1 || { tail -40 gpurun_out/r05aa_tests.log; exit 1; }
tail -2 gpurun_out/r05aa_tests.log
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --only train --steps 40 --warmup 5 --no-cpu-baseline --option bn_vec=$v > gpurun_out/r05aa_v${v}_$i.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r05aa_v${v}_$i.log; exit 1; }
    python3 - "$v" "gpurun_out/r05aa_v${v}_$i.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["record"]
print("bn_vec", sys.argv[1], r["ms_per_step"], r["device_ms"])
PY
  done
done
