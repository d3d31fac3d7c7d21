#!/bin/bash
# GPU-box: vectorised f32 -> bf16 convert — parity, then the UNetImage step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "convert" tests/test_gpu_image_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05y_tests.log 2>&1 || { tail -40 gpurun_out/r05y_tests.log; exit 1; }
tail -2 gpurun_out/r05y_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --only train_image --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05y_b_$i.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r05y_b_$i.log; exit 1; }
  python3 - "gpurun_out/r05y_b_$i.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["record"]
print("image step", r["ms_per_step"], r["device_ms"], r["roofline"]["frac"])
PY
done
