#!/bin/bash
# GPU-box: tiled filter re-pack — parity, then the UNetImage step and the config-5 step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -k "pack" tests/test_gpu_image_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z_tests.log 2>&1 || { tail -40 gpurun_out/r05z_tests.log; exit 1; }
tail -2 gpurun_out/r05z_tests.log
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --only train_image --steps 20 --warmup 3 --no-cpu-baseline --option pack_tiled=$v > gpurun_out/r05z_b${v}_$i.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r05z_b${v}_$i.log; exit 1; }
    python3 - "$v" "gpurun_out/r05z_b${v}_$i.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["record"]
print("pack_tiled", sys.argv[1], r["ms_per_step"], r["device_ms"], r["roofline"]["frac"])
PY
  done
done
