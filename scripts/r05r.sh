#!/bin/bash
# GPU-box: split-bf16 x6 fp32 refine kernel — parity, then the config-3 fp32 records with the exact-f32 kernel (4)
# and the x6 one (7), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_temporal.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05r_tests.log 2>&1 || { tail -30 gpurun_out/r05r_tests.log; exit 1; }
tail -2 gpurun_out/r05r_tests.log
for i in 1 2; do
  for v in 4 7; do
    timeout -k 10 200 python bench.py --only temporal --steps 50 --warmup 5 --no-cpu-baseline --option softmax_f32p=$v > gpurun_out/r05r_t${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r05r_t${v}_$i.log; exit 1; }
    python3 - "$v" "gpurun_out/r05r_t${v}_$i.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
for r in d["record"]:
    if r["dtype"] == "fp32":
        print(sys.argv[1], r["workload"][:40], r["ms_per_pair"], r["device_ms"], r["refine_kernel"][-30:],
              round(r["roofline"]["refine_conv_softmax"]["frac"], 3))
PY
  done
done
