#!/bin/bash
# round-3 GPU check of the packed-frames patch tiling: parity + training tests, same-box headline A/B against
# ab/libvmatting_base.so, and the training step with packing on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -q -x --timeout 200 \
    --timeout-method thread -rf > gpurun_out/pt_pack.log 2>&1; rc=$?; tail -4 gpurun_out/pt_pack.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS="1 2" AB_STEPS=200 bash scripts/ab_bench.sh || exit $?
for o in 1 0 1 0; do
  timeout -k 10 300 python bench.py --only train --steps 30 --warmup 5 --option pack_frames=$o > gpurun_out/train_pack$o.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/train_pack$o.log').read().strip().splitlines()[-1]); print('pack', $o, d['record']['ms_per_step'], d['record']['device_ms'])"
done
