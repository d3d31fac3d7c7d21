#!/bin/bash
# GPU-box: same-box A/B of the 1080p forward between vm_set_option values (OPT="key=v1,v2"), interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
FWD="--no-cpu-baseline --no-train --no-loader --no-augment --no-temporal --no-fp32 --video-frames 0 --steps ${AB_STEPS:-200} --warmup 10"
KEY=${OPT%%=*}; VALS=${OPT#*=}
for i in ${AB_ROUNDS:-1 2}; do
  for v in ${VALS//,/ }; do
    timeout -k 10 240 python bench.py $FWD ${AB_ARGS} --option $KEY=$v --layers > gpurun_out/ab_${v}_$i.log 2>&1 || { echo "ab $v failed"; tail -5 gpurun_out/ab_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${v}_$i.log').read().strip().splitlines()[-1]); print('$KEY=$v', $i, d['value'], d['roofline']['all_mfma_convs'])"
  done
done
for v in ${VALS//,/ }; do echo "== $KEY=$v"; grep -h "conv #" gpurun_out/ab_${v}_1.log | sed 's/vm::conv3x3_//g'; done
