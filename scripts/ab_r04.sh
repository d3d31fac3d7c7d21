#!/bin/bash
# GPU-box: same-box A/B of the 1080p forward, the round-4 build (abr04/, built from commit 53643ad) vs HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
FWD="--no-cpu-baseline --no-train --no-loader --no-augment --no-temporal --no-fp32 --video-frames 0 --steps ${AB_STEPS:-200} --warmup 10"
for i in 1 2 3; do
  for v in r04 head; do
    if [ $v = r04 ]; then L=$PWD/abr04/libvmatting_r04.so; else L=; fi
    VM_LIB_PATH=$L timeout -k 10 240 python bench.py $FWD --layers > gpurun_out/abr04_${v}_$i.log 2>&1 || { echo "ab $v failed"; tail -5 gpurun_out/abr04_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abr04_${v}_$i.log').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['roofline']['all_mfma_convs'])"
  done
done
paste <(grep -h "conv #" gpurun_out/abr04_r04_1.log) <(grep -h "conv #" gpurun_out/abr04_head_1.log) | awk -F'\t' '{print $1 " | " $2}' | sed 's/vm::conv3x3_//g'
