#!/bin/bash
# GPU-box: same-box A/B of the 1080p forward between ab/libvmatting_base.so and the in-tree build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
FWD="--no-cpu-baseline --no-train --no-loader --no-augment --no-temporal --no-fp32 --video-frames 0 --steps ${AB_STEPS:-200} --warmup 10"
for i in ${AB_ROUNDS:-1 2}; do
  for v in base new; do
    if [ $v = base ]; then L=$PWD/ab/libvmatting_base.so; else L=; fi
    VM_LIB_PATH=$L timeout -k 10 240 python bench.py $FWD ${AB_ARGS} --layers > gpurun_out/ab_${v}_$i.log 2>&1 || { echo "ab $v failed"; tail -5 gpurun_out/ab_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${v}_$i.log').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['roofline']['all_mfma_convs'])"
  done
done
grep -h "conv #" gpurun_out/ab_base_1.log > gpurun_out/ab_layers_base.txt
grep -h "conv #" gpurun_out/ab_new_1.log > gpurun_out/ab_layers_new.txt
paste gpurun_out/ab_layers_base.txt gpurun_out/ab_layers_new.txt | awk -F'\t' '{print $1 " | " $2}' | sed 's/vm::conv3x3_//g'
