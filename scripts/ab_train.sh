# A/B of two trainer versions on one box: put each version's train.py + unet_simple.py into ab/old/ and ab/new/,
# then  gpurun -- bash scripts/ab_train.sh   (3 alternating bench.py --only train runs of each)
mkdir -p gpurun_out/c17
V=video-matting_amd/vmatting
for i in 1 2 3; do
  for w in old new; do
    cp ab/$w/train.py ab/$w/unet_simple.py $V/ || exit 1
    timeout -k 10 120 python bench.py --only train --steps 30 --warmup 5 > gpurun_out/c17/$w$i.log 2>&1 || exit $?
    echo "$w $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c17/$w$i.log)"
  done
done
