# A/B of two versions of the host layer (_lib.py + ops.py) on one box: ab/old/ and ab/new/ hold them
#   gpurun -- bash scripts/ab_host.sh   (3 alternating bench.py --only train runs of each)
mkdir -p gpurun_out/c28
V=video-matting_amd/vmatting
for i in 1 2 3; do
  for w in old new; do
    cp ab/$w/_lib.py ab/$w/ops.py $V/ || exit 1
    timeout -k 10 120 python bench.py --only train --steps 30 --warmup 5 > gpurun_out/c28/$w$i.log 2>&1 || exit $?
    echo "$w $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c28/$w$i.log) $(grep -o '"device_ms": {[^}]*}' gpurun_out/c28/$w$i.log)"
  done
done
cp ab/new/_lib.py ab/new/ops.py $V/
