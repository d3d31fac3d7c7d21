S=68x120x512x512
python tools/convbench.py --shape $S --iters 50 && python tools/convbench.py --shape $S --iters 50 --splitk || exit 1
for c in 1 3 8 9 12 20 21 23 24 26 27 31; do
  VM_LIB_PATH=$PWD/video-matting_amd/study/libvmatting_study.so timeout -k 5 60 python tools/convbench.py --shape $S --iters 50 --patch-cfg $c 2>&1 | grep -v "^total" | sed "s/^/cfg $c /" || exit 1
done
