# r06: split-K on the f16x3 forward's 68x120 convs (splitk_tiles 512 = off there, 1024 / 2048: split in 2 / 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
for v in 512 1024 2048 512; do
  VM_OPT=splitk_tiles=$v timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6x_$v.log 2>&1 || exit 1
  echo "splitk_tiles=$v $(grep ms/frame $O/r6x_$v.log) L5: $(grep -E '^\s+vm::' $O/r6x_$v.log | sed -n '11,12p' | awk '{print $(NF-5)}' | tr '\n' ' ')" >> $O/r6x_ab.txt
done
