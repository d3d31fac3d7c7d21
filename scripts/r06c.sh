# r06: folded upconvs, rows kernel split form, conv1_1 slab 8 on the f16x3 path (tests, timing) + how the trainers'
# side streams land on hardware queues
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_gpu_split3.py -m gpu -s > $O/r6c_test.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc; \
timeout -k 10 240 python -u tools/x6bench.py 10 f16x3 > $O/r6c_x3.log 2>&1 && \
VM_OPT=rows_kernel=0 timeout -k 10 240 python -u tools/x6bench.py 10 f16x3 > $O/r6c_x3_norows.log 2>&1 && \
for cfg in "0 4" "8 4" "0 8" "8 8" "0 16"; do set -- $cfg; GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python -u bench.py --only train_image --steps 40 --warmup 5 --dummy-streams $1 > $O/r6c_img_$1_$2.log 2>&1 || exit 1; echo "img dummy=$1 hwq=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/r6c_img_$1_$2.log | head -1)"; done && \
for cfg in "0 4" "8 4" "0 8" "8 8"; do set -- $cfg; GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python -u bench.py --only train --steps 40 --warmup 5 --dummy-streams $1 > $O/r6c_trn_$1_$2.log 2>&1 || exit 1; echo "train dummy=$1 hwq=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/r6c_trn_$1_$2.log | head -1)"; done
