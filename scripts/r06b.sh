# r06: trainers with the vectorised weight-gradient reduction (tests + A/B), then the full bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_image_train.py tests/test_gpu_small_train.py -m gpu > $O/r6b_tests.log 2>&1 && \
for v in 0 1 0 1; do timeout -k 10 200 python -u bench.py --only train_image --steps 40 --warmup 5 --option wgrad_reduce4=$v > $O/r6b_img_$v.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' $O/r6b_img_$v.log | head -1; done && \
timeout -k 10 900 python -u bench.py > $O/r6b_bench.log 2>&1
