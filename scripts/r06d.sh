# r06: f16x3 with the resized (unfolded) upconvs + rows split kernel + conv1_1 slab 8 (tests, timing); the narrow-input
# conv kernel for UNetSmall (tests, train_small profile)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_narrowin.py tests/test_gpu_small_train.py -m gpu > $O/r6d_narrow.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_gpu_split3.py -m gpu -s > $O/r6d_test.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc; \
timeout -k 10 240 python -u tools/x6bench.py 10 f16x3 bf16x6 > $O/r6d_x3.log 2>&1 && \
SKIP="fwd mfma traffic temporal train train_image train_chain augment loader x3 x6 bench" timeout -k 10 300 bash tools/prof_bench.sh r06d > $O/r6d_prof.log 2>&1
