# r06: f16x3 with conv1_1 slabs of 32 (tests, timing); small_train's bf16 data gradients on the narrow-input kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_narrowin.py tests/test_gpu_small_train.py -m gpu > $O/r6f_narrow.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_gpu_split3.py -m gpu -s > $O/r6f_test.log 2>&1 && \
timeout -k 10 240 python -u tools/x6bench.py 10 f16x3 > $O/r6f_x3.log 2>&1 && \
SKIP="fwd mfma traffic temporal train train_image train_chain augment loader x3 x6 bench" timeout -k 10 300 bash tools/prof_bench.sh r06f > $O/r6f_prof.log 2>&1
