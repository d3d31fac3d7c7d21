# r06: f16x3 upconv_2 / _3 on the 3-slot ring (tests, timing); the full bench line again (train_image per-step spread)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_gpu_split3.py -m gpu -s > $O/r6l_test.log 2>&1 && \
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6l_x3.log 2>&1 && \
timeout -k 10 700 python -u bench.py > $O/r6l_bench.log 2>&1
