# r06: MFMA head with 16-byte weight staging (tests, f16x3 timing, UNetImage step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split3.py tests/test_gpu_parity.py tests/test_gpu_split6.py tests/test_gpu_image_train.py -m gpu > $O/r6u_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6u_x3.log 2>&1 && \
timeout -k 10 200 python -u bench.py --only train_image --steps 30 --warmup 5 > $O/r6u_img.log 2>&1
