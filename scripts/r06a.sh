set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_split3.py -m gpu -k "not 1080p" > gpurun_out/r6a_test.log 2>&1 && \
timeout -k 10 240 python -u tools/x6bench.py 10 f16x3 bf16x6 bf16 > gpurun_out/r6a_bench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_split3.py -m gpu -k "1080p" -s > gpurun_out/r6a_1080.log 2>&1
