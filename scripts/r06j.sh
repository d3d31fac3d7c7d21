# r06: f16x3 with the one-call aliased head and the two-slab input split (tests, timing, kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_gpu_split3.py -m gpu -s > $O/r6j_test.log 2>&1 && \
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6j_x3.log 2>&1 && \
SKIP="fwd mfma traffic temporal train train_small train_image train_chain augment loader x6 bench" timeout -k 10 300 bash tools/prof_bench.sh r06j > $O/r6j_prof.log 2>&1
