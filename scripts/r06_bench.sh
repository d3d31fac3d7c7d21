# r06 round-end: the default bench line (N=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u bench.py > gpurun_out/r06_bench.log 2>&1 && \
tail -n 1 gpurun_out/r06_bench.log > gpurun_out/r06_bench.json
