# r06: the probed side stream (ops.concurrent_stream): nine fresh UNetImage trainers (untraced), then the default line
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/img_streams.py probe > gpurun_out/r6q_probe.log 2>&1 && \
timeout -k 10 300 python -u tools/img_streams.py pool > gpurun_out/r6q_pool.log 2>&1 && \
timeout -k 10 700 python -u bench.py > gpurun_out/r6q_bench.log 2>&1
