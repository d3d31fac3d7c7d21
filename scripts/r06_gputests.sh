# r06 round-end: the whole GPU suite, one process
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gputests.log 2>&1
