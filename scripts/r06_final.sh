# r06 final: the whole GPU suite, then the default bench line
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_final_gputests.log 2>&1 || exit 1
