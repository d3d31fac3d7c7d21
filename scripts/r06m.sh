# r06: the UNetImage step against the pool position of its side stream
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/img_streams.py > gpurun_out/r6m_streams.log 2>&1
