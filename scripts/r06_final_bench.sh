# r06 final: the default bench line on the final code
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u bench.py > gpurun_out/r06_final_bench.log 2>&1 && tail -n 1 gpurun_out/r06_final_bench.log > gpurun_out/r06_final_bench.json
