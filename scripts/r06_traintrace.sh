# r06: kernel trace (queue ids) of the config-5 training step's streams
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/traintrace
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/traintrace -o run \
   -- python3 $GRAFT_REPO_ROOT/bench.py --only train --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r6r_traintrace.log 2>&1) && \
timeout -k 10 200 python3 bench.py --only train --steps 40 --warmup 5 > gpurun_out/r6r_train.log 2>&1
