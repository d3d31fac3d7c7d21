# r06: row-stationary kernel with 8-row tiles forced (rows_kernel=8) vs auto, per layer, bf16 headline and f16x3
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out
F="--steps 30 --warmup 3 --layers --no-train --no-loader --no-augment --no-temporal --no-fp32 --video-frames 0 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $F > $O/r6n_bf16_auto.log 2>&1 && \
timeout -k 10 300 python -u bench.py $F --option rows_kernel=8 > $O/r6n_bf16_rows8.log 2>&1 && \
timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6n_x3_auto.log 2>&1 && \
VM_OPT=rows_kernel=8 timeout -k 10 200 python -u tools/x6bench.py 10 f16x3 > $O/r6n_x3_rows8.log 2>&1
