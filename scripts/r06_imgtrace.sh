# r06: kernel traces (queue ids) of nine fresh UNetImage trainers per side-stream kind (pool / masked / high)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for kind in ${KINDS:-pool masked high}; do
  mkdir -p gpurun_out/imgtrace_$kind
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/imgtrace_$kind -o run \
     -- python3 $GRAFT_REPO_ROOT/tools/img_streams.py $kind > $GRAFT_REPO_ROOT/gpurun_out/r6o_imgtrace_$kind.log 2>&1) || exit 1
done
