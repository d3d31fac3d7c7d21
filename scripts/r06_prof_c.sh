# r06 round-end profile set, part C (after the last changes): the split forwards and the UNetImage step
cd $GRAFT_REPO_ROOT
SKIP="fwd mfma traffic temporal train train_small train_chain augment loader bench" timeout -k 10 900 bash tools/prof_bench.sh r06 > gpurun_out/r06_prof_c.log 2>&1
