# r06 round-end profile set, part B: config-3, the training steps, the chained config-5 pipeline, augment, loader
cd $GRAFT_REPO_ROOT
SKIP="fwd mfma traffic x3 x6 bench" timeout -k 10 1150 bash tools/prof_bench.sh r06 > gpurun_out/r06_prof_b.log 2>&1
