# r06 round-end profile set, part A: headline forward (stats, MFMA busy, HBM traffic) and the split forwards
cd $GRAFT_REPO_ROOT
SKIP="temporal train train_small train_image train_chain augment loader bench" timeout -k 10 1100 bash tools/prof_bench.sh r06 > gpurun_out/r06_prof_a.log 2>&1
