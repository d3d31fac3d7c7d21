# r06: kernel stats of the f16x3 forward alone (after the head's 16-byte weight staging)
cd $GRAFT_REPO_ROOT
SKIP="fwd mfma traffic temporal train train_small train_image train_chain augment loader x6 bench" timeout -k 10 400 bash tools/prof_bench.sh r06 > gpurun_out/r06_prof_x3.log 2>&1
