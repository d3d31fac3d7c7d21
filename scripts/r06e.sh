# r06: where the f16x3 forward's error on the goldens sits (kernel / layout variants vs fp32 and bf16x6)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/x3_golden_study.py unet_video_64x96 unet_image_70x90 unet_video_70x90 > gpurun_out/r6e_study.log 2>&1
