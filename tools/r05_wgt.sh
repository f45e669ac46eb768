# per-workgroup timelines of k_fragment (timing build), 4K P_over whole frame and part 0 of 8, raw dumps
set -o pipefail
mkdir -p gpurun_out/wgt
S3R_WGT_DUMP=gpurun_out/wgt/n1.npy timeout -k 10 240 python -u tools/wg_timeline.py > gpurun_out/wgt/n1.txt 2>&1 &&
S3R_LPT_MIN=100000000 S3R_WGT_DUMP=gpurun_out/wgt/n1_nolpt.npy timeout -k 10 240 python -u tools/wg_timeline.py > gpurun_out/wgt/n1_nolpt.txt 2>&1 &&
S3R_WGT_DUMP=gpurun_out/wgt/n8.npy timeout -k 10 240 python -u tools/wg_timeline.py --nparts 8 > gpurun_out/wgt/n8.txt 2>&1
