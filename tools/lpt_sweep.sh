#!/bin/bash
# The longest-first fragment order's threshold (S3R_LPT_MIN bins) on launches just below the default:
# 3840x2160 part 0 of 8 (2 040 bins), 1920x1080 whole (flat), 7680x4320 part 0 of 8 (2 700 bins).
mkdir -p gpurun_out
set -o pipefail
for rep in 1 2; do
for case in "3840 2160 8 full" "1920 1080 1 flat" "7680 4320 8 full"; do
  set -- $case
  for spec in "default|" "lpt2000|S3R_LPT_MIN=2000"; do
    IFS='|' read -r tag envs <<< "$spec"
    env $envs timeout -k 10 120 python3 tools/overhead_probe.py --width $1 --height $2 --nparts $3 --scene $4 --steps 2000 2>>gpurun_out/tools_stderr.log \
      | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1x$2 N=$3 $4 $tag', round(1e6/d['wall_us']), round(d['frag_us'],1))" || exit 1
  done
done
done
