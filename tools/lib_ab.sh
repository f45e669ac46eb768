#!/bin/bash
# Frame rate and HIP-event fragment time of the bench workload for several library builds / knob
# settings on one box.  Usage: bash tools/lib_ab.sh 'tag|lib|ENV=.. ENV=..' ...  (lib '' = the product
# library; GPU box).  BENCH_EXTRA: extra bench.py arguments.
mkdir -p gpurun_out
set -o pipefail
for spec in "$@"; do
  IFS='|' read -r tag lib envs <<< "$spec"
  env $envs ${lib:+S3R_LIB=$lib} timeout -k 10 120 python3 bench.py --steps 400 --warmup 40 --no-cpu-baseline $BENCH_EXTRA 2>>gpurun_out/tools_stderr.log \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), 'fps  device_fps', round(d['device_fps']), ' frag_ms', d['fragment_kernel_ms'])" || exit 1
done
# part 0 of 8 (one rank of an 8-GPU band split) when PARTS8=1
if [ -n "$PARTS8" ]; then
  for spec in "$@"; do
    IFS='|' read -r tag lib envs <<< "$spec"
    env $envs ${lib:+S3R_LIB=$lib} timeout -k 10 120 python3 tools/overhead_probe.py --nparts 8 --steps 2000 2>>gpurun_out/tools_stderr.log | grep '^{' \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag part 1/8', round(1e6/d['wall_us']), 'fps  frag_us', round(d['frag_us'],1))" || exit 1
  done
fi
