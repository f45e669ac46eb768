#!/bin/bash
# Time the fragment kernel with parts removed (build/librender_ablate<k>.so; wrong pixels):
# 1 = no shading, 5 = 1 + no pixel phase, 13 = 5 + no batch-0 work, 29 = 13 + no row-start state
# loads, 157 = 29 + no stores (skeleton: list load, loops).  Build first:
#   python -c "from swift3drenderer_amd import build; [build.build_library(ablate=k) for k in (1,5,13,29,157)]"
mkdir -p gpurun_out
for v in "" 1 5 13 29 157; do
  lib=swift3drenderer_amd/librender.so; [ -n "$v" ] && lib=build/librender_ablate$v.so
  for pose in P_over P_id; do
    S3R_LIB=$lib timeout -k 10 120 python bench.py --pose $pose --steps 100 --warmup 10 --no-cpu-baseline "$@" 2>>gpurun_out/tools_stderr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ablate=${v:-0}', '$pose', 'frag_ms', d['fragment_kernel_ms'], 'fps', d['value'])" || exit 1
  done
done
