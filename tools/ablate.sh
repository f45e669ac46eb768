#!/bin/bash
# Time the fragment kernel with parts removed (build/librender_ablate{1,2,3}.so; wrong pixels).
# 1 = no shading, 2 = no per-pixel fallback walk, 3 = both, 5 = no shading + no pixel phase,
# 13 = no shading + no batch-0 work at all (skeleton: list load, row-start loads, loop, stores),
# 61 = 13 without the row-start and list loads, 189 = 61 without the stores.
for v in "" 13 61 189; do
  lib=swift3drenderer_amd/librender.so; [ -n "$v" ] && lib=build/librender_ablate$v.so
  for pose in P_over P_id; do
    S3R_LIB=$lib timeout -k 10 120 python bench.py --pose $pose --steps 100 --warmup 10 --no-cpu-baseline --no-e2e 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ablate=${v:-0}', '$pose', 'frag_ms', d['fragment_kernel_ms'])" || exit 1
  done
done
