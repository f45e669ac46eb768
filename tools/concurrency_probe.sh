#!/bin/bash
# Would overlapping frames help?  One process renders part 0 of N (4K bench workload) alone, then two
# processes do the same concurrently on the one GPU: if the pair's summed frame rate is well above the
# single one, a frame's fragment kernel leaves the chip idle (tail, launch gaps).  (GPU box)
mkdir -p gpurun_out
set -o pipefail
for n in ${PARTS:-1 8}; do
  timeout -k 10 120 python3 tools/overhead_probe.py --nparts $n --steps 2000 2>>gpurun_out/tools_stderr.log | grep '^{' \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('alone N=$n', round(1e6/d['wall_us']), 'fps')" || exit 1
  timeout -k 10 120 python3 tools/overhead_probe.py --nparts $n --steps 2000 > gpurun_out/cc_a.log 2>>gpurun_out/tools_stderr.log &
  pa=$!
  timeout -k 10 120 python3 tools/overhead_probe.py --nparts $n --steps 2000 > gpurun_out/cc_b.log 2>>gpurun_out/tools_stderr.log &
  pb=$!
  wait $pa || exit 1
  wait $pb || exit 1
  for f in gpurun_out/cc_a.log gpurun_out/cc_b.log; do
    grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  pair N=$n', round(1e6/d['wall_us']), 'fps')"
  done
done
