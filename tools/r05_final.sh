#!/bin/bash
# Round 5 final evidence (GPU box): the GPU suite, every part of the N-way splits, the round evidence
# (default-workload and stress profiles with PMC passes, the bench matrix, the default bench line).
set -o pipefail
mkdir -p gpurun_out/r05 gpurun_out/ev_r05; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/gputest_final.log 2>&1 \
    || { tail -40 gpurun_out/r05/gputest_final.log; exit 1; }
tail -2 gpurun_out/r05/gputest_final.log
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
timeout -k 10 600 python3 -u tools/parts_all.py --configs 3,4,5 --out gpurun_out/r05/parts_all_final.jsonl > gpurun_out/r05/parts_all_final.log 2>&1 \
    || { tail -20 gpurun_out/r05/parts_all_final.log; exit 1; }
echo "parts done"
bash tools/round_evidence.sh gpurun_out/ev_r05 || exit 1
du -sh gpurun_out
