#!/bin/bash
# Round 5 measurements on the GPU box, into gpurun_out/r05:
#   every part of the N-way splits (configs 3, 4, 5; N = 1, 2, 4, 8) -> parts_all.jsonl;
#   the stress setup with and without its raster-record writes (ablation build, serialised rocprof);
#   the driver's multi-GPU bench command rehearsed with 2 ranks on the one GPU (gloo gather).
set -o pipefail
OUT=gpurun_out/r05
mkdir -p "$OUT"; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
echo "stress data ready"
timeout -k 10 600 python3 -u tools/parts_all.py --configs 3,4,5 --out "$OUT/parts_all.jsonl" > "$OUT/parts_all.log" 2>&1 || { tail -20 "$OUT/parts_all.log"; exit 1; }
cat "$OUT/parts_all.log" | grep '^{' | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], 'N', d['N'], 'band', d['band'], 'slowest', d['slowest_us'], 'max/mean', d['max_over_mean'], 'eff', d['efficiency_per_gpu'])"
PROF=1 PROF_NS="1" NS="1" bash tools/stress_lib_ab.sh "base||" "norec|build/librender_norec.so|" > "$OUT/norec_ab.txt" 2>&1 || { tail -20 "$OUT/norec_ab.txt"; exit 1; }
cat "$OUT/norec_ab.txt"
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --devices 0,0 --rank-devices 0,0 --gather-backend gloo --no-cpu-baseline > "$OUT/bench_rehearsal2.log" 2>&1 \
    || { tail -30 "$OUT/bench_rehearsal2.log"; exit 1; }
grep '^{' "$OUT/bench_rehearsal2.log" | tail -1 > "$OUT/bench_rehearsal2.json"
python3 -c "import json; d=json.load(open('$OUT/bench_rehearsal2.json')); print(json.dumps(d['ranks'], indent=1)); print('value', d['value'])"
timeout -k 10 300 python3 -u -m pytest -v -s -m gpu --timeout 280 --timeout-method thread tests/test_bench_ranks.py > "$OUT/bench_ranks_gpu.log" 2>&1 || { tail -30 "$OUT/bench_ranks_gpu.log"; exit 1; }
grep -E "PASS|FAIL" "$OUT/bench_ranks_gpu.log" | head
# the round-4 abort hunt, unchecked (S3R_CHECK serialises every launch, so it cannot show a race): the
# in-process RCCL gather first, then the whole suite, output not captured (-s), so a fault's message
# and the release-time check (render_api.cpp release_all) are in the log
S3R_TEST_RCCL_INPROCESS=1 timeout -k 10 900 python3 -u -m pytest -s -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_multi.py::test_nccl_gather_in_process tests > "$OUT/rccl_unchecked.log" 2>&1 || { tail -40 "$OUT/rccl_unchecked.log"; exit 1; }
tail -3 "$OUT/rccl_unchecked.log"
