#!/bin/bash
# Round 5, second pass (GPU box), into gpurun_out/r05: stress setup with / without 48 of its 64 record
# bytes written (ablation build, serialised rocprof); stress parts at N = 2, 4 with 135-row bands; the
# driver's multi-GPU bench command rehearsed with 2 ranks on one GPU; the ranks-leg GPU test; the
# unchecked whole suite after an in-process RCCL gather.
set -o pipefail
OUT=gpurun_out/r05
mkdir -p "$OUT"; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
echo "stress data ready"
PROF=1 PROF_NS="1" NS="1" bash tools/stress_lib_ab.sh "base||" "rec16|build/librender_rec16.so|" 2>&1 | tee "$OUT/rec16_ab.txt" || exit 1
for n in 2 4; do
  timeout -k 10 300 python3 -u tools/parts_all.py --configs 5 --nparts $n --band 135 2>&1 | tee -a "$OUT/parts_band135.jsonl" || exit 1
done
timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --devices 0,0 --rank-devices 0,0 --gather-backend gloo --no-cpu-baseline 2>&1 | tee "$OUT/bench_rehearsal2.log" || exit 1
timeout -k 10 300 python3 -u -m pytest -v -s -m gpu --timeout 280 --timeout-method thread tests/test_bench_ranks.py 2>&1 | tee "$OUT/bench_ranks_gpu.log" || exit 1
# the round-4 abort hunt, unchecked (S3R_CHECK serialises every launch, so it cannot show a race): the
# in-process RCCL gather first, then the whole suite, output not captured (-s), so a fault's message
# and the release-time check (render_api.cpp release_all) are in the log
S3R_TEST_RCCL_INPROCESS=1 timeout -k 10 900 python3 -u -m pytest -s -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_multi.py::test_nccl_gather_in_process tests > "$OUT/rccl_unchecked.log" 2>&1 || { tail -40 "$OUT/rccl_unchecked.log"; exit 1; }
tail -3 "$OUT/rccl_unchecked.log"
