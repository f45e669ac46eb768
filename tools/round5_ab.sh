#!/bin/bash
# Round 5's GPU-box experiments, one recipe each:  bash tools/round5_ab.sh <recipe>
# Every recipe writes under gpurun_out/<recipe>/; the summaries kept are the profiles/r05_*.txt files
# named beside each recipe.  Variant libraries (build/librender_<tag>.so) are made here beforehand with
# swift3drenderer_amd.build.build_variant(tag, {defines}); ablation builds render wrong pixels on purpose.
#
#   check     the GPU suite with every launch checked (S3R_CHECK=1), then the in-process RCCL gather
#             followed by the multi-device and tile suites         -> r05_gputest_check.log, r05_rccl_*.log
#   measure   every part of the N-way splits (configs 3/4/5), 135-row stress bands, the 16-B record
#             ablation (rec16), the 2-rank bench rehearsal, the unchecked suite after an RCCL gather
#                                                                   -> r05_parts_all*.jsonl, r05_rec16_ablation.txt
#   ntrec     raster records / bin entries stored non-temporal (ntrec / ntall builds) -> r05_ntrec_ab.txt
#   tablewalk table walk vs the linear-run k_fragment (alltab / segst / at7a / at7b / tw8 / tw9 builds:
#             parity of the row-path suites, frame rates, rocprof, SQ counters)
#                                                                   -> r05_fragment_ab.txt, r05_alltab_pmc.txt,
#                                                                      r05_fragment_occupancy_ab.txt, r05_tablewalk_tuning_ab.txt
#   wgt       per-workgroup k_fragment timelines (wgt build): 4K whole frame (work-unit order and launch
#             order) and part 0 of 8, raw dumps                     -> r05_order_ab.txt
#   seg       k_fragment segment widths 6 / 3 / 2 / 1 chunks at 4K  (negative, DESIGN Row path)
#   order     bin order by work units vs wall time (owall build): bench at 4K / 8K / P_id, part 0 of 8,
#             pipelined periods, geometry priority, rocprof traces, diagnosis builds -> r05_order_ab.txt
#   geo       k_geometry walk counters (stats build, --device) and per-workgroup timelines (wgt build:
#             HBM frames serialised / pipelined, delivered frames), a kernel trace of delivered frames
#   pf2       two-deep k_tile_setup pipeline vs the build before it  -> r05_setup_pf2_ab.txt
#   defer     k_tile_setup binning pipelined one iteration deep (negative) -> r05_defer_bins_negative.txt
#   tvruns    tile_visit key groups as runs of adjacent lanes vs the loop over distinct keys (tvloop
#             build), and the branch-free raster pixel loop (tbl build), with SQ counters; the stress
#             frame's staged / depth-culled (slot, tile) pairs (stats build); tab8: the raster's row and x
#             walks replaced by one multiply-add (timing only); trs: each staged triangle's walk down to
#             the tile's first row done once at staging (S3R_TROWSTART)
#   ob        the longest-first order's cost buckets at 1/8 octave (ob8 build) instead of 1/4
#   order1080 the bin orders (work units / wall time / launch order) at 1080p (flat, full) and 4K
#   georows   k_geometry row blocks of 256 / 320 rows (geo256 / geo320 builds) instead of 128
#   rasterpf  fused raster: list entries prefetched two stages ahead (tpf2), one 16-B read per row in the
#             per-triangle depth cull (tzv4), occupancy caps 5 / 6 (o5 / o6 builds, S3R_TOCC)
#   rasterocc fused raster occupancy caps 6 / 7 (to6 / to7), and 128-triangle stages for delivered frames
#             at occupancy 6 (to6l128): stress N=1 / part 0 of 8, delivered and device bench lines
#   setupocc  k_tile_setup occupancy caps 7 / 8 (so7 / so8 builds, S3R_SOCC)
#   setupgrid tile-path kernels' workgroups per shard (S3R_TILE_GRID 1024 default / 256 / 24 / 16)
#   fragocc   k_fragment's non-waterfall instance (2-chunk bins: 1080p, 4K / 8K parts) at occupancy 6
#             (occ6 build: 80 VGPRs, 16 spilled) vs 5: every part of configs 3 and 4, 1080p bench lines
#   stage192  the delivered frames' fused raster staging 192 triangles (tl192: 28.7 KB LDS, occupancy 5)
#             instead of 256 (35.4 KB, occupancy 4)
#   rec48     48-B raster records (box, bound, 1/z, the three raster corners; the raster and the resolve
#             recompute wstart and the steps: rec48 build, S3R_REC48) vs the 64-B records (product)
#   rec48s6   the 48-B records with k_tile_setup capped at 80 VGPRs (occupancy 6, as the 64-B build had)
#   rec48b    the 48-B records again, the corners stored before the depth bound (fewer live registers)
#   clshallow frame parts' setup (clusters) one deep again (product) vs two deep (prev build)
#   linfast   k_fragment: triangles whose three components are exactly linear over the chunk skip the
#             table fill (values c + k delta where read; linf build, S3R_LINFAST) vs every chunk tabled
#   (rec0     every tile frame without records -- an S3R_REC0 build since folded into the product for
#             delivered frames; its numbers and counters are in r05_rec0_ab.txt, the recipe is gone)
#   norec     delivered tile frames without raster records for the slots the raster sets up again
#             (product) vs the build before (prev: build_variant("prev") from commit 64b5d0e~3) and
#             S3R_TILE_NOREC=0: GPU suite, stress N=1 / part 0 of 8,
#             bench lines, delivered-frame rocprof                   -> r05_rec0_ab.txt
#   (norec2   frame parts without records too (a build of that session, S3R_TILE_NOREC=1 then) vs delivered
#             frames only (=2, now the product): not kept -- part 0 of 8 at the library's 135-row band
#             6 677 -> 6 370 fps (+7 % at 16-row bands); r05_rec0_ab.txt, the recipe is gone)
#   slotcull  k_geometry launching only the slots the host's cull keeps (product) vs every slot
#             (S3R_SLOT_CULL=0): parity suites, 4K / P_id / 8K / 1080p bench lines, geometry timelines
#   slotcull2 the same, device and delivered rates only, three alternating repetitions, overhead probes
#   slotcull3 1080p delivered frames, the variants in the other order
#   (socc6    the record-writing k_tile_setup instances capped at 80 VGPRs: negative, in r05_rec0_ab.txt;
#             the recipe and its S3R_SOCC_REC build are gone)
#   rcres     the recomputing raster's resolve in two phases (positions, then shading constants: 36 B
#             spilled at 80 VGPRs instead of 128) for every frame (S3R_TILE_NOREC=2 of that build) vs
#             records, and with the depth bucket's ceiling as the staged bound (rcbb build: 8 B) -- the
#             product since; the recipe's builds and knob values are gone  -> r05_rec0_ab.txt
#   cullparts part 0 of 8 and whole 4K frames (overhead probes, host enqueue time), cull vs no cull
#                                                                   -> r05_slot_cull_ab.txt
#   nearck    k_geometry without the clip-appended slots when the host's near-plane check allows it
#             (product) vs always with them (noclipck build): parity, delivered frames, geometry timeline
mkdir -p gpurun_out
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${1:?recipe}
OUT=gpurun_out/$R; mkdir -p "$OUT"
D=/tmp/s3r_stress.bin
stress_data() { [ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')"; }
gpu_suite() {   # log, pytest args...
  local log=$1; shift
  timeout -k 10 900 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread "$@" > "$log" 2>&1 || { tail -30 "$log"; return 1; }
  tail -1 "$log"
}
probe() {       # tag, env..., then overhead_probe args after --
  local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 180 python3 tools/overhead_probe.py "$@" 2>>gpurun_out/tools_stderr.log | grep '^{' | sed "s/^/$tag /" | cut -c1-200
}

case $R in
check)
  S3R_CHECK=1 gpu_suite $OUT/gputest_check.log tests || exit 1
  S3R_CHECK=1 S3R_TEST_RCCL_INPROCESS=1 gpu_suite $OUT/rccl_experiment.log tests/test_multi.py::test_nccl_gather_in_process \
      tests/test_multi_device.py tests/test_tiles.py || exit 1 ;;
measure)
  stress_data || exit 1
  timeout -k 10 600 python3 -u tools/parts_all.py --configs 3,4,5 --out $OUT/parts_all.jsonl > $OUT/parts_all.log 2>&1 || exit 1
  for n in 2 4; do timeout -k 10 300 python3 -u tools/parts_all.py --configs 5 --nparts $n --band 135 >> $OUT/parts_band135.jsonl || exit 1; done
  PROF=1 PROF_NS="1" NS="1" bash tools/stress_lib_ab.sh "base||" "rec16|build/librender_rec16.so|" 2>&1 | tee $OUT/rec16_ab.txt || exit 1
  timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
      bench.py --gpus 2 --devices 0,0 --rank-devices 0,0 --gather-backend gloo --no-cpu-baseline > $OUT/bench_rehearsal2.log 2>&1 || exit 1
  gpu_suite $OUT/bench_ranks_gpu.log tests/test_bench_ranks.py || exit 1
  S3R_TEST_RCCL_INPROCESS=1 gpu_suite $OUT/rccl_unchecked.log -s tests/test_multi.py::test_nccl_gather_in_process tests || exit 1 ;;
ntrec)
  stress_data || exit 1
  NS="1 8" BAND=135 PROF=1 PROF_NS="1" bash tools/stress_lib_ab.sh "base||" "ntrec|build/librender_ntrec.so|" \
      "ntall|build/librender_ntall.so|" "base2||" 2>&1 | tee $OUT/ntrec_ab.txt ;;
tablewalk)
  for v in alltab segst at7a at7b tw8 tw9; do
    S3R_LIB=build/librender_$v.so gpu_suite $OUT/${v}_parity.log tests/test_gpu_parity.py tests/test_multi_device.py tests/test_multi.py || exit 1
  done
  PARTS8=1 bash tools/lib_ab.sh "base||" "alltab|build/librender_alltab.so|" "segst|build/librender_segst.so|" \
      "at7a|build/librender_at7a.so|" "at7b|build/librender_at7b.so|" "tw8|build/librender_tw8.so|" \
      "base_wf||S3R_WATERFALL_BINS=0" "base2||" 2>&1 | tee $OUT/ab.txt || exit 1
  cp swift3drenderer_amd/librender.so build/librender_prod.so
  S3R_VARIANTS='{"prod": {}, "alltab": {}, "segst": {}, "at7a": {}, "tw8": {}, "tw9": {}}' S3R_VARIANT_BENCH="--scene full --pose P_over" \
      timeout -k 10 900 python3 tools/variants.py run 2>&1 | tee -a $OUT/ab.txt || exit 1
  find gpurun_out/variants \( -name '*kernel_trace.csv' -o -name '*agent_info.csv' \) -delete
  bash tools/variant_pmc.sh $OUT/vpmc prod alltab segst 2>&1 | tee $OUT/pmc.txt ;;
wgt)
  S3R_WGT_DUMP=$OUT/n1.npy timeout -k 10 240 python3 -u tools/wg_timeline.py > $OUT/n1.txt 2>&1 &&
  S3R_LPT_MIN=100000000 S3R_WGT_DUMP=$OUT/n1_nolpt.npy timeout -k 10 240 python3 -u tools/wg_timeline.py > $OUT/n1_nolpt.txt 2>&1 &&
  S3R_WGT_DUMP=$OUT/n8.npy timeout -k 10 240 python3 -u tools/wg_timeline.py --nparts 8 > $OUT/n8.txt 2>&1 ;;
seg)
  PARTS8=1 bash tools/lib_ab.sh 'base||' 'seg3||S3R_SEG3=1 S3R_MIN_BLOCKS=6000' 'seg2||S3R_MIN_BLOCKS=8000' \
      'seg1||S3R_MIN_BLOCKS=20000' 'base2||' 2>&1 | tee $OUT/ab.txt ;;
order)
  W=build/librender_owall.so
  PARTS8=1 bash tools/lib_ab.sh 'work||' "wall|$W|" 'work2||' "wall2|$W|" 2>&1 | tee $OUT/ab4k.txt || exit 1
  BENCH_EXTRA='--width 7680 --height 4320' bash tools/lib_ab.sh 'work 8K||' "wall 8K|$W|" 2>&1 | tee $OUT/ab8k.txt || exit 1
  BENCH_EXTRA='--pose P_id' bash tools/lib_ab.sh 'work P_id||' "wall P_id|$W|" 2>&1 | tee $OUT/abpid.txt || exit 1
  for rep in 1 2; do
    for spec in "work|" "wall|S3R_LIB=$W" "wsky|S3R_LIB=build/librender_wsky.so" "wgeo|S3R_LIB=build/librender_wgeo.so" \
                "owgeo|S3R_LIB=build/librender_owgeo.so"; do
      IFS='|' read -r tag envs <<< "$spec"
      probe $tag $envs -- --steps 2000 | tee -a $OUT/probe.txt || exit 1
    done
  done
  for spec in "work|" "wall|$W"; do
    IFS='|' read -r tag lib <<< "$spec"
    S3R_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$tag -o tr -- \
        python3 tools/overhead_probe.py --steps 300 > $OUT/tr_$tag.log 2>&1 || exit 1
    f=$(find $OUT/tr_$tag -name '*kernel_trace.csv' | head -1)
    python3 tools/trace_timeline.py "$f" --first 200 --count 12 > $OUT/timeline_$tag.txt || exit 1
    rm -f "$f"
  done ;;
geo)
  timeout -k 10 180 python3 tools/frame_stats.py --device > $OUT/stats_dev.txt 2>&1 || exit 1
  S3R_SERIAL=1 timeout -k 10 180 python3 tools/geo_timeline.py > $OUT/serial.txt 2>&1 || exit 1
  timeout -k 10 180 python3 tools/geo_timeline.py > $OUT/pipelined.txt 2>&1 || exit 1
  timeout -k 10 180 python3 tools/geo_timeline.py --delivered > $OUT/delivered.txt 2>&1 || exit 1
  S3R_LIB= timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- \
      python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-device > $OUT/tr.log 2>&1 || exit 1
  f=$(find $OUT/tr -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_timeline.py "$f" --first -40 --count 8 > $OUT/timeline_delivered.txt || exit 1
  rm -f "$f" ;;
pf2)
  gpu_suite $OUT/tiles.log tests/test_tiles.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'pf2||' 'old|build/librender_old.so|' 'pf2b||' \
      'oldb|build/librender_old.so|' 2>&1 | tee $OUT/stress_ab.txt ;;
defer)
  gpu_suite $OUT/tiles.log tests/test_tiles.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1" bash tools/stress_lib_ab.sh 'defer|build/librender_defer.so|' 'base||' \
      'defer_g256|build/librender_defer.so|S3R_TILE_GRID=256' 'base_g256||S3R_TILE_GRID=256' \
      'defer_g64|build/librender_defer.so|S3R_TILE_GRID=64' 'base_g64||S3R_TILE_GRID=64' 2>&1 | tee $OUT/ab.txt ;;
tvruns)
  S3R_LIB=build/librender_tbl.so gpu_suite $OUT/tests.log tests/test_tiles.py || exit 1
  S3R_LIB=build/librender_trs.so gpu_suite $OUT/tests_trs.log tests/test_tiles.py || exit 1
  timeout -k 10 300 python3 tools/tile_stats.py > $OUT/tile_stats.txt 2>&1 || { tail -5 $OUT/tile_stats.txt; exit 1; }
  cat $OUT/tile_stats.txt
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'runs||' 'loop|build/librender_tvloop.so|' 'tbl|build/librender_tbl.so|' \
      'runs2||' 'loop2|build/librender_tvloop.so|' 'tbl2|build/librender_tbl.so|' 'tab8|build/librender_tab8.so|' 'trs|build/librender_trs.so|' 'trs2|build/librender_trs.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  for spec in 'runs|' 'loop|build/librender_tvloop.so' 'tbl|build/librender_tbl.so'; do
    IFS='|' read -r tag lib <<< "$spec"
    env S3R_SERIAL=1 ${lib:+S3R_LIB=$lib} timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
        SQ_BUSY_CYCLES --output-format csv -d "$PWD/$OUT/pmc_$tag" -o run -- python3 tools/overhead_probe.py --scene icosa-stress \
        --pose P_id --data $D --steps 10 > $OUT/pmc_$tag.log 2>&1 || { tail -5 $OUT/pmc_$tag.log; exit 1; }
    python3 tools/pmc_summary.py $OUT/pmc_$tag --last 10 > $OUT/pmc_$tag.txt 2>&1 || true
    find $OUT/pmc_$tag -name '*.csv' -size +5M -delete
  done ;;
ob)
  PARTS8=1 bash tools/lib_ab.sh 'base||' 'ob8|build/librender_ob8.so|' 'base2||' 'ob8b|build/librender_ob8.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  BENCH_EXTRA='--pose P_id' bash tools/lib_ab.sh 'base P_id||' 'ob8 P_id|build/librender_ob8.so|' 2>&1 | tee -a $OUT/ab.txt ;;
nearck)
  gpu_suite $OUT/parity.log tests/test_gpu_parity.py tests/test_host_loop.py tests/test_multi_device.py tests/test_abi.py || exit 1
  timeout -k 10 180 python3 tools/geo_timeline.py --delivered > $OUT/geo_delivered.txt 2>&1 || exit 1
  for rep in 1 2; do
    bash tools/lib_ab.sh 'check||' 'nocheck|build/librender_noclipck.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  BENCH_EXTRA='--pose P_id' bash tools/lib_ab.sh 'check P_id||' 'nocheck P_id|build/librender_noclipck.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'check 1080p||' 'nocheck 1080p|build/librender_noclipck.so|' 2>&1 | tee -a $OUT/ab.txt ;;
order1080)
  for rep in 1 2; do
    BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'work 1080p||' 'wall 1080p|build/librender_owall.so|' \
        'launch 1080p||S3R_LPT_MIN=100000000' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  BENCH_EXTRA='--scene full --width 1920 --height 1080' bash tools/lib_ab.sh 'work full1080||' 'wall full1080|build/librender_owall.so|' \
      'launch full1080||S3R_LPT_MIN=100000000' 2>&1 | tee -a $OUT/ab.txt || exit 1
  bash tools/lib_ab.sh 'work 4K||' 'wall 4K|build/librender_owall.so|' 'launch 4K||S3R_LPT_MIN=100000000' 2>&1 | tee -a $OUT/ab.txt ;;
georows)
  S3R_LIB=build/librender_geo256.so gpu_suite $OUT/parity256.log tests/test_gpu_parity.py tests/test_multi_device.py tests/test_host_loop.py || exit 1
  for rep in 1 2; do
    bash tools/lib_ab.sh 'g128||' 'g256|build/librender_geo256.so|' 'g320|build/librender_geo320.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  PARTS8=1 bash tools/lib_ab.sh 'g128 P_id||' 'g256 P_id|build/librender_geo256.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'g128 1080p||' 'g256 1080p|build/librender_geo256.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  BENCH_EXTRA='--width 7680 --height 4320' bash tools/lib_ab.sh 'g128 8K||' 'g256 8K|build/librender_geo256.so|' 2>&1 | tee -a $OUT/ab.txt ;;
rasterpf)
  S3R_LIB=build/librender_tbotho5.so gpu_suite $OUT/tiles.log tests/test_tiles.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1" bash tools/stress_lib_ab.sh 'base||' 'tpf2|build/librender_tpf2.so|' 'tzv4|build/librender_tzv4.so|' \
      'tpf2o5|build/librender_tpf2o5.so|' 'tbotho5|build/librender_tbotho5.so|' 'to6|build/librender_to6.so|' \
      'tbotho6|build/librender_tbotho6.so|' 'base2||' 2>&1 | tee $OUT/ab.txt ;;
rasterocc)
  S3R_LIB=build/librender_to6l128.so gpu_suite $OUT/tiles.log tests/test_tiles.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1" bash tools/stress_lib_ab.sh 'base||' 'to6|build/librender_to6.so|' 'to7|build/librender_to7.so|' \
      'base2||' 'to6b|build/librender_to6.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  for rep in 1 2; do
    BENCH_EXTRA="--scene icosa-stress --pose P_id --data $D" bash tools/lib_ab.sh 'base stress||' 'to6 stress|build/librender_to6.so|' \
        'to6l128 stress|build/librender_to6l128.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done ;;
setupocc)
  S3R_LIB=build/librender_so8.so gpu_suite $OUT/tiles.log tests/test_tiles.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'base||' 'so7|build/librender_so7.so|' 'so8|build/librender_so8.so|' \
      'base2||' 'so7b|build/librender_so7.so|' 'so8b|build/librender_so8.so|' 2>&1 | tee $OUT/ab.txt ;;
setupgrid)
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1" bash tools/stress_lib_ab.sh 'g1024||' 'g256||S3R_TILE_GRID=256' 'g24||S3R_TILE_GRID=24' \
      'g16||S3R_TILE_GRID=16' 'g1024b||' 'g256b||S3R_TILE_GRID=256' 2>&1 | tee $OUT/ab.txt ;;
fragocc)
  S3R_LIB=build/librender_occ6.so gpu_suite $OUT/parity.log tests/test_gpu_parity.py tests/test_multi_device.py || exit 1
  for tag in base occ6; do
    lib=; [ $tag = occ6 ] && lib=build/librender_occ6.so
    env ${lib:+S3R_LIB=$lib} timeout -k 10 600 python3 -u tools/parts_all.py --configs 3,4 --out $OUT/parts_$tag.jsonl > $OUT/parts_$tag.log 2>&1 || exit 1
  done
  BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'base 1080p||' 'occ6 1080p|build/librender_occ6.so|' \
      'base2 1080p||' 'occ6b 1080p|build/librender_occ6.so|' 2>&1 | tee $OUT/ab.txt ;;
stage192)
  S3R_LIB=build/librender_tl192.so gpu_suite $OUT/tiles.log tests/test_tiles.py || exit 1
  stress_data || exit 1
  for rep in 1 2; do
    BENCH_EXTRA="--scene icosa-stress --pose P_id --data $D" bash tools/lib_ab.sh 'base stress||' 'tl192 stress|build/librender_tl192.so|' \
        2>&1 | tee -a $OUT/ab.txt || exit 1
  done ;;
rec48)
  S3R_LIB=build/librender_rec48.so gpu_suite $OUT/tiles.log tests/test_tiles.py tests/test_multi_device.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'rec64||' 'rec48|build/librender_rec48.so|' 'rec64b||' \
      'rec48b|build/librender_rec48.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  BENCH_EXTRA="--scene icosa-stress --pose P_id --data $D" bash tools/lib_ab.sh 'rec64 stress||' 'rec48 stress|build/librender_rec48.so|' \
      'rec64b stress||' 'rec48b stress|build/librender_rec48.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  for spec in 'rec64|' 'rec48|build/librender_rec48.so'; do
    IFS='|' read -r tag lib <<< "$spec"
    for c in FETCH_SIZE WRITE_SIZE; do
      env S3R_SERIAL=1 ${lib:+S3R_LIB=$lib} timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d "$PWD/$OUT/pmc_${tag}_$c" -o run -- \
          python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data $D --steps 10 > $OUT/pmc_${tag}_$c.log 2>&1 || { tail -5 $OUT/pmc_${tag}_$c.log; exit 1; }
    done
    python3 tools/pmc_summary.py $OUT --last 10 >> gpurun_out/tools_output.log 2>&1 || true
    find $OUT -name '*kernel_trace.csv' -delete
  done
  for spec in rec64 rec48; do
    python3 tools/pmc_summary.py $OUT/pmc_${spec}_FETCH_SIZE --last 10 > $OUT/pmcf_$spec.txt 2>&1 || true
    python3 tools/pmc_summary.py $OUT/pmc_${spec}_WRITE_SIZE --last 10 > $OUT/pmcw_$spec.txt 2>&1 || true
  done
  find $OUT -name '*.csv' -size +5M -delete ;;
rec48s6)
  S3R_LIB=build/librender_rec48s6.so gpu_suite $OUT/tiles.log tests/test_tiles.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'rec64||' 'rec48|build/librender_rec48.so|' 'rec48s6|build/librender_rec48s6.so|' \
      'rec64b||' 'rec48s6b|build/librender_rec48s6.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  BENCH_EXTRA="--scene icosa-stress --pose P_id --data $D" bash tools/lib_ab.sh 'rec64 stress||' 'rec48s6 stress|build/librender_rec48s6.so|' \
      2>&1 | tee -a $OUT/ab.txt ;;
rec48b)
  S3R_LIB=build/librender_rec48.so gpu_suite $OUT/tiles.log tests/test_tiles.py tests/test_multi_device.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'rec64||' 'rec48|build/librender_rec48.so|' 'rec64b||' \
      'rec48b|build/librender_rec48.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  for rep in 1 2; do
    BENCH_EXTRA="--scene icosa-stress --pose P_id --data $D" bash tools/lib_ab.sh 'rec64 stress||' 'rec48 stress|build/librender_rec48.so|' \
        2>&1 | tee -a $OUT/ab.txt || exit 1
  done ;;
clshallow)
  gpu_suite $OUT/tiles.log tests/test_tiles.py tests/test_multi_device.py || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="8" bash tools/stress_lib_ab.sh 'shallow||' 'deep|build/librender_prev.so|' 'shallow2||' \
      'deep2|build/librender_prev.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  for n in 2 4; do
    NS="$n" bash tools/stress_lib_ab.sh 'shallow||' 'deep|build/librender_prev.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done ;;
linfast)
  S3R_LIB=build/librender_linf.so gpu_suite $OUT/parity.log tests/test_gpu_parity.py tests/test_multi_device.py tests/test_host_loop.py \
      tests/test_multi.py tests/test_stream_order.py || exit 1
  for rep in 1 2; do
    PARTS8=1 bash tools/lib_ab.sh 'base||' 'linf|build/librender_linf.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  BENCH_EXTRA='--pose P_id' bash tools/lib_ab.sh 'base P_id||' 'linf P_id|build/librender_linf.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  BENCH_EXTRA='--width 7680 --height 4320' bash tools/lib_ab.sh 'base 8K||' 'linf 8K|build/librender_linf.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'base 1080p||' 'linf 1080p|build/librender_linf.so|' 2>&1 | tee -a $OUT/ab.txt ;;
slotcull)
  gpu_suite $OUT/parity.log tests/test_gpu_parity.py tests/test_host_loop.py tests/test_multi_device.py tests/test_multi.py \
      tests/test_abi.py tests/test_stream_order.py || exit 1
  for rep in 1 2; do
    PARTS8=1 bash tools/lib_ab.sh 'cull||' 'nocull||S3R_SLOT_CULL=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  BENCH_EXTRA='--pose P_id' bash tools/lib_ab.sh 'cull P_id||' 'nocull P_id||S3R_SLOT_CULL=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
  BENCH_EXTRA='--width 7680 --height 4320' bash tools/lib_ab.sh 'cull 8K||' 'nocull 8K||S3R_SLOT_CULL=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
  BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'cull 1080p||' 'nocull 1080p||S3R_SLOT_CULL=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
  timeout -k 10 180 python3 tools/geo_timeline.py --delivered > $OUT/geo_delivered.txt 2>&1 || exit 1
  S3R_SLOT_CULL=0 timeout -k 10 180 python3 tools/geo_timeline.py --delivered > $OUT/geo_delivered_nocull.txt 2>&1 ;;
slotcull2)
  for rep in 1 2 3; do
    bash tools/lib_ab.sh 'cull||' 'nocull||S3R_SLOT_CULL=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
    BENCH_EXTRA='--pose P_id' bash tools/lib_ab.sh 'cull P_id||' 'nocull P_id||S3R_SLOT_CULL=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
    BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'cull 1080p||' 'nocull 1080p||S3R_SLOT_CULL=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  for rep in 1 2; do
    for spec in "cull|" "nocull|S3R_SLOT_CULL=0"; do
      IFS='|' read -r tag envs <<< "$spec"
      probe $tag $envs -- --steps 2000 | tee -a $OUT/probe.txt || exit 1
    done
  done ;;
slotcull3)
  for rep in 1 2 3 4; do
    BENCH_EXTRA='--scene flat --width 1920 --height 1080' bash tools/lib_ab.sh 'nocull 1080p||S3R_SLOT_CULL=0' 'cull 1080p||' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  for rep in 1 2; do
    BENCH_EXTRA='--scene full --width 1920 --height 1080' bash tools/lib_ab.sh 'nocull full1080||S3R_SLOT_CULL=0' 'cull full1080||' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done ;;
norec)
  gpu_suite $OUT/gputest.log tests || exit 1
  stress_data || exit 1
  NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'norec||' 'prev|build/librender_prev.so|' 2>&1 | tee $OUT/ab.txt || exit 1
  for rep in 1 2; do
    BENCH_EXTRA="--scene icosa-stress --pose P_id --data $D" bash tools/lib_ab.sh 'norec stress||' 'prev stress|build/librender_prev.so|' \
        'rec stress||S3R_TILE_NOREC=0' 2>&1 | tee -a $OUT/ab.txt || exit 1
  done
  bash tools/lib_ab.sh 'norec 4K||' 'prev 4K|build/librender_prev.so|' 2>&1 | tee -a $OUT/ab.txt || exit 1
  for spec in 'norec|' 'prev|build/librender_prev.so'; do
    IFS='|' read -r tag lib <<< "$spec"
    env ${lib:+S3R_LIB=$lib} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/del_$tag -o run -- \
        python3 bench.py --scene icosa-stress --pose P_id --data $D --steps 60 --warmup 10 --no-cpu-baseline --no-device > $OUT/del_$tag.log 2>&1 || exit 1
    f=$(find $OUT/del_$tag -name '*kernel_stats.csv' | head -1)
    echo "== $tag delivered (rocprof)"; python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:6]: print('  %-60s %8s calls  avg %9.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))" | tee -a $OUT/ab.txt
    find $OUT/del_$tag -name '*kernel_trace.csv' -delete
  done ;;
cullparts)
  gpu_suite $OUT/parity.log tests/test_gpu_parity.py tests/test_host_loop.py tests/test_multi_device.py tests/test_multi.py || exit 1
  for rep in 1 2 3; do
    for spec in "cull|" "nocull|S3R_SLOT_CULL=0"; do
      IFS='|' read -r tag envs <<< "$spec"
      probe "$tag N8" $envs -- --nparts 8 --steps 3000 | tee -a $OUT/probe.txt || exit 1
      probe "$tag N1" $envs -- --steps 2000 | tee -a $OUT/probe.txt || exit 1
    done
  done ;;
*)
  echo "unknown recipe $R"; exit 2 ;;
esac
