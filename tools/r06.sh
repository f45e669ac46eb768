#!/bin/bash
# Round-6 experiments on the GPU box, one recipe per call:  bash tools/r06.sh <recipe> [<recipe> ...]
# Every step writes its stdout AND stderr to its own file under gpurun_out/r06/ (nothing discarded,
# nothing held back in a pipe, so a stalled step leaves what it printed), runs under its own time limit,
# and a failing step ends the call (no retries).  Variant libraries come from tools/variants.py build.
OUT=${OUT_R06:-gpurun_out/r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
STRESS=/tmp/s3r_stress.bin

step() {   # step <name> <seconds> <command...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T)): $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -n 4 "$OUT/$name.log"
  return $rc
}

bench_line() {   # bench_line <name> <env...> -- the bench workload, one JSON line kept in <name>.json
  local name=$1; shift
  step "$name" 150 env "$@" python3 -u bench.py --steps 400 --warmup 40 --no-cpu-baseline || return 1
  grep '^{' "$OUT/$name.log" | tail -1 > "$OUT/$name.json"
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('  $name', round(d['value']), 'fps  device', round(d['device_fps']), 'frag_ms', d['fragment_kernel_ms'])"
}

part8() {   # part8 <name> <env...> -- part 0 of an 8-way band split of the bench frame, pipelined
  local name=$1; shift
  step "$name" 150 env "$@" python3 -u tools/overhead_probe.py --nparts 8 --steps 2000 || return 1
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/$name.log') if l.startswith('{')][-1]
print('  $name part 0/8', round(1e6/d['wall_us']), 'fps  frag_us', round(d['frag_us'], 2))"
}

kstats() {   # kstats <name> <env...> -- rocprofv3 kernel averages of the bench workload
  local name=$1; shift
  step "$name" 200 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
      python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline || return 1
  local f
  f=$(find "$OUT/$name" -name '*kernel_stats.csv' | sort | tail -1)
  python3 - "$f" <<'EOF'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:6]:
    print('  %-58s %7s calls  avg %8.2f us' % (r['Name'][:58], r['Calls'], float(r['AverageNs']) / 1e3))
EOF
}

lds_pmc() {   # lds_pmc <name> <env...> -- LDS counters of the bench workload's kernels
  local name=$1; shift
  step "$name" 120 env "$@" rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
      SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/$name" -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-device || return 1
  python3 tools/pmc_summary.py "$OUT/$name" --last 10 > "$OUT/$name.summary.txt" 2>&1 || return 1
  python3 - "$OUT/$name/pmc_summary.json" <<'EOF2'
import json, sys
for k, c in json.load(open(sys.argv[1])).items():
    if 'k_fragment' in k or 'k_geometry' in k:
        print('  %-44s conflict/active %.3f  lds-wait/wave-cycles %.3f  stall %.3f  VALU %.3g SALU %.3g LDS %.3g' % (
            k[-44:], c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1), c['SQ_WAIT_INST_LDS'] / max(c['SQ_WAVE_CYCLES'], 1),
            c['SQ_WAIT_INST_ANY'] / max(c['SQ_WAVE_CYCLES'], 1), c['SQ_INSTS_VALU'], c['SQ_INSTS_SALU'], c['SQ_INSTS_LDS']))
EOF2
}

for recipe in "$@"; do
  case $recipe in
    tabpad)   # padded table rows (product) vs the round-5 layout (S3R_TAB_PAD=0 build)
      for i in 1 2; do
        bench_line tabpad_bench_pad$i || exit 1
        bench_line tabpad_bench_pad0_$i S3R_LIB=build/librender_pad0.so || exit 1
      done
      part8 tabpad_part8_pad || exit 1
      part8 tabpad_part8_pad0 S3R_LIB=build/librender_pad0.so || exit 1
      kstats tabpad_k_pad || exit 1
      kstats tabpad_k_pad0 S3R_LIB=build/librender_pad0.so || exit 1
      lds_pmc tabpad_pmc_pad || exit 1
      lds_pmc tabpad_pmc_pad0 S3R_LIB=build/librender_pad0.so || exit 1
      ;;
    ab)   # product vs the variant library $AB (build/librender_$AB.so): bench x2, part 0 of 8, rocprof, counters
      V=build/librender_$AB.so
      for i in 1 2; do
        bench_line ${AB}_bench_prod$i || exit 1
        bench_line ${AB}_bench_var$i S3R_LIB=$V || exit 1
      done
      part8 ${AB}_part8_prod || exit 1
      part8 ${AB}_part8_var S3R_LIB=$V || exit 1
      kstats ${AB}_k_prod || exit 1
      kstats ${AB}_k_var S3R_LIB=$V || exit 1
      lds_pmc ${AB}_pmc_prod || exit 1
      lds_pmc ${AB}_pmc_var S3R_LIB=$V || exit 1
      ;;
    k8)   # part 0 of 8 of the 8K frame (config 4's split) and of the 4K frame under fragment-launch thresholds
      for sz in "7680 4320" "3840 2160"; do
        set -- $sz
        for envs in "S3R_NOTHING=0" "S3R_WATERFALL_BINS=2000" "S3R_LPT_MIN=100000000" "S3R_WATERFALL_BINS=2000 S3R_LPT_MIN=100000000"; do
          tag=k8_${1}_$(echo $envs | tr ' =' '__')
          step $tag 120 env $envs python3 -u tools/overhead_probe.py --width $1 --height $2 --nparts 8 --steps 2000 || exit 1
          python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/$tag.log') if l.startswith('{')][-1]
print('  $1 $envs: part 0/8', round(1e6/d['wall_us']), 'fps  frag_us', round(d['frag_us'], 2), 'host_us', round(d['host_enqueue_us'], 2))"
        done
      done
      ;;
    spab|stressab)  # config 5 whole frame: product vs the variant build/librender_$AB.so (spab: AB=sp0)
      [ $recipe = spab ] && AB=sp0
      [ -f $STRESS ] || step stress_data 300 python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$STRESS')" || exit 1
      for v in prod $AB; do
        L=""; [ $v = $AB ] && L=build/librender_$AB.so
        step spab_bench_$v 300 env ${L:+S3R_LIB=$L} python3 -u bench.py --scene icosa-stress --pose P_id --data $STRESS --no-cpu-baseline || exit 1
        grep '^{' "$OUT/spab_bench_$v.log" | tail -1 > "$OUT/spab_bench_$v.json"
        python3 -c "import json; d=json.load(open('$OUT/spab_bench_$v.json')); print('  $v stress', round(d['value']), 'fps  device', round(d['device_fps']), 'setup_ms', d['setup_ms'], 'frag_ms', d['fragment_kernel_ms'])"
        step spab_k_$v 300 env ${L:+S3R_LIB=$L} S3R_SERIAL=1 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/spab_k_$v" -o run -- \
            python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data $STRESS --steps 20 || exit 1
        f=$(find "$OUT/spab_k_$v" -name '*kernel_stats.csv' | sort | tail -1)
        python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:6]: print('  $v %-50s %6s calls avg %9.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))"
        for c in FETCH_SIZE WRITE_SIZE; do
          step spab_pmc_${v}_$c 200 env ${L:+S3R_LIB=$L} rocprofv3 --pmc $c --output-format csv -d "$OUT/spab_pmc_$v/$c" -o run -- \
              python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data $STRESS --steps 10 || exit 1
        done
        python3 tools/pmc_summary.py "$OUT/spab_pmc_$v" --last 10 > "$OUT/spab_pmc_$v.txt" 2>&1 || exit 1
        python3 -c "
import json
for k, c in json.load(open('$OUT/spab_pmc_$v/pmc_summary.json')).items():
    if 'k_tile' in k: print('  $v %-44s FETCH %.1f MB  WRITE %.1f MB' % (k[-44:], c.get('FETCH_SIZE', 0) / 1024, c.get('WRITE_SIZE', 0) / 1024))"
      done
      ;;
    eighth)   # per-stage breakdown of part 0 of 8 at 4K and 8K (pipelined frames, kernel trace + host enqueue)
      for sz in "3840 2160" "7680 4320"; do
        set -- $sz
        tag=eighth_$1
        step ${tag}_probe 120 python3 -u tools/overhead_probe.py --width $1 --height $2 --nparts 8 --steps 2000 || exit 1
        H=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/${tag}_probe.log') if l.startswith('{')][-1]
print(round(d['host_enqueue_us'], 2))")
        step ${tag}_trace 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${tag}_trace" -o run -- \
            python3 tools/overhead_probe.py --width $1 --height $2 --nparts 8 --steps 2000 || exit 1
        f=$(find "$OUT/${tag}_trace" -name '*kernel_trace.csv' | sort | tail -1)
        python3 tools/eighth_breakdown.py "$f" --frames 1000 --host-us $H --label "part 0 of 8, $1x$2" | tee "$OUT/${tag}_breakdown.json"
      done
      ;;
    seg8k)   # part 0 of 8 of the 8K and 4K frames under fragment segment widths (S3R_MIN_BLOCKS / S3R_SEG3)
      for cfg in "7680 4320 S3R_NOTHING=0" "7680 4320 S3R_SEG3=1 S3R_MIN_BLOCKS=3000" "7680 4320 S3R_MIN_BLOCKS=6000" \
                 "7680 4320 S3R_MIN_BLOCKS=10000" "3840 2160 S3R_NOTHING=0" "3840 2160 S3R_SEG3=1 S3R_MIN_BLOCKS=1300"; do
        set -- $cfg
        w=$1; h=$2; shift 2
        tag=seg_${w}_$(echo "$*" | tr ' =' '__')
        step $tag 120 env "$@" python3 -u tools/overhead_probe.py --width $w --height $h --nparts 8 --steps 2000 || exit 1
        python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/$tag.log') if l.startswith('{')][-1]
print('  $w $*: part 0/8', round(1e6/d['wall_us']), 'fps  frag_us', round(d['frag_us'], 2), 'host_us', round(d['host_enqueue_us'], 2))"
      done
      ;;
    timeline)   # per-workgroup k_fragment timelines (timing build build/librender_wgt.so): 8K and 4K eighths, 4K whole
      step tl_8k_n8 240 python3 -u tools/wg_timeline.py --width 7680 --height 4320 --nparts 8 || exit 1
      step tl_4k_n8 240 python3 -u tools/wg_timeline.py --nparts 8 || exit 1
      step tl_8k_n1 240 python3 -u tools/wg_timeline.py --width 7680 --height 4320 || exit 1
      grep -h "launch span\|total\|in flight" "$OUT"/tl_*.log
      ;;
    nobin)   # config 5 whole frame, serialised kernel times: product vs the no-binning ablation (wrong pixels)
      [ -f $STRESS ] || step stress_data 300 python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$STRESS')" || exit 1
      for v in prod nobin; do
        L=""; [ $v = nobin ] && L=build/librender_nobin.so
        step nobin_k_$v 300 env ${L:+S3R_LIB=$L} S3R_SERIAL=1 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nobin_k_$v" -o run -- \
            python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data $STRESS --steps 20 || exit 1
        f=$(find "$OUT/nobin_k_$v" -name '*kernel_stats.csv' | sort | tail -1)
        python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:4]: print('  $v %-50s %6s calls avg %9.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))"
      done
      ;;
    bands)   # every part of the 8-way split of configs 4 and 3 at several band heights
      for b in 8 16 32 64; do
        step bands_$b 300 python3 -u tools/parts_all.py --configs 4,3 --nparts 1,8 --band $b --out "$OUT/bands_$b.jsonl" || exit 1
        python3 -c "
import json
for l in open('$OUT/bands_$b.jsonl'):
    d=json.loads(l); print('  band $b config', d['config'], 'N', d['N'], 'slowest', d['slowest_us'], 'max/mean', d['max_over_mean'], 'eff', d['efficiency_per_gpu'])"
      done
      ;;
    geovar)   # configs 4 and 3, whole frame and every eighth, for geometry variants (VARIANTS="tag tag ...")
      for rep in 1 2; do
        for v in prod ${VARIANTS:-geoprio0 georows256 georows64}; do
          L=""; [ $v != prod ] && L=build/librender_$v.so
          step geovar_${v}_$rep 300 env ${L:+S3R_LIB=$L} python3 -u tools/parts_all.py --configs 4,3 --nparts 1,8 --out "$OUT/geovar_${v}_$rep.jsonl" || exit 1
          python3 -c "
import json
for l in open('$OUT/geovar_${v}_$rep.jsonl'):
    d=json.loads(l); print('  $v rep $rep config', d['config'], 'N', d['N'], 'slowest', d['slowest_us'], 'eff', d['efficiency_per_gpu'])"
        done
      done
      ;;
    split)   # the split k_fragment instance (S3R_SPLIT_BINS): parity forced on every HBM launch, then part 0 of 8
      step split_parity 600 env S3R_SPLIT_BINS=100000000 python3 -u -m pytest -s -x -v --timeout 120 --timeout-method thread -m gpu \
          tests/test_gpu_parity.py tests/test_multi_device.py tests/test_multi.py tests/test_stream_order.py || exit 1
      for sz in "7680 4320" "3840 2160"; do
        set -- $sz
        for sb in 0 3000; do
          tag=split_${1}_$sb
          step $tag 120 env S3R_SPLIT_BINS=$sb python3 -u tools/overhead_probe.py --width $1 --height $2 --nparts 8 --steps 2000 || exit 1
          python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/$tag.log') if l.startswith('{')][-1]
print('  $1 split_bins $sb: part 0/8', round(1e6/d['wall_us']), 'fps  frag_us', round(d['frag_us'], 2), 'host_us', round(d['host_enqueue_us'], 2))"
        done
      done
      for sb in 0 3000 0 3000; do
        step split_parts_$sb 300 env S3R_SPLIT_BINS=$sb python3 -u tools/parts_all.py --configs 4,3 --nparts 1,8 --out "$OUT/split_parts_$sb.jsonl" || exit 1
        python3 -c "
import json
for l in open('$OUT/split_parts_$sb.jsonl'):
    d=json.loads(l); print('  split_bins $sb config', d['config'], 'N', d['N'], 'slowest', d['slowest_us'], 'eff', d['efficiency_per_gpu'])"
      done
      ;;
    stresspart)   # config 5: part 0 of 8 at the library's band, product vs build/librender_$AB.so
      [ -f $STRESS ] || step stress_data 300 python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$STRESS')" || exit 1
      for v in prod $AB prod $AB; do
        L=""; [ $v = $AB ] && L=build/librender_$AB.so
        step stresspart_$v 300 env ${L:+S3R_LIB=$L} python3 -u tools/overhead_probe.py --scene icosa-stress --pose P_id --data $STRESS --nparts 8 --band 135 --steps 100 || exit 1
        python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/stresspart_$v.log') if l.startswith('{')][-1]
print('  $v stress part 0/8', round(1e6/d['wall_us']), 'fps  frag_us', round(d['frag_us'], 1))"
      done
      ;;
    rowparity)   # the row path's parity suite
      step rowparity 600 python3 -u -m pytest -s -x -v --timeout 120 --timeout-method thread -m gpu \
          tests/test_gpu_parity.py tests/test_multi_device.py || exit 1
      ;;
    stall)   # the bounded-wait tests (each a child process that must end with status 86)
      step stall 300 python3 -u -m pytest -s -x -v --timeout 120 --timeout-method thread -m gpu tests/test_stall.py || exit 1
      ;;
    tiles)   # the tile path's parity suite
      step tiles 900 python3 -u -m pytest -s -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tiles.py || exit 1
      ;;
    stress)  # config 5 (1 M icosahedra, 4K, tile path): the bench line, part 0 of 8 at the library's band
      [ -f $STRESS ] || step stress_data 300 python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$STRESS')" || exit 1
      step stress_bench 300 python3 -u bench.py --scene icosa-stress --pose P_id --data $STRESS --no-cpu-baseline || exit 1
      grep '^{' "$OUT/stress_bench.log" | tail -1 > "$OUT/stress_bench.json"
      python3 -c "import json; d=json.load(open('$OUT/stress_bench.json')); print('  stress', round(d['value']), 'fps  device', round(d['device_fps']), 'setup_ms', d['setup_ms'], 'frag_ms', d['fragment_kernel_ms'])"
      step stress_part8 300 python3 -u tools/overhead_probe.py --scene icosa-stress --pose P_id --data $STRESS --nparts 8 --band 135 --steps 100 || exit 1
      python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/stress_part8.log') if l.startswith('{')][-1]
print('  stress part 0/8', round(1e6/d['wall_us']), 'fps  frag_us', round(d['frag_us'], 1))"
      ;;
    parts)   # every part of the N = 1, 2, 4, 8 band splits of configs 3, 4 (and 5 with PARTS_CONFIGS)
      step parts 900 python3 -u tools/parts_all.py --configs ${PARTS_CONFIGS:-3,4} --out "$OUT/parts_all.jsonl" || exit 1
      python3 -c "
import json
for l in open('$OUT/parts_all.jsonl'):
    d=json.loads(l); print('  config', d['config'], 'N', d['N'], 'band', d['band'], 'slowest', d['slowest_us'], 'max/mean', d['max_over_mean'], 'eff', d['efficiency_per_gpu'])"
      ;;
    suite)   # the whole GPU suite, once
      step suite 1100 python3 -u -m pytest -s -x -v --timeout 200 --timeout-method thread -m gpu tests || exit 1
      ;;
    *) echo "unknown recipe $recipe"; exit 2 ;;
  esac
done
