#!/bin/bash
# Config 5 A/B: the product library against build/librender_<tag>.so for each tag in $AB -- tile parity of the product, then
# two alternations of part 0 of 8 (135-row band), the delivered stress bench line and the serialised
# kernel times.  Usage: AB='<tag> [<tag> ...]' bash tools/r06_stress_ab.sh
OUT=gpurun_out/sab_${AB// /_}; mkdir -p $OUT; export TMPDIR=/tmp; D=/tmp/s3r_stress.bin
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "   rc=$rc"; tail -n 2 "$OUT/$name.log"; return $rc; }
step tiles_prod 300 python3 -u -m pytest tests/test_tiles.py -m gpu -x -q -s --timeout 200 --timeout-method thread || exit 1
step data 300 python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
for i in 1 2; do
  for v in prod $AB; do
    L=""; [ $v != prod ] && L=build/librender_$v.so
    step part8_${v}_$i 200 env ${L:+S3R_LIB=$L} python3 -u tools/overhead_probe.py --scene icosa-stress --pose P_id --data $D --nparts 8 --band 135 --steps 100 || exit 1
    step bench_${v}_$i 300 env ${L:+S3R_LIB=$L} python3 -u bench.py --scene icosa-stress --pose P_id --data $D --no-cpu-baseline || exit 1
    step k_${v}_$i 300 env ${L:+S3R_LIB=$L} S3R_SERIAL=1 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k_${v}_$i -o run -- python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data $D --steps 20 || exit 1
  done
done
python3 - "$OUT" $AB <<'PY'
import json, glob, csv, sys
OUT, AB = sys.argv[1], sys.argv[2:]
for i in (1, 2):
    for v in ['prod'] + AB:
        b=[json.loads(l) for l in open(f'{OUT}/bench_{v}_{i}.log') if l.startswith('{')][-1]
        p=[json.loads(l) for l in open(f'{OUT}/part8_{v}_{i}.log') if l.startswith('{')][-1]
        st=glob.glob(f'{OUT}/k_{v}_{i}/**/run_kernel_stats.csv', recursive=True)
        ks={r['Name'].split('(')[0].replace('void ','').replace('s3r::',''): float(r['AverageNs'])/1e3 for r in csv.DictReader(open(st[0]))}
        print(f"{v:6s} {i}: delivered {b['value']:.1f} device {b['device_fps']:.1f} setup_ms {b['setup_ms']}  part0/8 frag {p['frag_us']:.1f} wall {p['wall_us']:.1f}  "
              + '  '.join(f"{k} {t:.1f}" for k, t in ks.items() if 'k_tile_raster' in k or 'k_tile_setup' in k))
PY
