#!/bin/bash
# Depth buckets per tile (S3R_DEPTH_BUCKETS 32 / 128 / 256; db128c256: 128 with a first bin capacity of 256): tile parity with each variant, the stress
# frame's kernels serialised, part 0 of 8 at the library's band, the delivered stress bench line.
OUT=gpurun_out/buckets; mkdir -p $OUT; export TMPDIR=/tmp; D=/tmp/s3r_stress.bin
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "   rc=$rc"; tail -n 2 "$OUT/$name.log"; return $rc; }
for v in db128 db256; do
  step tiles_$v 300 env S3R_LIB=build/librender_$v.so python3 -u -m pytest tests/test_tiles.py -m gpu -x -q -s --timeout 200 --timeout-method thread || exit 1
done
step data 300 python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
cat > /tmp/bv.json <<'J'
{"prod32": {}, "db64": {}, "db128": {}}
J
for v in prod32 db128 db256 db128c256 prod32 db128 db256 db128c256; do
  L=""; E=""; [ $v != prod32 ] && L=build/librender_${v%c256}.so; [ $v = db128c256 ] && E=S3R_TILE_BIN_CAP=256
  step part8_$v 200 env ${L:+S3R_LIB=$L} $E python3 -u tools/overhead_probe.py --scene icosa-stress --pose P_id --data $D --nparts 8 --band 135 --steps 100 || exit 1
  step bench_$v 300 env ${L:+S3R_LIB=$L} $E python3 -u bench.py --scene icosa-stress --pose P_id --data $D --no-cpu-baseline || exit 1
  step k_$v 300 env ${L:+S3R_LIB=$L} $E S3R_SERIAL=1 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k_$v -o run -- python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data $D --steps 20 || exit 1
done
python3 - <<'PY'
import json, glob, csv, os
OUT='gpurun_out/buckets'
for v in ['prod32','db128','db256','db128c256']:
    for f in sorted(glob.glob(f'{OUT}/bench_{v}.log')):
        d=[json.loads(l) for l in open(f) if l.startswith('{')][-1]
        print(v, 'delivered', round(d['value'],1), 'device', round(d['device_fps'],1), 'setup_ms', d['setup_ms'])
    d=[json.loads(l) for l in open(f'{OUT}/part8_{v}.log') if l.startswith('{')][-1]
    print(v, 'part0/8 wall_us', round(d['wall_us'],1), 'frag_us', round(d['frag_us'],1))
    st=glob.glob(f'{OUT}/k_{v}/**/run_kernel_stats.csv', recursive=True)
    for r in csv.DictReader(open(st[0])):
        if 'k_tile' in r['Name']: print('   ', r['Name'].split('(')[0][-40:], round(float(r['AverageNs'])/1e3,1))
PY
