#!/bin/bash
# rocprofv3 kernel stats of the stress scene (tile path) at 3840x2160, part 0 of N (N = 1 and 8),
# into $1/n<N>/ (run on the GPU box; the scene is cached in /tmp/s3r_stress.bin).  S3R_SERIAL=1 (default
# here): frames do not overlap, so each kernel is timed alone.
set -o pipefail
OUT=${1:-gpurun_out/stress_trace}
export TMPDIR=/tmp
mkdir -p "$OUT"
for n in 1 8; do
  S3R_SERIAL=${S3R_SERIAL:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/n$n" -o run --output-format csv -- \
    python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts $n --steps 20 \
    > "$OUT/n$n.log" 2>&1 || exit 1
  python3 - "$OUT/n$n" <<'PY'
import csv, glob, sys
for r in csv.DictReader(open(glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0])):
    print('  ', sys.argv[1].split('/')[-1], r['Name'].split('(')[0][:44], round(float(r['AverageNs']) / 1e3, 1), 'us x', r['Calls'])
PY
done
