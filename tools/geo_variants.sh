#!/bin/bash
# Serial kernel times of k_geometry variants (GPU box): full, no segment starts, no walks.
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base geo1 geo2; do
  lib=swift3drenderer_amd/librender.so; [ "$v" != base ] && lib=build/librender_$v.so
  for np in 1 8; do
    d=gpurun_out/geov/$v-$np
    S3R_LIB=$lib S3R_SERIAL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/overhead_probe.py --nparts $np --steps 100 >> gpurun_out/tools_output.log 2>&1 || exit 1
    python3 - "$d" "$v" "$np" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
parts = [f"{r['Name'].split('(')[0].replace('void ','')[5:]} {float(r['AverageNs'])/1e3:.1f}" for r in csv.DictReader(open(f)) if 's3r::' in r['Name']]
print(sys.argv[2], 'N', sys.argv[3], ' | '.join(parts))
PY
  done
done
