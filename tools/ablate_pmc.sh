#!/bin/bash
# VALU / SALU instruction counts of k_fragment per ablation variant (GPU box; see tools/ablate.sh).
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" 1 5 13 29 157; do
  lib=swift3drenderer_amd/librender.so; [ -n "$v" ] && lib=build/librender_ablate$v.so
  d=gpurun_out/apmc/v${v:-0}
  S3R_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_BRANCH --output-format csv -d $d -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/tools_output.log 2>&1 || exit 1
  python3 - "$d" "${v:-0}" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if 'k_fragment' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
out = {k: sum(v.values()) / len(v) for k, v in acc.items()}
w = out.get('SQ_WAVES', 1)
print('ablate', sys.argv[2], ' '.join(f"{k[8:] if k.startswith('SQ_INSTS') else k}={v/1e6:.2f}M" for k, v in sorted(out.items())), f"valu/wave={out.get('SQ_INSTS_VALU',0)/w:.0f} salu/wave={out.get('SQ_INSTS_SALU',0)/w:.0f}")
PY
done
