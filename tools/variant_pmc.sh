#!/bin/bash
# SQ counters of k_fragment for several variant builds (build/librender_<tag>.so, tools/variants.py
# build), two rocprofv3 --pmc passes each, then one table.  On the GPU box:
#   bash tools/variant_pmc.sh <outdir> tag1 tag2 ...      (env BENCH_ARGS: extra bench.py args)
set -o pipefail
OUT=${1:-gpurun_out/vpmc}; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
ROOTDIR=$(pwd)
ARGS="--steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS"
for tag in "$@"; do
  lib=build/librender_$tag.so; [ "$tag" = prod ] && lib=swift3drenderer_amd/librender.so
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"; do
    i=$((i+1))
    S3R_SERIAL=1 S3R_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$ROOTDIR/$OUT/$tag/p$i" -o run -- python3 bench.py $ARGS > "$OUT/$tag.p$i.log" 2>&1 || { echo "$tag pass $i failed"; tail -3 "$OUT/$tag.p$i.log"; exit 1; }
  done
done
python3 - "$OUT" "$@" <<'EOF'
import csv, glob, os, sys
from collections import defaultdict
out, tags = sys.argv[1], sys.argv[2:]
rows = {}
for tag in tags:
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(out, tag, 'p*', '**', '*counter_collection.csv'), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if 'k_fragment' in r.get('Kernel_Name', ''):
                per[(int(r['Dispatch_Id']), r['Counter_Name'])] += float(r['Counter_Value'])
        ids = sorted({i for i, _ in per})[-10:]
        for (i, c), v in per.items():
            if i in ids:
                acc[c].append(v)
    rows[tag] = {c: sum(v) / len(v) for c, v in acc.items()}
cs = sorted({c for r in rows.values() for c in r})
print('counter'.ljust(26) + ''.join(t.rjust(14) for t in tags))
for c in cs:
    print(c.ljust(26) + ''.join(f'{rows[t].get(c, float("nan")):14.4g}' for t in tags))
EOF
find "$OUT" \( -name '*counter_collection.csv' -o -name '*agent_info.csv' \) -delete
