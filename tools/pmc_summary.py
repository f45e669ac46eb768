#!/usr/bin/env python3
"""Average each PMC counter per dispatch of each kernel over the pass directories of tools/pmc.sh."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, 'p*', '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get('Kernel_Name', '')
                short = name.split('(')[0].replace('void ', '')
                acc[short][row['Counter_Name']].append(float(row['Counter_Value']))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]['_dispatches'] = max(len(v) for v in cs.values())
    json.dump(out, open(os.path.join(d, 'summary.json'), 'w'), indent=1)
    for k, cs in out.items():
        print(k)
        for c in sorted(cs):
            print(f'   {c:28s} {cs[c]:.4g}')


if __name__ == '__main__':
    main(sys.argv[1])
