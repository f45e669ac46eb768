#!/usr/bin/env python3
"""Per-kernel PMC averages over the last N dispatches (the bench's timed frames) of every pass
directory under <dir>, and the HBM traffic of k_fragment per launch.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE (KiB, from the TCC EA request
counters) each in their own pass; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
reads, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (the read side is an upper bound for
narrower accesses); WRITE_SIZE is exact for streaming stores.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--last', type=int, default=0)
    ap.add_argument('--workload', default=None)
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(a.dir, '**', '*counter_collection.csv'), recursive=True)):
        rows = defaultdict(lambda: defaultdict(float))
        with open(f) as fh:
            for row in csv.DictReader(fh):
                short = row.get('Kernel_Name', '').split('(')[0].replace('void ', '')
                rows[short][(int(row['Dispatch_Id']), row['Counter_Name'])] += float(row['Counter_Value'])
        for k, d in rows.items():
            ids = sorted({i for i, _ in d})
            if a.last:
                ids = ids[-a.last:]
            for (i, c), val in d.items():
                if i in ids:
                    acc[k][c].append(val)
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]['_dispatches'] = max(len(v) for v in cs.values())
    with open(os.path.join(a.dir, 'pmc_summary.json'), 'w') as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, cs in out.items():
        print(k)
        for c in sorted(cs):
            print(f'   {c:28s} {cs[c]:.6g}')
    # the fragment stage: k_fragment (row path; its HBM instance, HOSTW = false -- the delivered
    # instance's stores go to the host) or k_tile_raster + k_tile_resolve (tile path)
    frag = [k for k in out if 'k_fragment' in k]
    stage = ([k for k in frag if k.replace(' ', '').endswith(',false>')] or frag or
             [k for k in out if 'k_tile_raster' in k or 'k_tile_resolve' in k])
    if stage and a.workload and all('FETCH_SIZE' in out[k] and 'WRITE_SIZE' in out[k] for k in stage):
        fetch = sum(out[k]['FETCH_SIZE'] for k in stage)
        write = sum(out[k]['WRITE_SIZE'] for k in stage)
        t = {a.workload: {'kernel': '+'.join(k.split('::')[-1] for k in stage), 'fetch_size_kib': fetch,
                          'write_size_kib': write, 'hbm_bytes_per_launch': int((2 * fetch + write) * 1024),
                          'formula': '(2*FETCH_SIZE + WRITE_SIZE) * 1024, MI355X_MICROARCH.md HBM section'}}
        with open(os.path.join(a.dir, 'pmc_traffic.json'), 'w') as fh:
            json.dump(t, fh, indent=1)
        print(json.dumps(t))


if __name__ == '__main__':
    main()
