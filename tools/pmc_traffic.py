#!/usr/bin/env python3
"""HBM bytes per launch of a workload's kernels from a PMC summary (tools/pmc_summary.py output), merged
into a pmc_traffic.json together with the SHA-256 of the library the passes ran -- bench.py reports a
figure only when that hash is the library it renders with (every figure from the
same build).

    python3 tools/pmc_traffic.py <pmc dir> --workload full/P_over/3840x2160/N1 --kernel 'k_fragment<6u, true, false>' \
        [--setup-kernel 'k_tile_setup<false, false>'] --out gpurun_out/r06/pmc_traffic.json --source '...'

Bytes follow MI355X_MICROARCH.md's HBM section: (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (FETCH_SIZE and
WRITE_SIZE from their own passes; gfx950 reports half the bytes of wide coalesced reads).
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(summary, needle):
    keys = [k for k in summary if needle in k]
    if len(keys) != 1:
        sys.exit(f'pmc_traffic: {needle!r} matches {keys}')
    c = summary[keys[0]]
    return keys[0], c['FETCH_SIZE'], c['WRITE_SIZE'], int((2 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--workload', required=True)
    ap.add_argument('--kernel', required=True)
    ap.add_argument('--setup-kernel', default=None)
    ap.add_argument('--out', required=True)
    ap.add_argument('--source', default='')
    ap.add_argument('--lib', default=os.environ.get('S3R_LIB') or os.path.join(ROOT, 'swift3drenderer_amd', 'librender.so'))
    a = ap.parse_args()
    summary = json.load(open(os.path.join(a.dir, 'pmc_summary.json')))
    with open(a.lib, 'rb') as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    k, fetch, write, b = per_launch(summary, a.kernel)
    e = {'kernel': k.split('::')[-1], 'fetch_size_kib': fetch, 'write_size_kib': write, 'hbm_bytes_per_launch': b}
    if a.setup_kernel:
        sk, sf, sw, sb = per_launch(summary, a.setup_kernel)
        e.update({'setup_kernel': sk.split('::')[-1], 'setup_fetch_size_kib': sf, 'setup_write_size_kib': sw,
                  'setup_hbm_bytes_per_launch': sb})
    e.update({'formula': '(2*FETCH_SIZE + WRITE_SIZE) * 1024, MI355X_MICROARCH.md HBM section',
              'source': a.source or a.dir, 'library_sha256': sha})
    out = {}
    if os.path.exists(a.out):
        out = json.load(open(a.out))
    out[a.workload] = e
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps({a.workload: e}, indent=1))


if __name__ == '__main__':
    main()
