#!/usr/bin/env python3
"""Build tuning / ablation variants here (tools/variants.py build) and time them on the GPU box
(tools/variants.py run): per-kernel average us from rocprofv3 --kernel-trace --stats per variant.
Env: S3R_VARIANT_BENCH = extra bench.py args (default: the stress scene)."""
import csv
import glob
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import json

# S3R_VARIANTS='{"tag": {"MACRO": value, ...}, ...}' overrides the default set
# (or S3R_VARIANTS_FILE=<path of such a JSON file>)
if os.environ.get('S3R_VARIANTS_FILE'):
    os.environ['S3R_VARIANTS'] = open(os.environ['S3R_VARIANTS_FILE']).read()
VARIANTS = json.loads(os.environ['S3R_VARIANTS']) if os.environ.get('S3R_VARIANTS') else {
    'base': {},
    'st64': {'S3R_TSTAGE': 64},
    'st256': {'S3R_TSTAGE': 256},
}


def build():
    from swift3drenderer_amd.build import build_variant
    for tag, d in VARIANTS.items():
        print(build_variant(tag, d))


def run():
    extra = shlex.split(os.environ.get('S3R_VARIANT_BENCH', '--scene icosa-stress --pose P_id'))
    out_root = os.path.join(ROOT, 'gpurun_out', 'variants')
    for tag in VARIANTS:
        env = dict(os.environ, S3R_LIB=os.path.join(ROOT, 'build', f'librender_{tag}.so'), TMPDIR='/tmp',
                   S3R_SERIAL=os.environ.get('S3R_SERIAL', '1'))
        d = os.path.join(out_root, tag)
        cmd = ['rocprofv3', '--kernel-trace', '--stats', '-d', d, '-o', 'run', '--output-format', 'csv', '--',
               sys.executable, 'bench.py', '--steps', '10', '--warmup', '2', '--no-cpu-baseline'] + extra
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
        line = [l for l in r.stdout.splitlines() if l.startswith('{')]
        fps = line[-1].split('"value": ')[1].split(',')[0] if line else '?'
        stats = glob.glob(os.path.join(d, '**', 'run_kernel_stats.csv'), recursive=True)
        parts = []
        if stats:
            for row in csv.DictReader(open(stats[0])):
                if 's3r::' in row['Name']:
                    name = row['Name'].split('s3r::', 1)[1].split('(')[0]
                    parts.append(f"{name} {float(row['AverageNs']) / 1e3:.1f}")
        print(f'{tag:8s} fps {fps:>10s}  ' + '  '.join(parts), flush=True)


if __name__ == '__main__':
    build() if sys.argv[1] == 'build' else run()
