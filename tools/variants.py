#!/usr/bin/env python3
"""Build tuning variants here (tools/variants.py build) and time them on the GPU box
(tools/variants.py run): fragment-kernel ms per variant, interleaved rounds in separate processes."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    'calls': {'S3R_INLINE': 0},
    'inline': {'S3R_INLINE': 1},
    'inline_skel': {'S3R_INLINE': 1, 'S3R_ABLATE': 189},
    'calls_skel': {'S3R_INLINE': 0, 'S3R_ABLATE': 189},
}


def build():
    from swift3drenderer_amd.build import build_variant
    for tag, d in VARIANTS.items():
        print(build_variant(tag, d))


def run(poses=('P_over', 'P_id')):
    res = {}
    for rnd in range(2):
        for tag in VARIANTS:
            for pose in poses:
                env = dict(os.environ, S3R_LIB=os.path.join(ROOT, 'build', f'librender_{tag}.so'))
                out = subprocess.run([sys.executable, 'bench.py', '--pose', pose, '--steps', '100', '--warmup', '10',
                                      '--no-cpu-baseline', '--no-e2e'], env=env, capture_output=True, text=True,
                                     timeout=120, cwd=ROOT)
                d = json.loads(out.stdout.strip().splitlines()[-1])
                res.setdefault((tag, pose), []).append((d['fragment_kernel_ms'], d['value']))
    for (tag, pose), v in sorted(res.items()):
        print(f'{tag:14s} {pose:8s} frag_ms {min(a for a, _ in v):.4f}  fps {max(b for _, b in v):9.1f}  rounds {v}')


if __name__ == '__main__':
    build() if sys.argv[1] == 'build' else run()
