#!/usr/bin/env python3
"""Tile-path counters (stats build, GPU box): staged (slot, tile) pairs and how many the
hierarchical depth test culled, for one frame of the stress scene.
    python tools/tile_stats.py [--scene icosa-stress --pose P_id --width 3840 --height 2160]"""
import argparse, ctypes, os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--scene', default='icosa-stress')
    ap.add_argument('--pose', default='P_id')
    ap.add_argument('--width', type=int, default=3840)
    ap.add_argument('--height', type=int, default=2160)
    a = ap.parse_args()
    from swift3drenderer_amd import build, poses, renderer, scene
    lib = renderer.load_library(build.build_library(stats=True))
    lib.s3r_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    d = tempfile.mkdtemp()
    data = os.path.join(d, a.scene + '.bin')
    scene.write_named(a.scene, data)
    r = renderer.Renderer(data)
    r.set_raster_path('tiles')
    for t in poses.script(a.pose):
        r.update_and_render(a.width, a.height, t)
    out = (ctypes.c_uint64 * 16)()
    lib.s3r_stats(out, 1)
    r.update_and_render(a.width, a.height, poses.hold(a.pose))
    lib.s3r_stats(out, 0)
    pairs = r.scene_counts()[5]
    print(f'{a.scene}/{a.pose} {a.width}x{a.height}: (slot, tile) pairs {pairs}, staged with rows {out[0]}, '
          f'culled by depth {out[1]} ({100.0 * out[1] / max(out[0], 1):.1f}%)')
    print(f'resolve: foreground pixels {out[2]}, runs of one winner along a row {out[3]} '
          f'({out[2] / max(out[3], 1):.2f} px per run), wave setup rounds run-shared {out[4]} of {4 * out[5]} '
          f'per-pixel (waves {out[5]}, most runs in one wave {out[6]})')
    print(f'setup: live triangles {out[8]} of {out[9]} set up ({100.0 * out[8] / max(out[9], 1):.1f} %)')
    r.shutdown()


if __name__ == '__main__':
    main()
