#!/usr/bin/env python3
"""Synchronous updateAndRender frames into a main.swift-style double buffer, for tracing where a
frame's wall time goes (run under rocprofv3 --kernel-trace [--hip-trace] on the GPU box).

    python tools/e2e_probe.py [--delivery fill|direct|copy|auto] [--devices 0,0] [--frames 300]
Prints one JSON line: median / p10 / p90 call time and the delivery counters.
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def numa_report(buf):
    """NUMA placement: the node of the caller buffer's pages (move_pages query), the CPU / node the
    calling thread runs on, the GPU's node (sysfs of its PCI device)."""
    out = {}
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        n = 8
        pages = (ctypes.c_void_p * n)(*[buf.ptr + k * (2 * buf.size // n) for k in range(n)])
        status = (ctypes.c_int * n)()
        libc.syscall(279, 0, ctypes.c_ulong(n), pages, None, status, 0)     # SYS_move_pages, query
        out['buffer_nodes'] = sorted(set(status))
        with open('/proc/self/stat') as f:
            cpu = int(f.read().rsplit(')', 1)[1].split()[36])
        out['cpu'] = cpu
        for d in os.listdir('/sys/devices/system/node'):
            if d.startswith('node') and os.path.exists(f'/sys/devices/system/node/{d}/cpu{cpu}'):
                out['cpu_node'] = int(d[4:])
        hip = ctypes.CDLL('libamdhip64.so')
        bus = ctypes.create_string_buffer(64)
        hip.hipDeviceGetPCIBusId(bus, 64, 0)
        bid = bus.value.decode().lower()
        with open(f'/sys/bus/pci/devices/{bid}/numa_node') as f:
            out['gpu_node'] = int(f.read())
        out['gpu_bus'] = bid
        out['nodes'] = open('/sys/devices/system/node/online').read().strip()
    except Exception as e:      # diagnostics only
        out['numa_error'] = repr(e)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--scene', default='full')
    p.add_argument('--pose', default='P_over')
    p.add_argument('--width', type=int, default=3840)
    p.add_argument('--height', type=int, default=2160)
    p.add_argument('--frames', type=int, default=300)
    p.add_argument('--delivery', default='auto')
    p.add_argument('--fill-threads', type=int, default=-1)
    p.add_argument('--devices', default='0')
    p.add_argument('--torch', action='store_true', help='import torch and make device 0 current first (as bench.py)')
    p.add_argument('--warmup', type=int, default=30)
    p.add_argument('--line-offset', type=int, default=None, help='buffer this many bytes past a 64-B line')
    p.add_argument('--data', default=None, help='a data.bin to reuse (written there once when missing)')
    a = p.parse_args()
    if a.torch:
        import torch
        torch.cuda.set_device(0)
        torch.empty(1, device='cuda')
    import numpy as np
    from bench import DoubleBuffer
    from swift3drenderer_amd import poses, scene
    from swift3drenderer_amd.abi import Input
    from swift3drenderer_amd.renderer import Renderer
    path = a.data or os.path.join(tempfile.mkdtemp(), 's.bin')
    if not (a.data and os.path.exists(path)):
        scene.write_named(a.scene, path)
    devs = [int(x) for x in a.devices.split(',')]
    r = Renderer(path, device=devs[0])
    r.configure_devices(devs if len(devs) > 1 else [])
    r.configure(path, devs[0])
    r.set_delivery(a.delivery, a.fill_threads)
    W, H = a.width, a.height
    buf = DoubleBuffer(W, H, a.line_offset)
    for t in poses.script(a.pose):
        r.lib.updateAndRender(ctypes.byref(buf.next()), ctypes.byref(Input.of(t)))
    hold = Input.of(poses.hold(a.pose))
    hr = ctypes.byref(hold)
    refs = [ctypes.byref(h) for h in buf.halves]
    for k in range(a.warmup):
        r.lib.updateAndRender(refs[k & 1], hr)
    r.fill_profile()                                  # clear
    per = np.empty(a.frames)
    for k in range(a.frames):
        t0 = time.perf_counter()
        r.lib.updateAndRender(refs[k & 1], hr)
        per[k] = time.perf_counter() - t0
    st = r.host_stats()
    st['fill_profile'] = r.fill_profile()
    st.update(numa_report(buf))
    print(json.dumps({'delivery': a.delivery, 'devices': devs, 'median_ms': round(float(np.median(per)) * 1e3, 4),
                      'p10_ms': round(float(np.percentile(per, 10)) * 1e3, 4),
                      'p90_ms': round(float(np.percentile(per, 90)) * 1e3, 4),
                      'fps': round(1 / float(np.median(per)), 1), **st}))
    r.shutdown()
    buf.free()


if __name__ == '__main__':
    main()
