#!/usr/bin/env python3
"""Per-stage breakdown of one frame part's pipelined frames from a rocprofv3 --kernel-trace CSV
(VERDICT r05 item 4): over the last `--frames` fragment launches, the mean period between fragment
starts, the fragment kernel's span, the geometry kernel's span, the idle gap between one fragment
launch's end and the next one's start, and how much of each geometry launch ran under the previous
fragment launch.  With the probe's host enqueue time (tools/overhead_probe.py host_enqueue_us) this
says what bounds the part's frame period: the host, the fragment kernel, or the boundary.

    python3 tools/eighth_breakdown.py <kernel_trace.csv> [--frames 400] [--host-us 18.5]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--frames', type=int, default=400)
    ap.add_argument('--host-us', type=float, default=None)
    ap.add_argument('--label', default='')
    a = ap.parse_args()
    rows = []
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            name = r['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1]
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), name))
    rows.sort()
    frag = [r for r in rows if r[2].startswith('k_fragment') or r[2].startswith('k_tile_raster')]
    geo = [r for r in rows if r[2].startswith('k_geometry') or r[2].startswith('k_tile_setup')]
    frag = frag[-a.frames:]
    t0 = frag[0][0]
    geo = [g for g in geo if g[0] >= t0 - 100000]
    n = len(frag)
    us = lambda ns: ns / 1e3                                     # noqa: E731
    period = us(frag[-1][0] - frag[0][0]) / (n - 1)
    frag_span = sum(us(e - s) for s, e, _ in frag) / n
    gaps = [us(frag[i][0] - frag[i - 1][1]) for i in range(1, n)]
    geo_span = sum(us(e - s) for s, e, _ in geo) / max(len(geo), 1)
    # geometry k+1 under fragment k: the part of each geometry launch before the previous fragment end
    under = []
    for s, e, _ in geo:
        prev = [f for f in frag if f[0] <= s]
        if prev:
            pe = prev[-1][1]
            under.append(max(0.0, us(min(e, pe) - s)))
    out = {'label': a.label, 'frames': n, 'period_us': round(period, 2), 'fragment_span_us': round(frag_span, 2),
           'geometry_span_us': round(geo_span, 2), 'gap_us_mean': round(sum(gaps) / len(gaps), 2),
           'gap_us_max': round(max(gaps), 2), 'geometry_under_previous_fragment_us': round(sum(under) / max(len(under), 1), 2),
           'fragment_kernel': frag[-1][2], 'geometry_kernel': geo[-1][2] if geo else None}
    if a.host_us is not None:
        out['host_enqueue_us'] = a.host_us
        out['bound'] = 'host' if a.host_us >= period * 0.95 else ('fragment' if frag_span >= period * 0.9 else 'boundary')
    print(json.dumps(out))


if __name__ == '__main__':
    main()
