#!/usr/bin/env python3
"""Kernel timeline of one window of a rocprofv3 --kernel-trace CSV: for the fragment launches
[first, first + count) and every kernel that overlaps them, start / end / duration in microseconds
relative to the first one's start, plus the gap after the previous fragment launch.

    python3 tools/trace_timeline.py <kernel_trace.csv> --first 7 --count 20
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--first', type=int, default=0)
    ap.add_argument('--count', type=int, default=20)
    ap.add_argument('--frag', default='k_fragment')
    a = ap.parse_args()
    rows = []
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            name = r['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1]
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), name))
    rows.sort()
    frags = [r for r in rows if a.frag in r[2]]
    win = frags[a.first:][:a.count]                 # (a negative --first counts from the last launch)
    if not win:
        raise SystemExit('no fragment launches in the window')
    t0, t1 = win[0][0], win[-1][1]
    prev_end = None
    busy = 0
    for s, e, n in rows:
        if e < t0 - 200_000 or s > t1:
            continue
        gap = ''
        if a.frag in n:
            if prev_end is not None:
                gap = f'gap {(s - prev_end) / 1e3:7.2f}'
            prev_end = e
            busy += e - s
        print(f'{(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  {n:24s} {gap}')
    print(f'window {(t1 - t0) / 1e3:.2f} us for {len(win)} fragment launches: '
          f'{(t1 - t0) / 1e3 / len(win):.2f} us per frame, fragment busy {busy / 1e3 / len(win):.2f} us per frame')


if __name__ == '__main__':
    main()
