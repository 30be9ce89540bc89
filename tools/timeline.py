"""Kernel timeline of the last K dispatches of a rocprofv3 kernel trace: each kernel's
duration and the idle gap before it, summed by kernel name, plus the wall span, busy time
and gap total -- where a short-launch cadence (the 1-spp OnRun of one rank's tiles) loses
its time.

usage: python tools/timeline.py run_kernel_trace.csv [last_dispatches=200] [--list 40]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("pupil::(anonymous namespace)::", "").replace("pupil::", "")
    return re.sub(r"\(.*", "", name)


def main(path, last=200, listing=0):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-last:]
    if not rows:
        return
    t0 = int(rows[0]["Start_Timestamp"])
    busy = 0
    gaps = defaultdict(float)
    dur = defaultdict(float)
    calls = defaultdict(int)
    prev_end = None
    for i, r in enumerate(rows):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        g = 0 if prev_end is None else max(0, s - prev_end)
        gaps[k] += g / 1e3
        dur[k] += (e - s) / 1e3
        calls[k] += 1
        busy += e - s
        if i >= len(rows) - listing:
            print(f"{(s - t0) / 1e3:10.1f} us  +{g / 1e3:7.1f} gap  {(e - s) / 1e3:8.1f} us  {k}")
        prev_end = max(prev_end or 0, e)
    span = (prev_end - t0) / 1e3
    print(f"last {len(rows)} dispatches: span {span:.1f} us, kernels {busy / 1e3:.1f} us, gaps {span - busy / 1e3:.1f} us")
    print(f"{'kernel':44s} {'calls':>6s} {'us total':>10s} {'us avg':>8s} {'gap before us':>14s}")
    for k in sorted(dur, key=lambda k: -dur[k]):
        print(f"{k[:44]:44s} {calls[k]:6d} {dur[k]:10.1f} {dur[k] / calls[k]:8.1f} {gaps[k]:14.1f}")


if __name__ == "__main__":
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    lst = int(sys.argv[sys.argv.index("--list") + 1]) if "--list" in sys.argv else 0
    if "--list" in sys.argv:
        a.remove(str(lst))
    main(a[0], int(a[1]) if len(a) > 1 else 200, lst)
