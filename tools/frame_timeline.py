"""Per-frame kernel timeline from a rocprofv3 --kernel-trace csv: span of the last
frame (k_generate .. k_accumulate), summed kernel busy time, and per kernel the
busy time and the idle gap before its launches (launch/dependency overhead).

usage: python tools/frame_timeline.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    return re.sub(r"\(.*", "", n.replace("void ", "").replace("pupil::(anonymous namespace)::", ""))


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gens = [i for i, r in enumerate(rows) if "k_generate" in r["Kernel_Name"]]
    i0 = gens[-1]
    i1 = [i for i, r in enumerate(rows) if i > i0 and "k_accumulate" in r["Kernel_Name"]][0]
    fr = rows[i0:i1 + 1]
    t0 = int(fr[0]["Start_Timestamp"])
    t1 = int(fr[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in fr)
    print(f"frame span {(t1 - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, {len(fr)} dispatches")
    prev = t0
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for r in fr:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += (e - s) / 1e3
        a[2] += (s - prev) / 1e3
        prev = e
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{k[:44]:44s} n={v[0]:3d} busy={v[1]:9.1f} us  gaps_before={v[2]:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
