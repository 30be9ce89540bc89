"""Dispatch timeline of the last frame of a rocprofv3 --kernel-trace csv, with the
queue of each dispatch, to see whether the stage sequences of several engine lanes
(PUPIL_LANES) overlap on the GPU.

usage: python tools/lane_timeline.py gpurun_out/<dir>/run_kernel_trace.csv [lanes=2]
"""
import csv
import re
import sys


def short(n):
    return re.sub(r"\(.*", "", n.replace("void ", "").replace("pupil::(anonymous namespace)::", ""))[:40]


def main(path, lanes=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gens = [i for i, r in enumerate(rows) if "k_generate" in r["Kernel_Name"]]
    i0 = gens[-lanes]
    fr = rows[i0:]
    t0 = int(fr[0]["Start_Timestamp"])
    qcol = next((c for c in ("Queue_Id", "Stream_Id") if c in fr[0]), None)
    busy = {}
    for r in fr:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        q = r.get(qcol, "?") if qcol else "?"
        busy[q] = busy.get(q, 0) + (e - s)
        print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q={q:>3}  {short(r['Kernel_Name'])}")
    t1 = max(int(r["End_Timestamp"]) for r in fr) - t0
    print(f"span {t1 / 1e3:.1f} us; busy per queue: " + ", ".join(f"{q}: {b / 1e3:.1f}" for q, b in busy.items()))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
