"""Per-dispatch durations of one kernel from a rocprofv3 kernel trace, in dispatch order,
and the mean of the last N (the timed region of a bench run, whose traversal launches
are the last ones of their kernel).

usage: python tools/timed_kernels.py run_kernel_trace.csv "k_trace4<4, false, false, false>" [N]
"""
import csv
import re
import sys


def short(name):
    name = name.replace("void ", "").replace("pupil::(anonymous namespace)::", "").replace("pupil::", "")
    return re.sub(r"\(.*", "", name)


def main(path, kernel, last):
    rows = [r for r in csv.DictReader(open(path)) if short(r["Kernel_Name"]) == kernel]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    print(f"{kernel}: {len(d)} dispatches, ms: " + " ".join(f"{x:.4f}" for x in d))
    if last and len(d) >= last:
        t = d[-last:]
        print(f"last {last} (timed region): mean {sum(t) / len(t):.4f} ms, min {min(t):.4f}, max {max(t):.4f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0)
