"""Summarise a rocprofv3 *_kernel_stats.csv: short kernel name, calls, total and average ms."""
import csv
import re
import sys


def short(name):
    name = name.replace("void ", "").replace("pupil::(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)  # drop the argument list


def main(path):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':40s} {'calls':>6s} {'total ms':>10s} {'avg ms':>9s} {'%':>6s}")
    for r in rows:
        t = float(r["TotalDurationNs"])
        print(f"{short(r['Name'])[:40]:40s} {int(r['Calls']):6d} {t / 1e6:10.3f} {float(r['AverageNs']) / 1e6:9.4f} "
              f"{100 * t / tot:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
