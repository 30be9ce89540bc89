"""Compare the last 1-GPU frame with the last N-way-shard frame of one
rocprofv3 --kernel-trace csv written by tools/shard_probe.py --worlds 1 N:
per kernel the busy time at 1 GPU, at the shard, the ideal (1-GPU / N) and
the excess, plus the frame span and idle gaps.

usage: python tools/timeline_compare.py gpurun_out/<dir>/run_kernel_trace.csv N
"""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from frame_timeline import short  # noqa: E402


def frame(rows, i0):
    i1 = [i for i, r in enumerate(rows) if i > i0 and "k_accumulate" in r["Kernel_Name"]][0]
    fr = rows[i0:i1 + 1]
    agg = defaultdict(float)
    prev = int(fr[0]["Start_Timestamp"])
    gap = 0.0
    for r in fr:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        agg[short(r["Kernel_Name"])] += (e - s) / 1e3
        gap += max(0, s - prev) / 1e3
        prev = max(prev, e)
    return (int(fr[-1]["End_Timestamp"]) - int(fr[0]["Start_Timestamp"])) / 1e3, agg, gap


def main(path, n):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gens = [i for i, r in enumerate(rows) if "k_generate" in r["Kernel_Name"]]
    per_world1 = len(gens) - n * (len(gens) // (n + 1))  # frames of the 1-GPU pass come first
    s1, a1, g1 = frame(rows, gens[per_world1 - 1])
    s8, a8, g8 = frame(rows, gens[-1])
    print(f"1 GPU frame span {s1:.1f} us (gaps {g1:.1f}); shard 1/{n}: span {s8:.1f} us (gaps {g8:.1f}), "
          f"ideal {s1 / n:.1f} us")
    for k in sorted(a1, key=lambda k: -a1[k]):
        print(f"{k[:40]:40s} {a1[k]:9.1f} {a8.get(k, 0):8.1f} ideal {a1[k] / n:8.1f} excess {a8.get(k, 0) - a1[k] / n:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
