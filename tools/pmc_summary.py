"""Summarise rocprofv3 --pmc passes (one directory per pass, csv output) per kernel.

usage: python tools/pmc_summary.py gpurun_out/pmc [kernel-substring ...]

Per kernel name (template arguments kept, argument list dropped) it prints the
dispatch count, average duration and, per counter, the average value per
dispatch.  FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3; on gfx950
FETCH_SIZE counts wide (>=64 B) requests at half size (MI355X_MICROARCH.md,
HBM section), so the HBM estimate below doubles it - the raw value is printed
as well.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("pupil::(anonymous namespace)::", "").replace("pupil::", "")
    return re.sub(r"\(.*", "", name)


def load(root):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
    durs = defaultdict(dict)                        # kernel -> dispatch -> ns
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
            durs[(f, names[r["Dispatch_Id"]])][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (d, c), v in per.items():
            vals[names[d]][c].append(v)
    dur = defaultdict(list)
    for (f, k), m in durs.items():
        dur[k].extend(m.values())
    return vals, dur


def traffic_json(root, kernels, out_path, note=""):
    """Per-launch L2->fabric bytes of one kernel (or of several template
    instances of it, "a|b", averaged over their dispatches): 2 x FETCH_SIZE
    (gfx950 half-count correction for 16 B/lane loads) + WRITE_SIZE, both KiB
    in rocprofv3."""
    import json

    vals, dur = load(root)
    names = kernels.split("|")
    ks = [k for k in vals if k in names]
    assert ks, f"no kernel named {names} in {root}"

    def pooled(c):
        v = [x for k in ks for x in vals[k].get(c, [])]
        return sum(v) / max(1, len(v))

    def total(c):
        return sum(x for k in ks for x in vals[k].get(c, []))

    # rays the plain traversal kernels traced in each pass (bench.py's JSON line,
    # config.rays_traced_plain_process): identical work in every pass
    rays = set()
    simd = None  # the bench line's SIMD efficiency of the traversal (counter frame, same in every pass)
    for lg in sorted(glob.glob(os.path.join(root, "p*.log"))):
        for line in open(lg):
            if line.startswith("{") and '"metric"' in line:
                bl = json.loads(line)
                rays.add(bl["config"].get("rays_traced_plain_process"))
                simd = (bl.get("roofline") or {}).get("simd_efficiency") or simd
    rays.discard(None)
    assert len(rays) <= 1, f"passes traced different ray counts: {rays}"
    n_rays = rays.pop() if rays else None

    f, w = pooled("FETCH_SIZE"), pooled("WRITE_SIZE")
    hit, miss = pooled("TCC_HIT_sum"), pooled("TCC_MISS_sum")
    d = [x for k in ks for x in dur[k]]
    avg_ms = sum(d) / len(d) / 1e6
    valu, grbm = pooled("SQ_INSTS_VALU"), pooled("GRBM_GUI_ACTIVE")
    rec = {"kernel": " + ".join(ks), "round": os.environ.get("PUPIL_ROUND", ""),
           "fetch_size_kib": f, "write_size_kib": w,
           "traffic_bytes_per_launch": (2.0 * f + w) * 1024.0,
           "l2_hit_rate": hit / max(1.0, hit + miss),
           "avg_ms_under_pmc": avg_ms,
           # VALU issue: SQ_INSTS_VALU wave-instructions; GRBM_GUI_ACTIVE is summed over the
           # 8 XCDs, so the engine clock is GRBM / 8 / launch time
           "valu_insts_per_launch": valu or None,
           "clock_ghz": (grbm / 8.0 / (avg_ms * 1e-3) / 1e9) if grbm else None,
           # per traced ray over all dispatches of the pass (launch sizes vary: pipelined
           # launches, a rank's tiles), what bench.py scales by its own rays per launch
           "rays_traced": n_rays,
           "traffic_bytes_per_ray": (2.0 * total("FETCH_SIZE") + total("WRITE_SIZE")) * 1024.0 / n_rays if n_rays else None,
           "valu_insts_per_ray": total("SQ_INSTS_VALU") / n_rays if n_rays and valu else None,
           # vector-memory address processing: TA busy cycles summed over the 256 CUs' TAs, and the
           # VMEM wave-instructions they processed (r05: the traversal's binding unit)
           "ta_busy_cycles_per_ray": total("TA_TA_BUSY_sum") / n_rays if n_rays and pooled("TA_TA_BUSY_sum") else None,
           "vmem_insts_per_ray": total("TA_TOTAL_WAVEFRONTS_sum") / n_rays
           if n_rays and pooled("TA_TOTAL_WAVEFRONTS_sum") else None,
           # the data-return unit (TD, one per CU) and the L1 (TCP) it waits on (r06: the traversal's
           # binding unit, busy ~0.99 of the cycles, about half of them stalled on L1 misses)
           "td_busy_cycles_per_ray": total("TD_TD_BUSY_sum") / n_rays if n_rays and pooled("TD_TD_BUSY_sum") else None,
           "td_tc_stall_cycles_per_ray": total("TD_TC_STALL_sum") / n_rays
           if n_rays and pooled("TD_TC_STALL_sum") else None,
           # the same within the PMC passes themselves: TD busy over 256 TDs and the per-XCD cycles
           # (per-dispatch averages of the TD pass and of the GRBM pass; no live launch time involved)
           "td_busy_frac_under_pmc": pooled("TD_TD_BUSY_sum") / 256.0 / (grbm / 8.0)
           if grbm and pooled("TD_TD_BUSY_sum") else None,
           "td_tc_stall_frac_under_pmc": pooled("TD_TC_STALL_sum") / 256.0 / (grbm / 8.0)
           if grbm and pooled("TD_TC_STALL_sum") else None,
           "tcp_accesses_per_ray": total("TCP_TOTAL_CACHE_ACCESSES_sum") / n_rays
           if n_rays and pooled("TCP_TOTAL_CACHE_ACCESSES_sum") else None,
           "tcp_l2_reads_per_ray": total("TCP_TCC_READ_REQ_sum") / n_rays
           if n_rays and pooled("TCP_TCC_READ_REQ_sum") else None,
           "dispatches": len(d),
           "simd_efficiency": simd,
           "note": note}
    with open(out_path, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


def main(root, filters):
    vals, dur = load(root)
    for k in sorted(vals, key=lambda k: -sum(dur[k])):
        if filters and not any(s in k for s in filters):
            continue
        d = dur[k]
        avg_ms = sum(d) / len(d) / 1e6
        print(f"{k}  dispatches/pass~{len(vals[k][next(iter(vals[k]))])}  avg {avg_ms:.4f} ms")
        for c, v in sorted(vals[k].items()):
            a = sum(v) / len(v)
            extra = ""
            if c == "FETCH_SIZE":
                extra = f"   (x2 gfx950 -> {2 * a / 1e6:.3f} GB, {2 * a * 1e3 / (avg_ms * 1e-3) / 1e9:.1f} GB/s)"
            if c == "WRITE_SIZE":
                extra = f"   ({a / 1e6:.3f} GB)"
            print(f"    {c:24s} {a:16.1f}{extra}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "--json":  # pmc_summary.py ROOT --json KERNEL OUT [NOTE]
        traffic_json(sys.argv[1], sys.argv[3], sys.argv[4], " ".join(sys.argv[5:]))
    else:
        main(sys.argv[1], sys.argv[2:])
