"""Per-kernel ISA statistics of a built object (instructions, LDS/global/scratch ops,
VGPRs, spills): python tools/isa_stats.py build/obj/pt_kernels.o [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main(obj, filt=""):
    with tempfile.TemporaryDirectory() as d:
        import shutil

        local = os.path.join(d, os.path.basename(obj))
        shutil.copy(obj, local)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", local], cwd=d, check=True, capture_output=True)
        co = [os.path.join(d, f) for f in os.listdir(d) if "gfx950" in f][0]
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], capture_output=True, text=True).stdout
        sy = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "-W", co], capture_output=True, text=True).stdout
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    regs = {}
    for blk in notes.split(".name:")[1:]:
        name = blk.split()[0]
        m = {k: re.search(rf"\.{k}:\s+(\d+)", blk) for k in ("vgpr_count", "vgpr_spill_count")}
        regs[name] = {k: int(v.group(1)) for k, v in m.items() if v}
    syms = set()
    for l in sy.split("\n"):
        p = l.split()
        if len(p) >= 8 and p[3] == "FUNC":
            syms.add((int(p[1], 16), int(p[2]), p[7]))
    ins = []
    for l in dis.split("\n"):
        m = re.search(r"//\s*([0-9A-F]{12}):", l)
        if m:
            ins.append((int(m.group(1), 16), l.strip()))
    for addr, size, name in sorted(syms):
        if filt not in name:
            continue
        body = [l for a, l in ins if addr <= a < addr + size]
        c = lambda k: sum(1 for l in body if l.startswith(k))
        r = regs.get(name, {})
        print(f"{name[:70]:70s} n={len(body):5d} ds={c('ds_'):4d} global={c('global_'):4d} "
              f"scratch={c('scratch_'):3d} vgpr={r.get('vgpr_count')} spill={r.get('vgpr_spill_count')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
