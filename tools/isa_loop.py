"""Dump one kernel's disassembly from a built object and count the instructions of
the basic blocks between two markers (default: the BVH4 node loop of k_trace4, from
the block holding the node's four global_load_dwordx4 up to the stack pushes).

usage: python tools/isa_loop.py build/obj/pt_kernels.o "k_trace4<4, false, false, false>" [out.s]
Prints per-class counts (VALU, SALU, VMEM, LDS) of the whole kernel and of the node
loop body (the straight-line path from the node fetch to the next fetch's branch)."""
import os
import re
import shutil
import subprocess
import sys
import tempfile
from collections import Counter

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(obj, kernel):
    with tempfile.TemporaryDirectory() as d:
        local = os.path.join(d, os.path.basename(obj))
        shutil.copy(obj, local)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", local], cwd=d, check=True, capture_output=True)
        co = [os.path.join(d, f) for f in os.listdir(d) if "gfx950" in f][0]
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", co], capture_output=True,
                             text=True).stdout
        sy = subprocess.run(f"{LLVM}/llvm-readelf -s -W {co} | c++filt", shell=True, capture_output=True,
                            text=True).stdout
    addr = size = None
    for l in sy.split("\n"):
        p = l.split(None, 7)
        if len(p) >= 8 and p[3] == "FUNC" and kernel in p[7]:
            addr, size = int(p[1], 16), int(p[2])
            break
    assert addr is not None, kernel
    out = []
    for l in dis.split("\n"):
        m = re.search(r"//\s*([0-9A-F]{12}):", l)
        if m and addr <= int(m.group(1), 16) < addr + size:
            out.append(re.sub(r"\s+//\s*[0-9A-F]{12}:.*", "", l).strip())
        elif re.match(r"^[0-9a-f]{16} <L\d+>:", l) and addr <= int(l[:16], 16) < addr + size:
            out.append(l.split()[1])
    return out


def klass(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    return "other"


def main(obj, kernel, out_path=None):
    lines = disasm(obj, kernel)
    if out_path:
        open(out_path, "w").write("\n".join(lines) + "\n")
    body = [l for l in lines if not l.startswith("<")]
    print(f"{kernel}: {len(body)} instructions", dict(Counter(klass(l) for l in body)))
    # node loop: from the first block with 4 global_load_dwordx4 within 5 lines (the node) to the
    # first ds_write after it (the stack pushes) and the loop-control tail up to the back-edge
    idx = next(i for i in range(len(lines) - 4)
               if sum(lines[i + k].startswith("global_load_dwordx4") for k in range(5)) == 4
               and lines[i].startswith("global_load_dwordx4"))
    start = max(j for j in range(idx) if lines[j].startswith("<"))
    seg = []
    for l in lines[start:]:
        seg.append(l)
        if l.startswith("s_cbranch_execz") and len(seg) > 40 and any(x.startswith("v_cmp_neq_f32") for x in seg):
            break
    c = Counter(klass(l) for l in seg if not l.startswith("<"))
    print(f"node fetch + box test + sort head ({seg[0]}): {dict(c)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
