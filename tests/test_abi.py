"""The C-ABI library loads on a GPU-less host and exports every declared symbol;
the ctypes mirrors match the C struct layouts (checked against a compiled probe)."""
import os
import re
import subprocess

import pytest

from pupiloptixlab_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pupil_pt.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pupil_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = abi.load_library()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes signature table covers the header exactly
    assert sorted(abi.SIGNATURES) == names


def test_nm_shows_extern_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (pupil_\w+)", out))
    assert set(declared_functions()) <= exported


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "pupil_pt.h"
#define S(t) printf(#t " %zu\n", sizeof(t));
#define O(t, f) printf(#t "." #f " %zu\n", offsetof(t, f));
int main(void) {
  S(pupil_texture) S(pupil_material) S(pupil_shape) S(pupil_instance) S(pupil_emitter)
  S(pupil_scene_desc) S(pupil_pt_frame) S(pupil_pt_launch) S(pupil_pt_counters)
  O(pupil_texture, rgba) O(pupil_material, tex) O(pupil_instance, emitter_offset) O(pupil_emitter, radiance)
  O(pupil_emitter, scale) O(pupil_scene_desc, shapes) O(pupil_scene_desc, env) O(pupil_pt_counters, trace_launches) O(pupil_pt_counters, node_loop_iters) O(pupil_pt_counters, refill_lanes) O(pupil_pt_counters, frame_launches) O(pupil_pt_counters, frame_ms) O(pupil_pt_counters, coop_slots)
  O(pupil_pt_launch, collect_stats) O(pupil_pt_launch, hints)
  printf("PUPIL_HINT_CONTINUE %u\n", PUPIL_HINT_CONTINUE);
  return 0;
}
"""


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True,
                                                               text=True).stdout.split("\n") if line)
    import ctypes as C

    py = {"pupil_texture": abi.Texture, "pupil_material": abi.Material, "pupil_shape": abi.Shape,
          "pupil_instance": abi.Instance, "pupil_emitter": abi.Emitter, "pupil_scene_desc": abi.SceneDesc,
          "pupil_pt_frame": abi.Frame, "pupil_pt_launch": abi.Launch, "pupil_pt_counters": abi.Counters}
    for cname, cls in py.items():
        assert int(got[cname]) == C.sizeof(cls), cname
    assert int(got["PUPIL_HINT_CONTINUE"]) == 1  # what PTPass.render(continues=True) sets
    for key, val in got.items():
        if "." in key:
            cname, field = key.split(".")
            assert getattr(py[cname], field).offset == int(val), key


def test_errors_are_codes_not_exceptions():
    lib = abi.load_library()
    # null arguments -> PUPIL_ERR_INVALID with a message, never a crash
    assert lib.pupil_pt_create(None, 0, None) == -1
    assert b"null" in lib.pupil_last_error()
    import ctypes as C

    n = C.c_uint32(0)
    assert lib.pupil_pt_local_pixels(0, 10, 32, 0, 1, None, C.byref(n)) == -1
    with pytest.raises(abi.PupilError):
        abi.check(-4)


def test_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("host has a GPU")
    from pupiloptixlab_amd import World, scenes

    w = World().load_scene(scenes.cornell_xml(os.path.join(ROOT, "gpurun_out", "abi_cb.xml"), 16, 16))
    d = w.desc()
    import ctypes as C

    h = C.c_void_p()
    rc = abi.load_library().pupil_pt_create(C.byref(d), 0, C.byref(h))
    assert rc == -2  # PUPIL_ERR_HIP: no device, no silent CPU fallback
