"""ctypes mirror of include/pupil_pt.h (the C ABI of libpupil_pt.so).

The structures below must match the header field for field; tests/test_abi.py
checks sizes against a compiled probe and that every declared symbol is
exported.
"""
from __future__ import annotations

import ctypes as C
import os

TEX_RGB, TEX_BITMAP, TEX_CHECKERBOARD = 0, 1, 2
MAT_UNKNOWN, MAT_DIFFUSE, MAT_DIELECTRIC, MAT_ROUGH_DIELECTRIC = 0, 1, 2, 3
MAT_CONDUCTOR, MAT_ROUGH_CONDUCTOR, MAT_PLASTIC, MAT_ROUGH_PLASTIC = 4, 5, 6, 7
EMITTER_NONE, EMITTER_TRI_AREA, EMITTER_SPHERE, EMITTER_CONST_ENV, EMITTER_ENV_MAP = 0, 1, 2, 3, 4
SHAPE_MESH, SHAPE_SPHERE = 0, 1

PUPIL_OK = OK = 0
ERR_INVALID, ERR_HIP, ERR_OOM, ERR_IO, ERR_UNSUPPORTED = -1, -2, -3, -4, -5
IMAGE_AUTO, IMAGE_EXR, IMAGE_HDR, IMAGE_PFM = 0, 1, 2, 3
ERR_NAMES = {-1: "PUPIL_ERR_INVALID", -2: "PUPIL_ERR_HIP", -3: "PUPIL_ERR_OOM", -4: "PUPIL_ERR_IO",
             -5: "PUPIL_ERR_UNSUPPORTED"}

f32p = C.POINTER(C.c_float)
u32p = C.POINTER(C.c_uint32)


class Texture(C.Structure):
    _fields_ = [("type", C.c_uint32), ("c0", C.c_float * 3), ("c1", C.c_float * 3),
                ("transform", C.c_float * 16), ("width", C.c_uint32), ("height", C.c_uint32),
                ("filter", C.c_uint32), ("pad", C.c_uint32), ("rgba", f32p)]


class Material(C.Structure):
    _fields_ = [("type", C.c_uint32), ("twosided", C.c_uint32), ("int_ior", C.c_float),
                ("ext_ior", C.c_float), ("nonlinear", C.c_uint32), ("tex", Texture * 4)]


class Shape(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("num_vertices", C.c_uint32), ("num_faces", C.c_uint32),
                ("positions", f32p), ("normals", f32p), ("texcoords", f32p), ("indices", u32p)]


class Instance(C.Structure):
    _fields_ = [("shape", C.c_uint32), ("material", C.c_uint32), ("to_world", C.c_float * 12),
                ("to_object", C.c_float * 12), ("flip_normals", C.c_uint32),
                ("flip_tex_coords", C.c_uint32), ("emitter_offset", C.c_int32), ("pad", C.c_uint32)]


class Emitter(C.Structure):
    _fields_ = [("type", C.c_uint32), ("weight", C.c_float), ("select_probability", C.c_float),
                ("area", C.c_float), ("radiance", Texture), ("pos", (C.c_float * 3) * 3),
                ("nrm", (C.c_float * 3) * 3), ("tex", (C.c_float * 2) * 3), ("center", C.c_float * 3),
                ("radius", C.c_float), ("color", C.c_float * 3), ("to_world", C.c_float * 9),
                ("to_local", C.c_float * 9), ("scale", C.c_float)]


class SceneDesc(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("max_depth", C.c_uint32),
                ("pad0", C.c_uint32), ("sample_to_camera", C.c_float * 16),
                ("camera_to_world", C.c_float * 16), ("num_shapes", C.c_uint32),
                ("num_materials", C.c_uint32), ("num_instances", C.c_uint32),
                ("num_area_emitters", C.c_uint32), ("shapes", C.POINTER(Shape)),
                ("materials", C.POINTER(Material)), ("instances", C.POINTER(Instance)),
                ("area_emitters", C.POINTER(Emitter)), ("env", C.POINTER(Emitter))]


class Frame(C.Structure):
    _fields_ = [("accum", C.c_void_p), ("frame", C.c_void_p), ("albedo", C.c_void_p),
                ("normal", C.c_void_p), ("test", C.c_void_p), ("compact", C.c_uint32),
                ("pad", C.c_uint32)]


class Launch(C.Structure):
    _fields_ = [("random_seed", C.c_uint32), ("sample_cnt", C.c_uint32), ("spp", C.c_uint32),
                ("max_depth", C.c_uint32), ("accumulate", C.c_uint32), ("tile_size", C.c_uint32),
                ("tile_rank", C.c_uint32), ("tile_world", C.c_uint32), ("collect_stats", C.c_uint32),
                ("hints", C.c_uint32)]


class Counters(C.Structure):
    _fields_ = [("primary_rays", C.c_uint64), ("extension_rays", C.c_uint64),
                ("shadow_rays", C.c_uint64), ("path_samples", C.c_uint64),
                ("node_visits", C.c_uint64), ("prim_tests", C.c_uint64), ("bvh_nodes", C.c_uint64),
                ("bvh_prims", C.c_uint64), ("build_ms", C.c_double), ("last_render_ms", C.c_double),
                ("trace_ms", C.c_double), ("trace_bytes", C.c_double), ("trace_launches", C.c_uint64),
                ("extend_ms", C.c_double), ("extend_launches", C.c_uint64), ("extend_node_visits", C.c_uint64),
                ("extend_prim_tests", C.c_uint64), ("extend_bytes", C.c_double), ("shade_ms", C.c_double),
                ("two_level", C.c_uint64), ("shadow_rays_reference", C.c_uint64),
                ("bvh_depth", C.c_uint64), ("unique_node_fetches", C.c_uint64),
                # ABI 3
                ("rays_traced_total", C.c_uint64), ("frames_in_flight", C.c_uint64),
                ("pipeline_slots", C.c_uint64), ("tlas_sah_splits", C.c_uint64),
                ("queue_handed", C.c_uint64), ("queue_activated", C.c_uint64), ("queue_retired", C.c_uint64),
                ("queue_listed", C.c_uint64), ("ring_bytes", C.c_uint64), ("ring_budget_bytes", C.c_uint64),
                ("accel_refits", C.c_uint64), ("node_bound", C.c_float * 3), ("pad_counters", C.c_uint32),
                # ABI 5
                ("node_loop_iters", C.c_uint64), ("node_loop_lanes", C.c_uint64), ("leaf_loop_iters", C.c_uint64),
                ("leaf_loop_lanes", C.c_uint64), ("refills", C.c_uint64), ("refill_lanes", C.c_uint64),
                ("frame_launches", C.c_uint64),
                # ABI 6
                ("frame_ms", C.c_double), ("coop_dma", C.c_uint64), ("coop_slots", C.c_uint64)]

    def as_dict(self):
        d = {name: getattr(self, name) for name, _ in self._fields_ if name != "pad_counters"}
        d["node_bound"] = [float(x) for x in self.node_bound]
        return d


DENOISE_USE_ALBEDO, DENOISE_USE_NORMAL, DENOISE_APPLY_TO_AOV = 1, 2, 4
DENOISE_USE_TEMPORAL, DENOISE_USE_UPSCALE_2X, DENOISE_TILED = 8, 16, 32


class DenoiseData(C.Structure):
    _fields_ = [("input", C.c_void_p), ("output", C.c_void_p), ("prev_output", C.c_void_p),
                ("albedo", C.c_void_p), ("normal", C.c_void_p), ("motion_vector", C.c_void_p)]


# name -> (restype, argtypes); every entry is declared in include/pupil_pt.h
SIGNATURES = {
    "pupil_last_error": (C.c_char_p, []),
    "pupil_abi_version": (C.c_int, []),
    "pupil_pt_create": (C.c_int, [C.POINTER(SceneDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "pupil_pt_set_camera": (C.c_int, [C.c_void_p, f32p, f32p]),
    "pupil_pt_update_instance": (C.c_int, [C.c_void_p, C.c_uint32, f32p, f32p]),
    "pupil_pt_update_instances": (C.c_int, [C.c_void_p, C.c_uint32, u32p, f32p, f32p]),
    "pupil_pt_update_emitters": (C.c_int, [C.c_void_p, C.POINTER(SceneDesc)]),
    "pupil_debug_fill_tlas_reserve": (C.c_int, [C.c_void_p, C.c_float]),
    "pupil_pt_render": (C.c_int, [C.c_void_p, C.POINTER(Frame), C.POINTER(Launch), C.c_void_p]),
    "pupil_pt_stats": (C.c_int, [C.c_void_p, C.POINTER(Counters)]),
    "pupil_pt_local_pixels": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         u32p, u32p]),
    "pupil_pt_destroy": (None, [C.c_void_p]),
    "pupil_pt_trace_rays": (C.c_int, [C.c_void_p, C.c_uint32, f32p, f32p, C.c_int]),
    "pupil_pt_export_bvh4": (C.c_int, [C.c_void_p, u32p, C.c_void_p, u32p, f32p, C.POINTER(C.c_int32)]),
    "pupil_debug_math": (C.c_int, [C.c_int, C.c_uint32, f32p, f32p, f32p]),
    "pupil_image_save": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, f32p, C.c_uint32]),
    "pupil_debug_select_emitter": (C.c_int, [C.c_void_p, C.c_uint32, f32p, C.POINTER(C.c_int32)]),
    "pupil_image_load": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), f32p]),
    "pupil_world_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "pupil_world_load_xml": (C.c_int, [C.c_void_p, C.c_char_p]),
    "pupil_world_set_film": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]),
    "pupil_world_set_sensor": (C.c_int, [C.c_void_p, C.c_float, C.c_char, C.c_float, C.c_float, f32p]),
    "pupil_world_add_mesh": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, f32p, f32p, f32p, u32p, u32p]),
    "pupil_world_add_builtin_shape": (C.c_int, [C.c_void_p, C.c_char_p, u32p]),
    "pupil_world_add_material": (C.c_int, [C.c_void_p, C.POINTER(Material), u32p]),
    "pupil_world_add_instance": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, f32p, C.c_uint32,
                                           C.c_uint32, C.c_uint32, C.POINTER(Texture), u32p]),
    "pupil_world_add_const_env": (C.c_int, [C.c_void_p, f32p]),
    "pupil_world_set_instance_transform": (C.c_int, [C.c_void_p, C.c_uint32, f32p]),
    "pupil_world_get_desc": (C.c_int, [C.c_void_p, C.POINTER(SceneDesc)]),
    "pupil_world_destroy": (None, [C.c_void_p]),
    "pupil_denoiser_create": (C.c_int, [C.c_int, C.c_uint32, C.POINTER(C.c_void_p)]),
    "pupil_denoiser_setup": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_float]),
    "pupil_denoiser_execute": (C.c_int, [C.c_void_p, C.POINTER(DenoiseData), C.c_void_p]),
    "pupil_denoiser_destroy": (None, [C.c_void_p]),
}

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libpupil_pt.so")


class PupilError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{ERR_NAMES.get(code, code)}: {message}")
        self.code = code


_LIB = None


def load_library(path: str | None = None):
    """Load libpupil_pt.so.  Raises if it is missing (never falls back)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # torch bundles its own libamdhip64.so.7; importing it first makes our
    # library bind to the same HIP runtime instead of loading a second copy.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for host-only use
        pass
    # PUPIL_LIB: an alternative build of the same library (A/B experiments, tools/gpu_lib_sweep.sh)
    p = path or os.environ.get("PUPIL_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        if p != LIB_PATH and not hasattr(lib, name):  # an older A/B build (PUPIL_LIB) lacks newer entry points
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


def check(code: int, lib=None):
    if code != PUPIL_OK:
        lib = lib or load_library()
        msg = lib.pupil_last_error()
        raise PupilError(code, msg.decode() if msg else "")
    return code
