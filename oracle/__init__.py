"""CPU oracle — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of oracle/_build/liboracle.so (built from pt_oracle.cpp by
oracle/Makefile).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it, as the checker / CPU baseline; the product
package (pupiloptixlab_amd) never imports it.

Parity status: unpinned against reference outputs (the OptiX reference cannot
be built or run here and ships no golden data); pinned by the
known-answer tests in tests/test_oracle_kat.py and the fixtures in tests/golden/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PUPIL_ORACLE_LIB: another build of the same source (bench.py's cpu_baseline builds
# one with -march=native on the host it runs on)
LIB_PATH = os.environ.get("PUPIL_ORACLE_LIB") or os.path.join(HERE, "_build", "liboracle.so")


class OracleStats(C.Structure):
    _fields_ = [("primary_rays", C.c_uint64), ("extension_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("seconds", C.c_double), ("threads", C.c_uint32), ("shadow_rays_reference", C.c_uint64)]


_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, f32p, u32p = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_uint32)
        L.oracle_scene_create.restype = vp
        L.oracle_scene_create.argtypes = [vp]
        L.oracle_scene_destroy.argtypes = [vp]
        L.oracle_render.restype = C.c_int
        L.oracle_render.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u32p,
                                    C.c_uint32, f32p, f32p, f32p, f32p, C.c_int, C.POINTER(OracleStats)]
        L.oracle_rng_sequence.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, f32p, u32p]
        L.oracle_camera_ray.argtypes = [vp, C.c_uint32, C.c_uint32, f32p]
        L.oracle_closest.argtypes = [vp, C.c_uint32, f32p, f32p, C.c_int]
        L.oracle_bsdf.argtypes = [vp, C.c_uint32, C.c_float, C.c_float, f32p, f32p, C.c_uint32, f32p]
        L.oracle_emitter_sample.argtypes = [vp, C.c_uint32, f32p, f32p, C.c_float, C.c_float, f32p]
        L.oracle_emitter_sample.restype = C.c_int
        L.oracle_math.argtypes = [C.c_uint32, f32p, f32p, f32p]
        L.oracle_num_prims.restype = C.c_uint32
        L.oracle_num_prims.argtypes = [vp]
        L.oracle_set_bvh4.restype = C.c_int
        L.oracle_set_bvh4.argtypes = [vp, C.c_uint32, vp, C.c_uint32, f32p, C.c_int32]
        _LIB = L
    return _LIB


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class OracleScene:
    """The oracle's own copy of a pupil_scene_desc (with its own SAH BVH)."""

    def __init__(self, desc):
        self._desc = desc  # the desc's arrays must outlive the oracle scene
        self.width, self.height = desc.width, desc.height
        self._h = lib().oracle_scene_create(C.byref(desc))

    def close(self):
        if self._h:
            lib().oracle_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, spp=1, random_seed=0, sample_cnt=0, max_depth=0, accumulate=True, pixels=None, accum=None,
               threads=0):
        """spp frames of PTPass::OnRun; returns dict(accum, albedo, normal, test, stats)."""
        n = self.width * self.height if pixels is None else len(pixels)
        acc = np.zeros((n, 4), np.float32) if accum is None else np.ascontiguousarray(accum, np.float32).copy()
        alb = np.zeros((n, 3), np.float32)
        nrm = np.zeros((n, 3), np.float32)
        tst = np.zeros((n,), np.float32)
        st = OracleStats()
        pix = None
        if pixels is not None:
            pix_arr = np.ascontiguousarray(pixels, np.uint32)
            pix = pix_arr.ctypes.data_as(C.POINTER(C.c_uint32))
        lib().oracle_render(self._h, random_seed, sample_cnt, spp, max_depth, int(accumulate), pix, n, _fp(acc),
                            _fp(alb), _fp(nrm), _fp(tst), threads, C.byref(st))
        return {"accum": acc, "albedo": alb, "normal": nrm, "test": tst,
                "stats": {k: getattr(st, k) for k, _ in OracleStats._fields_}}

    def camera_ray(self, pixel, seed):
        out = np.zeros(6, np.float32)
        lib().oracle_camera_ray(self._h, pixel, seed, _fp(out))
        return out

    def use_bvh4(self, nodes, records, root_link):
        """Traverse the engine's own BVH4 arrays (uint8 (n, 64) nodes, float32 (m, 12)
        world records, root link; pupil_pt_export_bvh4) instead of the oracle's BVH."""
        nodes = np.ascontiguousarray(nodes, np.uint8).reshape(-1, 64)
        records = np.ascontiguousarray(records, np.float32).reshape(-1, 12)
        rc = lib().oracle_set_bvh4(self._h, len(nodes), nodes.ctypes.data_as(C.c_void_p), len(records),
                                   _fp(records), int(root_link))
        if rc != 0:
            raise ValueError("engine BVH4 arrays do not match this scene")

    def closest(self, rays, brute_force=False):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        out = np.zeros((len(rays), 4), np.float32)
        lib().oracle_closest(self._h, len(rays), _fp(rays), _fp(out), int(brute_force))
        return out

    def bsdf(self, material, wo, wi_eval, seed, uv=(0.5, 0.5)):
        out = np.zeros(12, np.float32)
        wo = np.ascontiguousarray(wo, np.float32)
        wi = np.ascontiguousarray(wi_eval, np.float32)
        lib().oracle_bsdf(self._h, material, uv[0], uv[1], _fp(wo), _fp(wi), seed, _fp(out))
        return out

    def emitter_sample(self, emitter, pos, nrm, xi):
        """One SampleDirect of area emitter `emitter` from (pos, nrm): wi(3), pdf, distance, radiance(3)."""
        out = np.zeros(8, np.float32)
        p = np.ascontiguousarray(pos, np.float32)
        n = np.ascontiguousarray(nrm, np.float32)
        if lib().oracle_emitter_sample(self._h, emitter, _fp(p), _fp(n), float(xi[0]), float(xi[1]), _fp(out)) != 0:
            raise ValueError("no such emitter")
        return out

    @property
    def num_prims(self):
        return lib().oracle_num_prims(self._h)


def math_probe(x, y2):
    x = np.ascontiguousarray(x, np.float32)
    y2 = np.ascontiguousarray(y2, np.float32)
    out = np.zeros((len(x), 6), np.float32)
    lib().oracle_math(len(x), _fp(x), _fp(y2), _fp(out))
    return out


def rng_sequence(pixel, seed, n):
    out = np.zeros(n, np.float32)
    states = np.zeros(n, np.uint32)
    lib().oracle_rng_sequence(pixel, seed, n, _fp(out), states.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out, states
