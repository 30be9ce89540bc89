"""Python handle on the C++ scene/world layer (Pupil::resource::Scene +
Pupil::world::World inside libpupil_pt.so).

Mirrors the reference's world API (framework/world/world.h:26-66):
``World.load_scene(path)`` = World::LoadScene (world.cpp:76-139); the
programmatic ``add_*`` calls build the same ShapeInstance list the XML loader
would (resource/shape.cpp:181-217) for the procedural benchmark scenes.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import abi
from .abi import check, load_library


def _f32(a, n=None):
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))
    if n is not None and arr.size != n:
        raise ValueError(f"expected {n} floats, got {arr.size}")
    return arr


def _ptr(arr, ctype=C.c_float):
    return arr.ctypes.data_as(C.POINTER(ctype)) if arr is not None else None


def identity4():
    return np.eye(4, dtype=np.float32)


def rgb(r, g=None, b=None) -> abi.Texture:
    """util::Texture of type RGB (resource/texture.cpp:19-35)."""
    if g is None:
        g = b = r
    t = abi.Texture()
    t.type = abi.TEX_RGB
    t.c0[:] = (r, g, b)
    t.transform[:] = identity4().reshape(-1)
    return t


def checkerboard(color0, color1, uv_scale=(1.0, 1.0)) -> abi.Texture:
    """Checkerboard texture with a to_uv scale (scene.cpp:167-178, util_loader.cpp:188-194)."""
    t = abi.Texture()
    t.type = abi.TEX_CHECKERBOARD
    t.c0[:] = tuple(color0)
    t.c1[:] = tuple(color1)
    m = identity4()
    m[0, 0], m[1, 1] = uv_scale
    t.transform[:] = m.reshape(-1)
    return t


def _mat(mtype, textures, twosided=False, int_ior=1.0, ext_ior=1.0, nonlinear=False) -> abi.Material:
    m = abi.Material()
    m.type = mtype
    m.twosided = int(twosided)
    m.int_ior = int_ior
    m.ext_ior = ext_ior
    m.nonlinear = int(nonlinear)
    for k, t in enumerate(textures):
        m.tex[k] = t
    for k in range(len(textures), 4):
        m.tex[k] = rgb(0.0)
    return m


# material constructors with the reference loader defaults (resource/material.cpp:26-147)
def diffuse(reflectance=(0.5, 0.5, 0.5), twosided=False):
    return _mat(abi.MAT_DIFFUSE, [_tex(reflectance)], twosided)


def dielectric(int_ior=1.5046, ext_ior=1.000277, specular_reflectance=1.0, specular_transmittance=1.0):
    return _mat(abi.MAT_DIELECTRIC, [_tex(specular_reflectance), _tex(specular_transmittance)], False,
                int_ior, ext_ior)


def rough_dielectric(alpha=0.1, int_ior=1.5046, ext_ior=1.000277, specular_reflectance=1.0,
                     specular_transmittance=1.0):
    return _mat(abi.MAT_ROUGH_DIELECTRIC,
                [_tex(alpha), _tex(specular_reflectance), _tex(specular_transmittance)], False, int_ior, ext_ior)


def conductor(eta=(0.0, 0.0, 0.0), k=(1.0, 1.0, 1.0), specular_reflectance=1.0):
    return _mat(abi.MAT_CONDUCTOR, [_tex(eta), _tex(k), _tex(specular_reflectance)])


def rough_conductor(alpha=0.1, eta=(0.0, 0.0, 0.0), k=(1.0, 1.0, 1.0), specular_reflectance=1.0):
    return _mat(abi.MAT_ROUGH_CONDUCTOR, [_tex(alpha), _tex(eta), _tex(k), _tex(specular_reflectance)])


def plastic(diffuse_reflectance=0.5, specular_reflectance=1.0, int_ior=1.49, ext_ior=1.000277, nonlinear=False):
    return _mat(abi.MAT_PLASTIC, [_tex(diffuse_reflectance), _tex(specular_reflectance)], False, int_ior,
                ext_ior, nonlinear)


def rough_plastic(alpha=0.1, diffuse_reflectance=0.5, specular_reflectance=1.0, int_ior=1.49, ext_ior=1.000277,
                  nonlinear=False):
    return _mat(abi.MAT_ROUGH_PLASTIC, [_tex(alpha), _tex(diffuse_reflectance), _tex(specular_reflectance)],
                False, int_ior, ext_ior, nonlinear)


def twosided(m: abi.Material) -> abi.Material:
    m.twosided = 1
    return m


def _tex(v):
    if isinstance(v, abi.Texture):
        return v
    v = np.atleast_1d(np.asarray(v, dtype=np.float32))
    return rgb(float(v[0])) if v.size == 1 else rgb(float(v[0]), float(v[1]), float(v[2]))


@dataclass
class MeshData:
    positions: np.ndarray
    normals: np.ndarray | None
    texcoords: np.ndarray | None
    indices: np.ndarray


class World:
    """world::World + resource::Scene, owned by the C++ host layer."""

    def __init__(self):
        self._lib = load_library()
        h = C.c_void_p()
        check(self._lib.pupil_world_create(C.byref(h)))
        self._h = h
        self._keep = []  # numpy arrays referenced by the C++ side until get_desc copies them
        self._desc = None

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pupil_world_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def load_scene(self, path: str):
        check(self._lib.pupil_world_load_xml(self._h, str(path).encode()))
        self._desc = None
        return self

    def set_film(self, width: int, height: int, max_depth: int):
        check(self._lib.pupil_world_set_film(self._h, width, height, max_depth))

    def set_sensor(self, fov: float, to_world, fov_axis="x", near_clip=0.01, far_clip=10000.0):
        """Perspective sensor; ``to_world`` is a mitsuba-convention 4x4 (row-major)."""
        m = _f32(to_world, 16)
        check(self._lib.pupil_world_set_sensor(self._h, fov, fov_axis.encode(), near_clip, far_clip, _ptr(m)))

    def add_mesh(self, positions, indices, normals=None, texcoords=None) -> int:
        p = _f32(positions)
        i = np.ascontiguousarray(np.asarray(indices, dtype=np.uint32).reshape(-1))
        n = _f32(normals) if normals is not None else None
        t = _f32(texcoords) if texcoords is not None else None
        nv, nf = p.size // 3, i.size // 3
        out = C.c_uint32()
        check(self._lib.pupil_world_add_mesh(self._h, nv, nf, _ptr(p), _ptr(n), _ptr(t), _ptr(i, C.c_uint32),
                                             C.byref(out)))
        return out.value

    def add_builtin(self, name: str) -> int:
        out = C.c_uint32()
        check(self._lib.pupil_world_add_builtin_shape(self._h, name.encode(), C.byref(out)))
        return out.value

    def add_material(self, m: abi.Material) -> int:
        out = C.c_uint32()
        check(self._lib.pupil_world_add_material(self._h, C.byref(m), C.byref(out)))
        return out.value

    def add_instance(self, shape: int, material: int, to_world=None, flip_normals=False, flip_tex_coords=False,
                     emitter_radiance=None) -> int:
        m = _f32(identity4() if to_world is None else to_world, 16)
        rad = _tex(emitter_radiance) if emitter_radiance is not None else None
        out = C.c_uint32()
        check(self._lib.pupil_world_add_instance(self._h, shape, material, _ptr(m), int(flip_normals),
                                                 int(flip_tex_coords), int(rad is not None),
                                                 C.byref(rad) if rad is not None else None, C.byref(out)))
        self._desc = None
        return out.value

    def set_instance_transform(self, instance: int, to_world):
        """Move instance `instance` (index into desc().instances); the next desc()
        carries the new matrices and area emitters (world/world.cpp:45-54)."""
        m = _f32(to_world, 16)
        check(self._lib.pupil_world_set_instance_transform(self._h, int(instance), _ptr(m)))
        self._desc = None

    def add_const_env(self, radiance):
        r = _f32(radiance, 3)
        check(self._lib.pupil_world_add_const_env(self._h, _ptr(r)))

    def desc(self) -> abi.SceneDesc:
        """Flattened scene (pointers owned by the world; valid until it changes)."""
        d = abi.SceneDesc()
        check(self._lib.pupil_world_get_desc(self._h, C.byref(d)))
        d._owner = self  # the arrays live in this world: keep it alive with the desc
        self._desc = d
        return d


def transform(scale=(1.0, 1.0, 1.0), rotate=None, translate=(0.0, 0.0, 0.0)):
    """Transform::Scale -> Rotate -> Translate, each left-multiplied (util_loader.cpp:182-198)."""
    m = np.diag([scale[0], scale[1], scale[2], 1.0]).astype(np.float64)
    if rotate is not None:
        axis, angle = rotate
        u = np.asarray(axis, dtype=np.float64)
        u = u / np.linalg.norm(u)
        th = np.deg2rad(angle)
        a, (b, c, d) = np.cos(0.5 * th), np.sin(0.5 * th) * u
        r = np.array([[1 - 2 * c * c - 2 * d * d, 2 * b * c - 2 * a * d, 2 * a * c + 2 * b * d, 0],
                      [2 * b * c + 2 * a * d, 1 - 2 * b * b - 2 * d * d, 2 * c * d - 2 * a * b, 0],
                      [2 * b * d - 2 * a * c, 2 * a * b + 2 * c * d, 1 - 2 * b * b - 2 * c * c, 0],
                      [0, 0, 0, 1]])
        m = r @ m
    t = np.eye(4)
    t[:3, 3] = translate
    return (t @ m).astype(np.float32)


def look_at_mitsuba(origin, target, up):
    """Mitsuba look-at to_world (+X left, +Z view) as a 4x4, for set_sensor()."""
    o, t, u = (np.asarray(v, dtype=np.float64) for v in (origin, target, up))
    f = t - o
    f /= np.linalg.norm(f)
    left = np.cross(u, f)
    left /= np.linalg.norm(left)
    nu = np.cross(f, left)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = left, nu, f, o
    return m.astype(np.float32)
