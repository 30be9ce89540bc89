"""Save / load a flattened scene (pupil_scene_desc) as one .npz file.

A desc produced by World (the XML loader of resource/scene.cpp:27-227 and the
world/emitter.cpp tables) is a graph of C structs with pointers; this module
stores every struct's bytes and every array it points to, and rebuilds an
equivalent desc whose arrays are owned by the returned object.  Used for the
committed fixtures of the reference's own scene files (tests/golden/ref_scenes,
made by tests/golden/make_ref_scenes.py) and for resizing a film while keeping
its camera.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


def _raw(struct) -> np.ndarray:
    return np.frombuffer(bytes(struct), dtype=np.uint8).copy()


def _copy(cls, raw: np.ndarray):
    return cls.from_buffer_copy(raw.tobytes())


def _tex_texels(t: abi.Texture):
    if t.type == abi.TEX_BITMAP and t.rgba and t.width and t.height:
        return np.ctypeslib.as_array(t.rgba, shape=(int(t.width) * int(t.height) * 4,)).copy()
    return None


def save_desc(desc: abi.SceneDesc, path: str) -> None:
    out = {"header": _raw(desc)}
    for i in range(desc.num_shapes):
        s = desc.shapes[i]
        out[f"shape{i}"] = _raw(s)
        if s.kind == abi.SHAPE_MESH:
            nv, nf = int(s.num_vertices), int(s.num_faces)
            out[f"shape{i}_pos"] = np.ctypeslib.as_array(s.positions, shape=(3 * nv,)).copy()
            out[f"shape{i}_idx"] = np.ctypeslib.as_array(s.indices, shape=(3 * nf,)).copy()
            if s.normals:
                out[f"shape{i}_nrm"] = np.ctypeslib.as_array(s.normals, shape=(3 * nv,)).copy()
            if s.texcoords:
                out[f"shape{i}_uv"] = np.ctypeslib.as_array(s.texcoords, shape=(2 * nv,)).copy()
    for i in range(desc.num_materials):
        m = desc.materials[i]
        out[f"mat{i}"] = _raw(m)
        for k in range(4):
            tx = _tex_texels(m.tex[k])
            if tx is not None:
                out[f"mat{i}_tex{k}"] = tx
    out["instances"] = np.stack([_raw(desc.instances[i]) for i in range(desc.num_instances)])
    for i in range(desc.num_area_emitters):
        e = desc.area_emitters[i]
        out[f"area{i}"] = _raw(e)
        tx = _tex_texels(e.radiance)
        if tx is not None:
            out[f"area{i}_tex"] = tx
    if desc.env:
        out["env"] = _raw(desc.env[0])
        tx = _tex_texels(desc.env[0].radiance)
        if tx is not None:
            out["env_tex"] = tx
    np.savez_compressed(path, **out)


class LoadedScene:
    """A desc rebuilt from an .npz file; `desc` stays valid while this object lives."""

    def __init__(self, path: str):
        z = np.load(path, allow_pickle=False)
        self._keep = []
        d = _copy(abi.SceneDesc, z["header"])

        def ptr(arr, ctype):
            arr = np.ascontiguousarray(arr)
            self._keep.append(arr)
            return arr.ctypes.data_as(C.POINTER(ctype))

        def fix_tex(t: abi.Texture, key):
            t.rgba = ptr(z[key].astype(np.float32), C.c_float) if key in z.files else None

        shapes = (abi.Shape * max(1, d.num_shapes))()
        for i in range(d.num_shapes):
            s = _copy(abi.Shape, z[f"shape{i}"])
            s.positions = s.normals = s.texcoords = None
            s.indices = None
            if s.kind == abi.SHAPE_MESH:
                s.positions = ptr(z[f"shape{i}_pos"].astype(np.float32), C.c_float)
                s.indices = ptr(z[f"shape{i}_idx"].astype(np.uint32), C.c_uint32)
                if f"shape{i}_nrm" in z.files:
                    s.normals = ptr(z[f"shape{i}_nrm"].astype(np.float32), C.c_float)
                if f"shape{i}_uv" in z.files:
                    s.texcoords = ptr(z[f"shape{i}_uv"].astype(np.float32), C.c_float)
            shapes[i] = s
        mats = (abi.Material * max(1, d.num_materials))()
        for i in range(d.num_materials):
            m = _copy(abi.Material, z[f"mat{i}"])
            for k in range(4):
                fix_tex(m.tex[k], f"mat{i}_tex{k}")
            mats[i] = m
        insts = (abi.Instance * max(1, d.num_instances))()
        for i in range(d.num_instances):
            insts[i] = _copy(abi.Instance, z["instances"][i])
        areas = (abi.Emitter * max(1, d.num_area_emitters))()
        for i in range(d.num_area_emitters):
            e = _copy(abi.Emitter, z[f"area{i}"])
            fix_tex(e.radiance, f"area{i}_tex")
            areas[i] = e
        env = None
        if "env" in z.files:
            env = abi.Emitter.from_buffer_copy(z["env"].tobytes())
            fix_tex(env.radiance, "env_tex")
            self._keep.append(env)
        self._keep += [shapes, mats, insts, areas]
        d.shapes = C.cast(shapes, C.POINTER(abi.Shape))
        d.materials = C.cast(mats, C.POINTER(abi.Material))
        d.instances = C.cast(insts, C.POINTER(abi.Instance))
        d.area_emitters = C.cast(areas, C.POINTER(abi.Emitter)) if d.num_area_emitters else None
        d.env = C.pointer(env) if env is not None else None
        d._owner = self
        self.desc = d

    def resized(self, width: int, height: int) -> abi.SceneDesc:
        """The same scene on a film of another size with the same aspect ratio (the
        sample-to-camera matrix maps film [0,1]^2, so it is unchanged)."""
        d = self.desc
        assert abs(width * d.height - height * d.width) <= max(d.width, d.height), "aspect ratio must be kept"
        r = abi.SceneDesc.from_buffer_copy(bytes(d))
        r.width, r.height = int(width), int(height)
        r._owner = self
        return r
