"""Host-side mirror of the reference's pass API for the path tracer.

Reference surface (the drop-in boundary):
  * ``Pupil::Pass`` (framework/system/pass.h:22-39): ``run()`` times ``on_run()``.
  * ``Pupil::pt::PTPass`` (example/path_tracer/pt_pass.h:21-40,
    pt_pass.cpp:29-237): ``set_scene(world)``, ``on_run()``, the inspector
    knobs ``max_depth`` (clamped 1..128) and ``accumulate``; camera / instance
    events mark it dirty, which resets ``random_seed`` and ``sample_cnt``.
  * ``BufferManager`` (framework/system/buffer.h:44-63): named device buffers
    ("final result", "pt accum buffer", "albedo", "normal", "test").
  * ``System`` (framework/system/system.h:22-41), headless: ``add_pass``,
    ``set_scene``, ``run(frames)``.

The work itself happens in libpupil_pt.so through the C ABI
(include/pupil_pt.h); this module only owns buffers and frame counters.
There is no CPU fallback: without a HIP device ``PTPass`` raises.
"""
from __future__ import annotations

import ctypes as C
import time
from collections import defaultdict

from . import abi
from .abi import check, load_library

FINAL_RESULT = "final result"  # BufferManager::DEFAULT_FINAL_RESULT_BUFFER_NAME


class Events:
    """util::Event dispatcher subset: CameraChange / RenderInstanceUpdate / SceneLoad."""

    CAMERA_CHANGE = "CameraChange"
    RENDER_INSTANCE_UPDATE = "RenderInstanceUpdate"
    SCENE_LOAD = "SceneLoad"

    def __init__(self):
        self._subs = defaultdict(list)

    def bind(self, event, fn):
        self._subs[event].append(fn)

    def dispatch(self, event, payload=None):
        for fn in self._subs[event]:
            fn(payload)


class BufferManager:
    """Named device buffers (float tensors on the pass's device)."""

    def __init__(self, device: str):
        import torch

        self._torch = torch
        self.device = device
        self.buffers = {}

    def alloc(self, name: str, count: int, channels: int):
        t = self._torch.zeros((count, channels), dtype=self._torch.float32, device=self.device)
        self.buffers[name] = t
        return t

    def get(self, name: str):
        return self.buffers[name]


class Pass:
    """Pupil::Pass: run() = timed on_run() (pass.cpp:6-11)."""

    def __init__(self, name: str):
        self.name = name
        self.last_ms = 0.0

    def run(self):
        t0 = time.perf_counter()
        self.on_run()
        self.last_ms = (time.perf_counter() - t0) * 1e3

    def on_run(self):  # pragma: no cover - abstract
        raise NotImplementedError


class PTPass(Pass):
    def __init__(self, name: str = "Path Tracing", device: int = 0, events: Events | None = None):
        super().__init__(name)
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("PTPass needs a HIP device (no CPU fallback)")
        self._torch = torch
        self._lib = load_library()
        self.device_index = device
        self.device = f"cuda:{device}"
        self.buffers = BufferManager(self.device)
        self._pt = C.c_void_p()
        self.width = self.height = 0
        self.scene_max_depth = 1
        self._max_depth = 1
        self._accumulate = True
        self.random_seed = 0
        self.sample_cnt = 0
        self.dirty = True
        self.tile = (32, 0, 1)  # tile_size, rank, world
        self._world = None  # the World the scene came from: its sensor is re-read when dirty
        self._pending = {}  # RenderInstanceUpdate events since the last render: id(world) -> (world, instances)
        self.events = events or Events()
        self.events.bind(Events.CAMERA_CHANGE, lambda _: self.mark_dirty())
        self.events.bind(Events.RENDER_INSTANCE_UPDATE, self._on_instance_update)
        self.events.bind(Events.SCENE_LOAD, lambda w: self.set_scene(w))

    def _on_instance_update(self, arg):
        """RenderInstanceUpdate handler: only records the moved instance and marks the pass
        dirty, like the reference's (pt_pass.cpp:216-218); the next render refits once
        for every instance recorded since the last one (GetIASHandle(2, true), :46)."""
        if arg is not None:
            world, instance = arg
            self._pending.setdefault(id(world), (world, set()))[1].add(int(instance))
        self.mark_dirty()

    def update_instance(self, world, instance: int):
        """RenderInstanceUpdate applied now: push instance `instance`'s new transform from
        `world` (already moved with World.set_instance_transform) into the engine, and the
        emitter table when the instance is emissive; restarts accumulation."""
        self.update_instances(world, [instance])

    def update_instances(self, world, instances):
        """Several moved instances with ONE refit of the acceleration structure
        (pupil_pt_update_instances), then the emitter table if any of them emits."""
        import numpy as np

        ids = sorted({int(i) for i in instances})
        if not ids:
            return
        desc = world.desc()
        tw = np.array([list(desc.instances[i].to_world) for i in ids], np.float32)
        to = np.array([list(desc.instances[i].to_object) for i in ids], np.float32)
        idv = np.array(ids, np.uint32)
        check(self._lib.pupil_pt_update_instances(self._pt, len(ids), idv.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                  tw.ctypes.data_as(C.POINTER(C.c_float)),
                                                  to.ctypes.data_as(C.POINTER(C.c_float))))
        if any(desc.instances[i].emitter_offset >= 0 for i in ids):
            check(self._lib.pupil_pt_update_emitters(self._pt, C.byref(desc)))
        self.dirty = True

    # ---- inspector knobs (pt_pass.cpp:225-237)
    @property
    def max_depth(self):
        return self._max_depth

    @max_depth.setter
    def max_depth(self, v):
        v = max(1, min(128, int(v)))
        if v != self._max_depth:
            self._max_depth = v
            self.dirty = True

    @property
    def accumulate(self):
        return self._accumulate

    @accumulate.setter
    def accumulate(self, v):
        if bool(v) != self._accumulate:
            self._accumulate = bool(v)
            self.dirty = True

    def mark_dirty(self):
        self.dirty = True

    def set_tiling(self, tile_size: int, rank: int, world: int):
        """Render only the image tiles t with t % world == rank (multi-GPU sharding)."""
        self.tile = (tile_size, rank, world)
        self._alloc_buffers()

    def local_pixel_count(self):
        ts, rank, world = self.tile
        n = C.c_uint32(0)
        check(self._lib.pupil_pt_local_pixels(self.width, self.height, ts, rank, world, None, C.byref(n)))
        return n.value

    def local_pixels(self):
        import numpy as np

        ts, rank, world = self.tile
        n = C.c_uint32(self.local_pixel_count())
        out = np.zeros(max(1, n.value), dtype=np.uint32)
        check(self._lib.pupil_pt_local_pixels(self.width, self.height, ts, rank, world,
                                              out.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(n)))
        return out[: n.value]

    # ---- PTPass::SetScene (pt_pass.cpp:107-209)
    def set_scene(self, world):
        desc = world.desc() if hasattr(world, "desc") else world
        self._world = world if hasattr(world, "desc") else None
        self.close_engine()
        self._pending = {}
        self._torch.cuda.set_device(self.device_index)
        check(self._lib.pupil_pt_create(C.byref(desc), self.device_index, C.byref(self._pt)))
        self.width, self.height = desc.width, desc.height
        self.scene_max_depth = desc.max_depth
        self._max_depth = desc.max_depth
        self._accumulate = True
        self.random_seed = 0
        self.sample_cnt = 0
        self.dirty = True
        self._alloc_buffers()

    def _alloc_buffers(self):
        n = self.local_pixel_count() if self.tile[2] > 1 else self.width * self.height
        b = self.buffers
        b.alloc(FINAL_RESULT, n, 4)
        b.alloc("pt accum buffer", n, 4)
        b.alloc("albedo", n, 3)
        b.alloc("normal", n, 3)
        b.alloc("test", n, 1)

    def _frame(self):
        b = self.buffers
        f = abi.Frame()
        f.accum = b.get("pt accum buffer").data_ptr()
        f.frame = b.get(FINAL_RESULT).data_ptr()
        f.albedo = b.get("albedo").data_ptr()
        f.normal = b.get("normal").data_ptr()
        f.test = b.get("test").data_ptr()
        f.compact = 1 if self.tile[2] > 1 else 0
        return f

    def render(self, spp: int = 1, collect_stats: int = 0, stream=None, continues: bool = False):
        """spp consecutive OnRun frames in one wavefront batch (asynchronous).
        collect_stats: bit 0 counters (node visits, ...), bit 1 per-stage HIP events.
        continues: the next render() continues this one (progressive rendering), so the
        engine traces its camera rays ahead (PUPIL_HINT_CONTINUE; single-spp renders
        always do)."""
        if self.dirty:  # pt_pass.cpp:40-49: camera re-uploaded, instances refitted, accumulation restarted
            pending, self._pending = self._pending, {}
            for world, ids in pending.values():
                self.update_instances(world, ids)
            if self._world is not None:
                d = self._world.desc()
                check(self._lib.pupil_pt_set_camera(self._pt, d.sample_to_camera, d.camera_to_world))
            self.random_seed = 0
            self.sample_cnt = 0
            self.dirty = False
        la = abi.Launch()
        la.random_seed = self.random_seed
        la.sample_cnt = self.sample_cnt
        la.spp = spp
        la.max_depth = self._max_depth
        la.accumulate = int(self._accumulate)
        la.tile_size, la.tile_rank, la.tile_world = self.tile
        la.collect_stats = int(collect_stats)
        la.hints = 1 if continues else 0  # PUPIL_HINT_CONTINUE
        s = stream if stream is not None else self._torch.cuda.current_stream(self.device_index)
        f = self._frame()
        check(self._lib.pupil_pt_render(self._pt, C.byref(f), C.byref(la), C.c_void_p(s.cuda_stream)))
        self.random_seed += spp  # pt_pass.cpp:55-56
        if self._accumulate:
            self.sample_cnt += spp

    def on_run(self):
        self.render(1)
        self._torch.cuda.synchronize(self.device_index)  # m_optix_pass->Synchronize()

    def stats(self) -> dict:
        c = abi.Counters()
        check(self._lib.pupil_pt_stats(self._pt, C.byref(c)))
        return c.as_dict()

    def export_bvh4(self):
        """The flattened BVH4 the traversal kernels read: (uint8 (n, 64) nodes, float32 (m, 12)
        world records, root link), or None for the two-level structure / other node formats."""
        import numpy as np

        nn, nr, root = C.c_uint32(0), C.c_uint32(0), C.c_int32(0)
        if self._lib.pupil_pt_export_bvh4(self._pt, C.byref(nn), None, C.byref(nr), None, C.byref(root)) != 0:
            return None
        nodes = np.zeros((max(1, nn.value), 64), np.uint8)
        recs = np.zeros((max(1, nr.value), 12), np.float32)
        check(self._lib.pupil_pt_export_bvh4(self._pt, C.byref(nn), nodes.ctypes.data_as(C.c_void_p), C.byref(nr),
                                             recs.ctypes.data_as(C.POINTER(C.c_float)), C.byref(root)))
        return nodes[: nn.value], recs[: nr.value], root.value

    def image(self, name: str = FINAL_RESULT):
        """Full-frame (h, w, c) numpy image, row 0 = bottom (reference pixel order)."""
        t = self.buffers.get(name).cpu().numpy()
        if self.tile[2] > 1:
            import numpy as np

            full = np.zeros((self.width * self.height, t.shape[1]), dtype=np.float32)
            full[self.local_pixels()] = t
            t = full
        return t.reshape(self.height, self.width, -1)

    def close_engine(self):
        if self._pt:
            self._lib.pupil_pt_destroy(self._pt)
            self._pt = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close_engine()
        except Exception:
            pass


class System:
    """Headless Pupil::System: passes run in order once per frame (system.cpp:81-114)."""

    def __init__(self):
        self.passes = []
        self.events = Events()
        self.world = None

    def add_pass(self, p: Pass):
        self.passes.append(p)
        if isinstance(p, PTPass):
            p.events = self.events
            self.events.bind(Events.CAMERA_CHANGE, lambda _: p.mark_dirty())
            self.events.bind(Events.RENDER_INSTANCE_UPDATE, p._on_instance_update)
            self.events.bind(Events.SCENE_LOAD, lambda w: p.set_scene(w))

    def set_scene(self, world):
        self.world = world
        self.events.dispatch(Events.SCENE_LOAD, world)

    def run(self, frames: int = 1):
        for _ in range(frames):
            for p in self.passes:
                p.run()
