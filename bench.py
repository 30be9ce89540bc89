"""bench.py — headline benchmark (BASELINE.json metric, config 4).

One step = one frame: 1920x1080 x 8 spp x max_depth 4 over the synthetic
1M-triangle sphere field, rendered by the HIP wavefront path tracer (exactly
8 x PTPass::OnRun of the reference), i.e. BVH traversal + shading of every
primary, extension and shadow ray.  The BVH build is done once before the
timed region (reported separately as build_ms, like the reference's
GAS/IAS build in PTPass::SetScene).

Multi-GPU (torchrun, one process per GPU): image tiles (32x32) are dealt
round-robin over ranks (tile t -> rank t % N), each rank renders its tiles,
and per frame the compact tile radiance is gathered to rank 0 over RCCL and
scattered into the full image.  Total work is fixed -> "scaling": "strong".

value = Mrays/s over the whole job = (primary + extension + shadow rays of
all ranks) / (max over ranks of the frame time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, choices=(3, 4, 5),
                    help="BASELINE.json configs[k-1]: 3 = 250k-tri field, 4 = 1M-tri field (headline), "
                         "5 = 40 x 250k-tri instanced rough dielectric/plastic field, 3840x2160 16 spp D6")
    ap.add_argument("--spheres", type=int, default=None, help="spheres in the field (configs 3/4) or per BLAS (5)")
    ap.add_argument("--instances", type=int, default=40, help="config 5 instances")
    ap.add_argument("--emissive-groups", type=int, default=0,
                    help="configs 3/4: make that many of the 8 sphere groups emissive (one area emitter per "
                         "triangle; an emissive-mesh workload for NEE emitter selection)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--max-depth", type=int, default=None)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 (N=1 only)")
    ap.add_argument("--cpu-sample-stride", type=int, default=None,
                    help="CPU baseline renders every k-th pixel (default: full frame for configs 3/4, 1/16 for 5)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every CPU this process may run on, capped by the cgroup quota)")
    ap.add_argument("--dropin", type=int, default=1,
                    help="also time the C++ drop-in cadence (build/pupil_path_tracer: spp x PTPass::OnRun of 1 spp, "
                         "each synchronised) on the same scene exported as XML + OBJ (rank 0, N=1, configs 3/4)")
    ap.add_argument("--save", default="", help="write the frame as PNG (rank 0)")
    ap.add_argument("--dump", default="", help="write the full float32 frame as .npy (rank 0, after the timed steps)")
    args = ap.parse_args()
    defaults = {3: (125, 1920, 1080, 8, 4, 1), 4: (500, 1920, 1080, 8, 4, 1), 5: (125, 3840, 2160, 16, 6, 16)}
    sph, w, h, spp, depth, stride = defaults[args.config]
    args.spheres = sph if args.spheres is None else args.spheres
    args.width = w if args.width is None else args.width
    args.height = h if args.height is None else args.height
    args.spp = spp if args.spp is None else args.spp
    args.max_depth = depth if args.max_depth is None else args.max_depth
    args.cpu_sample_stride = stride if args.cpu_sample_stride is None else args.cpu_sample_stride
    return args


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank path on a box with fewer GPUs: PUPIL_BENCH_DEVICES=k maps
    # local rank r to GPU r % k (never set by the driver's runs: one rank per GPU)
    if os.environ.get("PUPIL_BENCH_DEVICES"):
        local_rank %= max(1, int(os.environ["PUPIL_BENCH_DEVICES"]))
    backend = os.environ.get("PUPIL_BENCH_BACKEND", "nccl")  # gloo: rehearsal with several ranks per GPU
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local_rank)
    dev = torch.device(f"cuda:{local_rank}")

    from pupiloptixlab_amd import scenes
    from pupiloptixlab_amd.pt_pass import PTPass, FINAL_RESULT

    if args.config == 5:
        # BASELINE config 5 names a two-level BVH (IAS -> GAS): the engine's world-mode
        # two-level structure (PUPIL_ACCEL=flat for the flattened BVH, A/B)
        os.environ.setdefault("PUPIL_ACCEL", "two_level")
        scene = scenes.instanced_field(args.instances, args.width, args.height, args.max_depth, seed=2,
                                       spheres_per_blas=args.spheres)
    else:
        scene = scenes.sphere_field(args.spheres, args.width, args.height, args.max_depth, seed=1,
                                    emissive_groups=args.emissive_groups)
    desc = scene.desc()
    n_prims = tris = 0
    for i in range(desc.num_instances):
        s = desc.shapes[desc.instances[i].shape]
        n_prims += 1 if s.kind == 1 else s.num_faces
        tris += 0 if s.kind == 1 else s.num_faces

    pt = PTPass(device=local_rank)
    pt.set_scene(desc)
    if world > 1:
        pt.set_tiling(args.tile, rank, world)
    n_local = pt.local_pixel_count() if world > 1 else args.width * args.height
    stream = torch.cuda.current_stream(dev)

    # gather plumbing (rank 0 assembles the frame)
    gather = None
    if world > 1:
        from pupiloptixlab_amd.dist import FrameGather

        gather = FrameGather(args.width, args.height, args.tile, rank, world, dev)
        assert gather.n_local == n_local

    handles = []

    def frame():
        # each step renders the next spp samples of a progressive render (seeds advance
        # by spp, accumulating), as consecutive batches of PTPass::OnRun do; the hint
        # lets the engine trace the next step's camera rays in this step's last launch
        pt.render(args.spp, stream=stream, continues=True)
        if gather is not None:  # overlapped with the next frame on a side stream (dist.FrameGather)
            handles.append(gather.gather_async(pt.buffers.get(FINAL_RESULT), stream))

    # one instrumented frame for the traversal byte counts (untimed)
    pt.mark_dirty()
    pt.render(args.spp, collect_stats=1, stream=stream)
    torch.cuda.synchronize(dev)
    st_bytes = pt.stats()

    pt.mark_dirty()  # the progressive render starts at seed 0
    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize(dev)
    seed_t0 = pt.random_seed  # the timed steps render seeds seed_t0 + k * spp

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    # Frames are enqueued back to back (no host sync inside the timed region).  Each
    # step traces exactly one frame of rays: its camera rays were traced in the previous
    # step's last launch, and the last step traces those of the step after it; the rays
    # of the timed frames are counted exactly afterwards by re-rendering them.
    for _ in range(args.steps):
        frame()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # the last timed frame as rank 0 assembles it (--dump / --save)
    last_frame = None
    if rank == 0 and (args.dump or args.save):
        last_frame = handles[-1].synchronize() if gather is not None else pt.buffers.get(FINAL_RESULT).clone()
    # exact ray count of the timed frames: each re-rendered (untimed) at its seed; every
    # render logs its per-bounce ray counts (the flags partition), no counter kernels needed
    rays_local = 0
    for k in range(args.steps):
        pt.dirty = False
        pt.random_seed, pt.sample_cnt = seed_t0 + k * args.spp, 0
        pt.render(args.spp, stream=stream)
        torch.cuda.synchronize(dev)
        c = pt.stats()
        rays_local += c["primary_rays"] + c["extension_rays"] + c["shadow_rays"]
    # one more frame, untimed, with HIP events around every stage launch (the timed
    # frames record none: each event adds ~6 us of stream gap) for the stage times
    pt.mark_dirty()
    pt.render(args.spp, collect_stats=2, stream=stream)
    torch.cuda.synchronize(dev)
    st = pt.stats()
    rays_frame = st["primary_rays"] + st["extension_rays"] + st["shadow_rays"]
    assert rays_frame == st_bytes["primary_rays"] + st_bytes["extension_rays"] + st_bytes["shadow_rays"]
    ext_ms, trace_ms, shade_ms = st["extend_ms"], st["trace_ms"], st["shade_ms"]
    trace_launches = st["trace_launches"]

    t = torch.tensor([elapsed, float(rays_local), trace_ms], dtype=torch.float64,
                     device=dev if backend == "nccl" else "cpu")
    if world > 1:
        t_max = t.clone()
        dist.all_reduce(t_max[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:2], op=dist.ReduceOp.SUM)
        elapsed = float(t_max[0].item())
        rays_total = float(t[1].item())
    else:
        rays_total = float(rays_local)

    ms_per_step = elapsed / args.steps * 1e3
    mrays = rays_total / elapsed / 1e6
    rays_frame_local = st_bytes["primary_rays"] + st_bytes["extension_rays"] + st_bytes["shadow_rays"]
    # roofline of the dominant kernel, the persistent BVH4 traversal k_trace4 (per
    # frame: the primary extend launch, then one launch per bounce over the
    # concatenated extension + shadow lists).  Three ceilings are evaluated and the
    # binding (highest) one is reported: dependent node gathers (live node-visit
    # rate / the gather ceiling measured on this box by build/ubench_gather), VALU
    # issue and HBM bytes (both from the committed PMC passes of this config).
    roof = roofline(args, st_bytes, trace_ms, trace_launches) if rank == 0 else None
    update = None
    if args.config == 5 and rank == 0:  # RenderInstanceUpdate cost: move instance 0, re-sync the accel
        from pupiloptixlab_amd import world as W

        t0 = time.perf_counter()
        scene.set_instance_transform(0, W.transform(translate=(0.25, 0.0, 0.0)) @
                                     np.asarray(scene.desc().instances[0].to_world[:] + [0, 0, 0, 1],
                                                np.float32).reshape(4, 4))
        pt.update_instance(scene, 0)
        torch.cuda.synchronize(dev)
        update = {"host_ms": round((time.perf_counter() - t0) * 1e3, 3), "engine_ms": round(pt.stats()["build_ms"], 3)}

    dropin = None
    if rank == 0 and world == 1 and args.dropin and args.config in (3, 4) and args.emissive_groups == 0:
        dropin = dropin_cadence(args, ms_per_step, mrays)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline and args.emissive_groups == 0:
        cpu = cpu_baseline(desc, args, pt)

    if rank == 0:
        if args.dump:
            np.save(args.dump, last_frame.cpu().numpy())
        if args.save:
            from tools import imgio

            img = last_frame.cpu().numpy()
            imgio.save_render(args.save, img.reshape(args.height, args.width, 4))
        out = {
            "metric": "Mrays/sec + ms/frame, 1M-tri scene @1920x1080 8spp; 1/2/4/8-GPU scaling",
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (40 instances of a procedural 250k-tri sphere-field BLAS, PCG64 seed 2)"
                     if args.config == 5 else "synthetic (procedural sphere field, PCG64 seed 1)"),
            "config": {"workload": (f"config{args.config}: {n_prims:,}-primitive "
                                    f"{'instanced field' if args.config == 5 else 'sphere field'} ({tris:,} tris), "
                                    f"{args.width}x{args.height}, {args.spp} spp, max_depth {args.max_depth}"),
                       "frame": f"{args.spp} x PTPass::OnRun, progressive (step k renders seeds "
                                f"{args.spp}k..{args.spp}k+{args.spp - 1} of one accumulating render; each step's camera "
                                "rays ride in the previous step's last launch, PUPIL_HINT_CONTINUE; rays counted "
                                "exactly per timed frame)",
                       "parallelism": f"tiles{args.tile}x{world}",
                       "area_emitters": int(desc.num_area_emitters),
                       "accel": "two_level" if st_bytes["two_level"] else "flat",
                       "emitter_select": os.environ.get("PUPIL_EMITTER_SELECT", "guide"),
                       "rays_per_frame": rays_total / args.steps,
                       # shadow rays the reference would trace (one per loop iteration past RR,
                       # main.cu:119-123); the engine and the oracle trace one only when the
                       # contribution is non-zero (radiance-equivalent: Eval draws no random
                       # numbers, optix_material.h:57-62), so value counts traced rays only
                       "shadow_rays_traced": int(st_bytes["shadow_rays"]),
                       "shadow_rays_reference_count": int(st_bytes["shadow_rays_reference"]),
                       "rays_per_frame_reference_count": int(st_bytes["primary_rays"] + st_bytes["extension_rays"] +
                                                             st_bytes["shadow_rays_reference"]),
                       "path_samples_per_s": round(args.width * args.height * args.spp / (ms_per_step * 1e-3), 1),
                       "bvh_build_ms": round(st_bytes["build_ms"], 3),
                       "bvh_nodes": int(st_bytes["bvh_nodes"]),
                       "avg_node_visits_per_ray": round(st_bytes["node_visits"] / max(1, rays_frame_local), 2),
                       "avg_prim_tests_per_ray": round(st_bytes["prim_tests"] / max(1, rays_frame_local), 2),
                       "extend_rays_nodes_prims": [
                           int(st_bytes["primary_rays"] + st_bytes["extension_rays"]),
                           round(st_bytes["extend_node_visits"] / max(1, st_bytes["primary_rays"] + st_bytes["extension_rays"]), 2),
                           round(st_bytes["extend_prim_tests"] / max(1, st_bytes["primary_rays"] + st_bytes["extension_rays"]), 2)],
                       "shadow_rays_nodes_prims": [
                           int(st_bytes["shadow_rays"]),
                           round((st_bytes["node_visits"] - st_bytes["extend_node_visits"]) / max(1, st_bytes["shadow_rays"]), 2),
                           round((st_bytes["prim_tests"] - st_bytes["extend_prim_tests"]) / max(1, st_bytes["shadow_rays"]), 2)],
                       "stage_ms_per_frame": {"primary_extend": round(ext_ms, 3),
                                              "bounce_trace": round(trace_ms - ext_ms, 3),
                                              "shade": round(shade_ms, 3)}},
            "dropin_cpp": dropin,
            "instance_update_ms": update,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dropin_cadence(args, batched_ms, batched_mrays):
    """The reference's cadence through the C++ drop-in: examples/path_tracer (System +
    PTPass, pt_pass.cpp:39-57: one 1-spp launch per OnRun, then a stream sync) on
    this scene exported as XML + OBJ (scenes.XmlWorld; loads bit-identically)."""
    import subprocess
    import tempfile

    from pupiloptixlab_amd import scenes

    exe = os.path.join(HERE, "build", "pupil_path_tracer")
    if not os.path.exists(exe):
        return {"error": "build/pupil_path_tracer not built"}
    with tempfile.TemporaryDirectory() as tmp:
        xw = scenes.XmlWorld()
        scenes.sphere_field(args.spheres, args.width, args.height, args.max_depth, seed=1, world=xw)
        path = xw.save(os.path.join(tmp, f"config{args.config}.xml"))
        env = dict(os.environ, PUPIL_BENCH=f"2,{max(3, args.steps)},{args.spp}")
        try:
            r = subprocess.run([exe, path], capture_output=True, text=True, timeout=600, env=env)
            rec = json.loads(r.stdout.strip().splitlines()[-1])
        except (OSError, ValueError, IndexError, subprocess.SubprocessError) as e:
            return {"error": f"{type(e).__name__}: {e}"}
    rec["vs_batched_ms"] = round(rec["ms_per_frame"] / batched_ms, 3) if batched_ms > 0 else None
    rec["what"] = (f"{args.spp} x C++ PTPass::OnRun (1 spp + hipStreamSynchronize each) per frame, "
                   "examples/path_tracer on the exported XML; value/ms_per_step above batch the frame's spp "
                   "in one launch sequence")
    return rec


def default_config(args):
    defaults = {3: (125, 1920, 1080, 8, 4), 4: (500, 1920, 1080, 8, 4), 5: (125, 3840, 2160, 16, 6)}
    return (args.spheres, args.width, args.height, args.spp, args.max_depth) == defaults[args.config] and \
        args.emissive_groups == 0


def pmc_record(args):
    """Per-launch PMC figures of k_trace4 for this config (tools/gpu_pmc.sh ->
    tools/pmc_summary.py --json, committed as profiles/pmc_config<k>.json): HBM
    bytes (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md), VALU instructions and GRBM cycles.  None when absent or
    when this run is not the default configuration the passes were taken on."""
    path = os.path.join(HERE, "profiles", f"pmc_config{args.config}.json")
    if not default_config(args) or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def gather_ceiling(bvh_nodes):
    """Dependent random 64-B gather ceiling of this GPU (G fetches/s), measured now by
    build/ubench_gather on a table of 2^floor(log2(bvh_nodes)) nodes (no larger
    than the scene's node array, so the ceiling is not understated)."""
    import subprocess

    exe = os.path.join(HERE, "build", "ubench_gather")
    if not os.path.exists(exe):
        return None
    log2 = max(12, int(np.floor(np.log2(max(2, bvh_nodes)))))
    try:
        r = subprocess.run([exe, str(log2), "--json"], capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except (OSError, ValueError, IndexError, subprocess.SubprocessError):
        return None


def roofline(args, st_bytes, trace_ms, trace_launches):
    # the counter frame records no stage events; its traversal launches are the timing frame's
    launches = max(1, trace_launches)
    ms = trace_ms / launches  # HIP events on the render stream, the extra timing frame
    sec = ms * 1e-3
    visits = st_bytes["node_visits"] / launches
    # lanes of a wave on the same node share one fetch: the distinct fetches per wave step are
    # the gathers the memory system serves, the quantity the random-gather ceiling measures
    nodes = (st_bytes.get("unique_node_fetches") or st_bytes["node_visits"]) / launches
    alg_bytes = st_bytes["trace_bytes"] / launches
    kernel = ("k_trace4 (persistent BVH4 traversal, all launches of a frame: primary extend + "
              "per-bounce extension+shadow)")
    cands = {}
    ceil = gather_ceiling(int(st_bytes["bvh_nodes"]))
    if ceil and sec > 0:
        cands["node-gather"] = {"achieved": nodes / sec / 1e9, "peak": ceil["ceiling_gnodes_per_s"],
                                "unit": "Gnode/s",
                                "how": "distinct node fetches per wave step, per launch (counter frame) / HIP-event "
                                       "launch time; peak = build/ubench_gather dependent random 64-B gathers, "
                                       f"{ceil['table_mb']:.0f} MB table (the BVH's size), best waves/SIMD, measured in "
                                       "this run",
                                "node_visits_per_launch": round(visits, 1),
                                "distinct_fetches_per_launch": round(nodes, 1),
                                "ceiling_per_waves_per_simd": ceil.get("per_waves_per_simd")}
    pmc = pmc_record(args)
    traffic = None
    if pmc and sec > 0:
        traffic = pmc["traffic_bytes_per_launch"]
        cands["hbm"] = {"achieved": traffic / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "how": "PMC 2 x FETCH_SIZE + WRITE_SIZE per launch (profiles/pmc_config%d.json, %s) / "
                               "HIP-event launch time" % (args.config, pmc.get("round", "?"))}
        if pmc.get("valu_insts_per_launch") and pmc.get("clock_ghz"):
            simds = 1024  # 256 CUs x 4 SIMD
            # wave64 VALU op = 2 issue cycles on a SIMD-32 (MI355X_MICROARCH.md)
            need = 2.0 * pmc["valu_insts_per_launch"]
            have = simds * pmc["clock_ghz"] * 1e9 * sec
            cands["valu-issue"] = {"achieved": need / sec / 1e9, "peak": simds * pmc["clock_ghz"], "unit": "G SIMD-cycles/s",
                                   "how": "PMC SQ_INSTS_VALU x 2 cycles (wave64 on SIMD-32) per launch over 1024 SIMDs at "
                                          "the GRBM-measured clock"}
    for c in cands.values():
        c["frac"] = round(c["achieved"] / c["peak"], 4)
        c["achieved"] = round(c["achieved"], 2)
    out = {"kernel": kernel, "ms_per_launch": round(ms, 4), "traffic": round(traffic, 1) if traffic else None,
           # SURVEY.md §8(d) algorithmic bytes (32 B ray + 16 B hit + 64 B/node + 48 B/primitive): the BVH
           # is cache-resident (L2 + Infinity Cache), so these exceed what HBM delivers; not a fraction of HBM
           "algorithmic": {"bytes_per_launch": round(alg_bytes, 1),
                           "gbs": round(alg_bytes / sec / 1e9, 1) if sec > 0 else None},
           "ceilings": cands}
    if cands:
        bound = max(cands, key=lambda k: cands[k]["frac"])
        b = cands[bound]
        out.update({"bound": bound, "achieved": b["achieved"], "peak": round(b["peak"], 2), "unit": b["unit"],
                    "frac": b["frac"]})
    else:
        out.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None})
    keys = ["bound", "achieved", "peak", "unit", "frac", "traffic"]
    return {**{k: out[k] for k in keys}, **{k: v for k, v in out.items() if k not in keys}}


def usable_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                n = min(n, max(1, int(np.ceil(int(quota) / int(period)))))
        except (OSError, ValueError):
            pass
    return n


def native_oracle():
    """Build the oracle for THIS host (-O3 -march=native, same -ffp-contract=off, no
    fast-math) into a scratch directory; None when no compiler is available."""
    import subprocess
    import tempfile

    src = os.path.join(HERE, "oracle", "pt_oracle.cpp")
    out = os.path.join(tempfile.gettempdir(), f"pupil_oracle_native_{os.getuid()}", "liboracle.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-march=native", "-ffp-contract=off", "-fno-fast-math", "-pthread",
           "-shared", "-I", os.path.join(HERE, "include"), "-o", out, src]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=300)
        return out
    except (OSError, subprocess.SubprocessError):
        return None


def cpu_baseline(desc, args, pt):
    """The CPU oracle (scalar C++ restatement of the same integrator, traversing the
    engine's own BVH4 arrays) on a bounded sample of the same frame: every k-th
    pixel, all spp, on every usable host CPU, timed with steady_clock.  The sampled
    pixels are also compared with the GPU frame just rendered (bit-exact expected)."""
    native = native_oracle()
    if native:
        os.environ["PUPIL_ORACLE_LIB"] = native
    try:
        import oracle
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}
    import platform

    threads = args.cpu_threads or usable_cpus()
    osc = oracle.OracleScene(desc)
    exported = pt.export_bvh4()  # the CPU traverses the GPU's own BVH arrays
    if exported is not None:
        osc.use_bvh4(*exported)
    npix = args.width * args.height
    pixels = np.arange(0, npix, args.cpu_sample_stride, dtype=np.uint32)
    r = osc.render(spp=args.spp, max_depth=args.max_depth, pixels=pixels, threads=threads)
    s = r["stats"]
    rays = s["primary_rays"] + s["extension_rays"] + s["shadow_rays"]
    gpu = pt.buffers.get("pt accum buffer").cpu().numpy().reshape(npix, 4)[pixels]
    exact = int(np.all(gpu.view(np.uint32) == r["accum"].view(np.uint32), axis=1).sum())
    cpu_model = platform.processor()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    osc.close()
    return {"value": round(rays / s["seconds"] / 1e6, 3), "unit": "Mrays/s", "cores": int(s["threads"]),
            "kind": "port",
            "sample": f"every {args.cpu_sample_stride}th pixel ({len(pixels)} px) x {args.spp} spp of the same frame, "
                      f"{rays} rays in {s['seconds']:.2f}s",
            "cpu": cpu_model, "host_cpus": os.cpu_count(), "usable_cpus": usable_cpus(),
            "build": "g++ -O3 -march=native (built on this host)" if native else "prebuilt -march=x86-64-v2",
            "bvh": ("the engine's own BVH4 arrays (pupil_pt_export_bvh4: the same nodes and records the GPU "
                    "traverses, near-to-far order, the GPU's conservative quantized box test)") if exported is not None
            else "the oracle's own binned-SAH BVH2 (two-level scene: no flattened BVH4 to export)",
            "gpu_pixels_bit_exact": f"{exact}/{len(pixels)}"}


if __name__ == "__main__":
    main()
