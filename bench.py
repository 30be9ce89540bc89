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
SPEC_CLOCK_GHZ = 2.4  # MI355X max engine clock, MI355X_MICROARCH.md chip table

def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=4,
                    help="untimed steps; max_depth of them fill the frame pipeline (one traversal launch per step)")
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
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group, rank 0 prints the ranks seen")
    args = ap.parse_args(argv)
    defaults = {3: (125, 1920, 1080, 8, 4, 1), 4: (500, 1920, 1080, 8, 4, 1), 5: (125, 3840, 2160, 16, 6, 16)}
    sph, w, h, spp, depth, stride = defaults[args.config]
    args.spheres = sph if args.spheres is None else args.spheres
    args.width = w if args.width is None else args.width
    args.height = h if args.height is None else args.height
    args.spp = spp if args.spp is None else args.spp
    args.max_depth = depth if args.max_depth is None else args.max_depth
    args.cpu_sample_stride = stride if args.cpu_sample_stride is None else args.cpu_sample_stride
    return args

def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv=None):
    """`python bench.py --gpus N` without a launcher: start N fresh rank processes of this
    script (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torchrun sets them)
    and return the exit status.  Runs before anything touches the GPU: this process only
    spawns and waits (children are started as new processes, never by an exec of this
    one).  Rank 0 prints the JSON line; a failing rank stops the others."""
    import subprocess

    argv = list(sys.argv[1:] if argv is None else argv)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env["MASTER_PORT"] = str(env.get("PUPIL_BENCH_PORT") or free_port())
    env["WORLD_SIZE"] = env["LOCAL_WORLD_SIZE"] = str(args.gpus)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(args.gpus):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # one rank failed: the group can never complete
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def dry_run(args, world, rank):
    """--dry-run: the rank wiring alone (gloo, no GPU): rank 0 prints the ranks that joined."""
    import torch
    import torch.distributed as dist

    if os.environ.get("PUPIL_BENCH_DRY_FAIL_RANK") == str(rank):  # launcher test: this rank dies
        sys.exit(3)
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.zeros(max(1, world), dtype=torch.int64)
    t[rank] = os.getpid()
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "gpus_requested": args.gpus,
                          "ranks_seen": int((t != 0).sum()), "pids": [int(x) for x in t]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch with --nproc-per-node equal to --gpus)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import torch.distributed as dist

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
        # by spp, accumulating), as consecutive batches of PTPass::OnRun do; the hint lets
        # the engine pipeline frames (engine.hip render_pipelined: the step's one traversal
        # launch also advances the frames of the next steps).  collect_stats=4: HIP events
        # around the traversal launches only, summed over the timed steps
        split = int(os.environ.get("PUPIL_BENCH_SPLIT", "1"))  # A/B: the step's spp as `split` renders
        for _ in range(split):
            pt.render(args.spp // split, stream=stream, continues=True, collect_stats=4)
        if gather is not None:  # overlapped with the next frame on a side stream (dist.FrameGather)
            handles.append(gather.gather_async(pt.buffers.get(FINAL_RESULT), stream))

    # one instrumented frame (untimed, rendered on its own) for the traversal counters:
    # node visits / primitive tests per ray, the algorithmic bytes of SURVEY.md §8(d)
    pt.mark_dirty()
    pt.render(args.spp, collect_stats=1, stream=stream)
    torch.cuda.synchronize(dev)
    st_bytes = pt.stats()
    rays_counter_frame = st_bytes["primary_rays"] + st_bytes["extension_rays"] + st_bytes["shadow_rays"]

    pt.mark_dirty()  # the progressive render starts at seed 0
    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize(dev)
    c0 = pt.stats()  # also restarts the traversal-event sum
    seed_t0 = pt.random_seed

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    # Frames are enqueued back to back (no host sync inside the timed region).
    for _ in range(args.steps):
        frame()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # exact work of the timed steps: the rays their launches traced (device running totals
    # of the flags partitions + the camera rays), whichever frame they belong to
    c1 = pt.stats()
    rays_local = c1["rays_traced_total"] - c0["rays_traced_total"]
    timed = {"trace_ms": c1["trace_ms"], "launches": c1["trace_launches"], "rays": rays_local,
             "frames_in_flight": c1["frames_in_flight"], "pipeline_slots": c1["pipeline_slots"],
             "ring_bytes": c1["ring_bytes"], "ring_budget_bytes": c1["ring_budget_bytes"]}
    # the last timed frame (seeds 0 .. seed_t0 + steps*spp - 1 accumulated), checked below
    last_accum = pt.buffers.get("pt accum buffer").clone() if rank == 0 and world == 1 else None
    last_frame = None
    if rank == 0 and (args.dump or args.save):
        last_frame = handles[-1].synchronize() if gather is not None else pt.buffers.get(FINAL_RESULT).clone()
    # one more frame, untimed, rendered on its own with HIP events around every stage
    # launch (stage times; each event adds ~6 us of stream gap)
    pt.mark_dirty()
    pt.render(args.spp, collect_stats=2, stream=stream)
    torch.cuda.synchronize(dev)
    st = pt.stats()
    rays_frame = st["primary_rays"] + st["extension_rays"] + st["shadow_rays"]
    assert rays_frame == rays_counter_frame
    ext_ms, trace_ms, shade_ms = st["extend_ms"], st["trace_ms"], st["shade_ms"]
    # rays traced by the plain (non-counter) traversal kernels over this process: the
    # denominator of the per-ray PMC figures (tools/pmc_summary.py --json)
    rays_plain_process = st["rays_traced_total"] - rays_counter_frame

    # N > 1: what each rank saw, so a scaling run verifies itself (which rank was slow, that the
    # communicator held N ranks, what the tile gather cost per step on its side stream)
    per_rank, comm = None, None
    if world > 1:
        per_rank, comm = rank_report(elapsed, rays_local, [h.elapsed_ms() for h in handles[-args.steps:]],
                                     dev if backend == "nccl" else "cpu")
    t = torch.tensor([elapsed, float(rays_local)], dtype=torch.float64,
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
    rays_frame_local = rays_counter_frame
    # roofline of the dominant kernel, the persistent BVH4 traversal k_trace4 (pipelined:
    # one launch per step over the shadow + extension rays of every frame in flight and
    # the camera rays of the newest).  Three ceilings are evaluated and the binding
    # (highest) one is reported: dependent node gathers (live node-visit rate / the
    # gather ceiling measured on this box by build/ubench_gather), VALU issue and HBM
    # bytes (per-ray figures of the committed PMC passes of this config, times this
    # rank's rays per launch).  Launch time: HIP events around the timed steps' launches.
    roof = roofline(args, st_bytes, timed) if rank == 0 else None
    dropin = None
    if rank == 0 and world == 1 and args.dropin and args.config in (3, 4) and args.emissive_groups == 0:
        dropin = dropin_cadence(args, ms_per_step, last_accum)

    cpu = None
    timed_check = None
    if rank == 0 and world == 1 and args.cpu_baseline and args.emissive_groups == 0:
        cpu = cpu_baseline(desc, args, pt)
        timed_check = timed_frame_check(desc, args, last_accum, seed_t0 + args.steps * args.spp)

    # RenderInstanceUpdate cost (config 5): move instance 0, re-sync the accel.  Last: the
    # checks above compare the frames rendered before the move with the unmoved scene
    update = None
    if args.config == 5 and rank == 0:
        from pupiloptixlab_amd import world as W

        t0 = time.perf_counter()
        scene.set_instance_transform(0, W.transform(translate=(0.25, 0.0, 0.0)) @
                                     np.asarray(scene.desc().instances[0].to_world[:] + [0, 0, 0, 1],
                                                np.float32).reshape(4, 4))
        pt.update_instance(scene, 0)
        torch.cuda.synchronize(dev)
        update = {"host_ms": round((time.perf_counter() - t0) * 1e3, 3), "engine_ms": round(pt.stats()["build_ms"], 3)}

    if rank == 0:
        assert world == args.gpus, (world, args.gpus)
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
                                f"{args.spp}k..{args.spp}k+{args.spp - 1} of one accumulating render, "
                                "PUPIL_HINT_CONTINUE: frames pipelined, each step's one traversal launch advances "
                                "every frame in flight by a bounce and the step's own frame is complete when it "
                                "returns; value counts exactly the rays the timed steps' launches traced)",
                       "pipeline": {"slots": int(timed["pipeline_slots"]),
                                    "frames_in_flight_after": int(timed["frames_in_flight"]),
                                    "traversal_launches_timed": int(timed["launches"]),
                                    "ring_gb": round(timed["ring_bytes"] / 1e9, 3),
                                    "ring_budget_gb": round(timed["ring_budget_bytes"] / 1e9, 3)},
                       "rays_traced_plain_process": int(rays_plain_process),
                       "parallelism": f"tiles{args.tile}x{world}",
                       "area_emitters": int(desc.num_area_emitters),
                       "accel": "two_level" if st_bytes["two_level"] else "flat",
                       "emitter_select": os.environ.get("PUPIL_EMITTER_SELECT", "guide"),
                       "rays_per_step": rays_total / args.steps,
                       "rays_per_frame_rank0": int(rays_frame_local),
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
            "ranks": per_rank,
            "comm": comm,
            "dropin_cpp": dropin,
            "instance_update_ms": update,
            "roofline": roof,
            "cpu_baseline": cpu,
            "timed_frame_bit_exact": timed_check,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()

def rank_report(elapsed_s, rays_local, gather_ms, device):
    """Every rank's timed-region view, gathered to all ranks (a collective: every rank calls it):
    per-rank elapsed ms, rays traced and mean tile-gather ms per step (side-stream events;
    None without gathers), and the communicator as torch.distributed saw it (backend, world
    size, the RCCL version torch links)."""
    import torch
    import torch.distributed as dist

    g = [x for x in gather_ms if x is not None]
    mine = torch.tensor([elapsed_s * 1e3, float(rays_local), sum(g) / len(g) if g else -1.0], dtype=torch.float64,
                        device=device)
    allr = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(allr, mine)
    per_rank = [{"rank": r, "elapsed_ms": round(v[0], 3), "rays": int(v[1]),
                 "gather_ms_per_step": round(v[2], 4) if v[2] >= 0 else None}
                for r, v in enumerate(x.cpu().tolist() for x in allr)]
    try:
        rccl = ".".join(str(x) for x in torch.cuda.nccl.version())
    except Exception as e:  # noqa: BLE001 - reported, not fatal
        rccl = f"unknown ({type(e).__name__})"
    comm = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "rccl_version": rccl,
            "ranks_reporting": len(per_rank)}
    return per_rank, comm


def dropin_cadence(args, batched_ms, last_accum):
    """The reference's cadence through the C++ drop-in: examples/path_tracer (System +
    PTPass, pt_pass.cpp:39-57: one 1-spp render per OnRun, then a stream sync) on this
    scene exported as XML + OBJ (scenes.XmlWorld; loads bit-identically), as a
    progressive sequence of the same length as the bench's (warmup + steps frames of
    spp OnRuns).  Its final accumulation buffer must equal the bench's last timed frame
    (same seeds) bit for bit."""
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
        accum_path = os.path.join(tmp, "accum.f32")
        env = dict(os.environ, PUPIL_BENCH=f"{args.warmup},{args.steps},{args.spp}", PUPIL_BENCH_ACCUM=accum_path)
        try:
            r = subprocess.run([exe, path], capture_output=True, text=True, timeout=600, env=env)
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            cpp = np.fromfile(accum_path, np.float32).reshape(-1, 4)
        except (OSError, ValueError, IndexError, subprocess.SubprocessError) as e:
            return {"error": f"{type(e).__name__}: {e}"}
    if last_accum is not None:
        gpu = last_accum.cpu().numpy().reshape(-1, 4)
        same = int(np.all(gpu.view(np.uint32) == cpp.view(np.uint32), axis=1).sum()) if gpu.shape == cpp.shape else 0
        rec["bit_exact"] = f"{same}/{len(gpu)}"
    rec["vs_batched_ms"] = round(rec["ms_per_frame"] / batched_ms, 3) if batched_ms > 0 else None
    rec["what"] = (f"{args.spp} x C++ PTPass::OnRun (1 spp + hipStreamSynchronize each) per frame, "
                   f"{args.warmup} + {args.steps} frames of one progressive render, examples/path_tracer on the "
                   "exported XML; bit_exact: its final accumulation vs the bench's last timed frame (same seeds)")
    return rec

def default_config(args):
    defaults = {3: (125, 1920, 1080, 8, 4), 4: (500, 1920, 1080, 8, 4), 5: (125, 3840, 2160, 16, 6)}
    return (args.spheres, args.width, args.height, args.spp, args.max_depth) == defaults[args.config] and \
        args.emissive_groups == 0

def pmc_record(args):
    """Per-ray PMC figures of the plain k_trace4 launches for this config (tools/gpu_pmc.sh
    -> tools/pmc_summary.py --json, committed as profiles/pmc_config<k>.json): HBM bytes
    (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md) and VALU
    instructions per traced ray, and the GRBM clock.  Per ray, so that they apply to any
    launch size: pipelined launches, and one rank's tiles at N > 1.  None when absent or
    when this run is not the scene the passes were taken on."""
    path = os.path.join(HERE, "profiles", f"pmc_config{args.config}.json")
    if not default_config(args) or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    return rec if rec.get("traffic_bytes_per_ray") else None

def gather_ceiling(footprint_bytes):
    """Dependent random 64-B gather ceiling of this GPU (G fetches/s), measured now by
    build/ubench_gather on a table of the next power of two at or above the node array
    (the fetches the node-gather figure counts), so the ceiling is not overstated by a
    table smaller than the real array."""
    import subprocess

    exe = os.path.join(HERE, "build", "ubench_gather")
    if not os.path.exists(exe):
        return None
    log2 = max(12, int(np.ceil(np.log2(max(2.0, footprint_bytes / 64.0)))))
    try:
        r = subprocess.run([exe, str(log2), "--json"], capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except (OSError, ValueError, IndexError, subprocess.SubprocessError):
        return None

def simd_efficiency(st):
    """Lane utilisation of the persistent traversal (counter frame, trace4_body's diagnostics):
    the fraction of a wave's 64 lanes doing useful work per node-loop and leaf-loop iteration,
    and the lanes each refill activates.  What the VALU-issue fraction hides: an issued wave
    instruction with 24 active lanes costs the same 2 cycles as one with 64."""
    if not st.get("node_loop_iters"):
        return None
    return {"node_loop": round(st["node_loop_lanes"] / (64.0 * st["node_loop_iters"]), 4),
            "leaf_loop": round(st["leaf_loop_lanes"] / (64.0 * max(1, st["leaf_loop_iters"])), 4),
            "lanes_per_refill": round(st["refill_lanes"] / max(1, st["refills"]), 2),
            "node_loop_iters": int(st["node_loop_iters"]), "leaf_loop_iters": int(st["leaf_loop_iters"])}

def roofline(args, st_bytes, timed):
    """st_bytes: the counter frame's stats (per-ray node visits, primitive tests, bytes);
    timed: this rank's timed steps -- summed traversal launch time (HIP events on the
    render stream), launches, rays traced."""
    launches = max(1, timed["launches"])
    ms = timed["trace_ms"] / launches
    sec = ms * 1e-3
    rays_cf = max(1, st_bytes["primary_rays"] + st_bytes["extension_rays"] + st_bytes["shadow_rays"])
    rays_launch = timed["rays"] / launches
    per_launch = lambda k: st_bytes[k] / rays_cf * rays_launch  # noqa: E731
    visits = per_launch("node_visits")
    # lanes of a wave on the same node share one fetch: the distinct fetches per wave step are
    # the gathers the memory system serves, the quantity the random-gather ceiling measures
    nodes = per_launch("unique_node_fetches") if st_bytes.get("unique_node_fetches") else visits
    alg_bytes = per_launch("trace_bytes")
    kernel = ("k_trace4 (persistent BVH4 traversal; pipelined frames: one launch per step over the shadow + "
              "extension rays of every frame in flight and the newest frame's camera rays)")
    cands = {}
    footprint = 64.0 * st_bytes["bvh_nodes"]
    ceil = gather_ceiling(footprint)
    if ceil and sec > 0:
        cands["node-gather"] = {"achieved": nodes / sec / 1e9, "peak": ceil["ceiling_gnodes_per_s"],
                                "unit": "Gnode/s",
                                "how": "distinct node fetches per ray (counter frame) x rays per launch / HIP-event "
                                       "launch time; peak = build/ubench_gather dependent uniformly random 64-B gathers "
                                       f"on a {ceil['table_mb']:.0f} MB table (>= the {footprint / 1e6:.0f} MB node array), "
                                       "best waves/SIMD, measured in this run",
                                "node_visits_per_launch": round(visits, 1),
                                "distinct_fetches_per_launch": round(nodes, 1),
                                "ceiling_per_waves_per_simd": ceil.get("per_waves_per_simd")}
    pmc = pmc_record(args)
    traffic = None
    if pmc and sec > 0:
        traffic = pmc["traffic_bytes_per_ray"] * rays_launch
        cands["hbm"] = {"achieved": traffic / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "how": "PMC (2 x FETCH_SIZE + WRITE_SIZE) per traced ray (profiles/pmc_config%d.json, %s) x "
                               "rays per launch / HIP-event launch time" % (args.config, pmc.get("round", "?"))}
        if pmc.get("valu_insts_per_ray") and pmc.get("clock_ghz"):
            simds = 1024  # 256 CUs x 4 SIMD
            # wave64 VALU op = 2 issue cycles on a SIMD-32 (MI355X_MICROARCH.md)
            need = 2.0 * pmc["valu_insts_per_ray"] * rays_launch
            cands["valu-issue"] = {"achieved": need / sec / 1e9, "peak": simds * pmc["clock_ghz"],
                                   "unit": "G SIMD-cycles/s",
                                   "how": "PMC SQ_INSTS_VALU per traced ray x rays per launch x 2 cycles (wave64 on "
                                          "SIMD-32) over 1024 SIMDs at the GRBM-measured clock",
                                   # the same issue rate against the 2.4 GHz spec clock (MI355X_MICROARCH.md)
                                   "frac_at_spec_clock": round(need / sec / 1e9 / (simds * SPEC_CLOCK_GHZ), 4),
                                   "valu_insts_per_ray": round(pmc["valu_insts_per_ray"], 2)}
        if pmc.get("ta_busy_cycles_per_ray") and pmc.get("clock_ghz"):
            # the vector-memory address unit (one TA per CU) processes every VMEM wave-instruction
            # (node and record gathers, ray loads); r05 counters put it at 0.77 busy
            need = pmc["ta_busy_cycles_per_ray"] * rays_launch
            cands["ta-busy"] = {"achieved": need / sec / 1e9, "peak": 256 * pmc["clock_ghz"],
                                "unit": "G TA-cycles/s",
                                "how": "PMC TA_TA_BUSY_sum per traced ray x rays per launch / HIP-event launch time, "
                                       "over 256 TAs (one per CU) at the GRBM-measured clock",
                                "frac_at_spec_clock": round(need / sec / 1e9 / (256 * SPEC_CLOCK_GHZ), 4),
                                "vmem_insts_per_ray": round(pmc.get("vmem_insts_per_ray") or 0.0, 2)}
        if pmc.get("td_busy_cycles_per_ray") and pmc.get("clock_ghz"):
            # the data-return unit (one TD per CU) returns every VMEM wave-instruction's data in
            # order (16 cycles per 16-B-per-lane load) and waits for the L1 on a miss; r06 counters
            # put it at ~0.99 busy, about half of it waiting on L1 misses (TD_TC_STALL)
            need = pmc["td_busy_cycles_per_ray"] * rays_launch
            td = {"achieved": need / sec / 1e9, "peak": 256 * pmc["clock_ghz"], "unit": "G TD-cycles/s",
                  "how": "PMC TD_TD_BUSY_sum per traced ray x rays per launch / HIP-event launch time, over 256 "
                         "TDs (one per CU) at the GRBM-measured clock",
                  "frac_at_spec_clock": round(need / sec / 1e9 / (256 * SPEC_CLOCK_GHZ), 4)}
            if pmc.get("td_tc_stall_cycles_per_ray"):
                td["tc_stall_share"] = round(pmc["td_tc_stall_cycles_per_ray"] / pmc["td_busy_cycles_per_ray"], 4)
            if pmc.get("tcp_accesses_per_ray"):
                td["tcp_accesses_per_ray"] = round(pmc["tcp_accesses_per_ray"], 2)
            if pmc.get("td_busy_frac_under_pmc"):  # busy fraction inside the PMC passes (no live timing)
                td["busy_frac_under_pmc"] = round(pmc["td_busy_frac_under_pmc"], 4)
            if pmc.get("tcp_l2_reads_per_ray") and pmc.get("tcp_accesses_per_ray"):
                td["l1_hit_rate"] = round(1.0 - pmc["tcp_l2_reads_per_ray"] / pmc["tcp_accesses_per_ray"], 4)
            cands["td-busy"] = td
    for c in cands.values():
        c["frac"] = round(c["achieved"] / c["peak"], 4)
        c["achieved"] = round(c["achieved"], 2)
    # a rate above the uniform-random gather rate is no ceiling: the traversal's fetches
    # have locality (hot upper levels in L2, coherent waves) that random gathers lack
    # (config 5's 137 MB node array); such a figure is reported but cannot bind
    binding = {k: v for k, v in cands.items() if v["frac"] <= 1.0 or k != "node-gather"}
    for k, v in cands.items():
        if v["frac"] > 1.0 and k == "node-gather":
            v["note"] = ("above the uniform-random gather rate of a node-array-sized table: the traversal's fetches "
                         "are served with more locality than random gathers; not a ceiling")
    out = {"kernel": kernel, "ms_per_launch": round(ms, 4), "launches": int(launches),
           "simd_efficiency": simd_efficiency(st_bytes),
           "rays_per_launch": round(rays_launch, 1), "traffic": round(traffic, 1) if traffic else None,
           # SURVEY.md §8(d) algorithmic bytes (32 B ray + 16 B hit + 64 B/node + 48 B/primitive): the BVH
           # is cache-resident (L2 + Infinity Cache), so these exceed what HBM delivers; not a fraction of HBM
           "algorithmic": {"bytes_per_launch": round(alg_bytes, 1),
                           "gbs": round(alg_bytes / sec / 1e9, 1) if sec > 0 else None},
           "ceilings": cands}
    if binding:
        bound = max(binding, key=lambda k: binding[k]["frac"])
        b = cands[bound]
        out.update({"bound": bound, "achieved": b["achieved"], "peak": round(b["peak"], 2), "unit": b["unit"],
                    "frac": b["frac"]})
        if "frac_at_spec_clock" in b:
            out["frac_at_spec_clock"] = b["frac_at_spec_clock"]
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

def timed_frame_check(desc, args, last_accum, n_frames):
    """The last timed frame (a progressive render of seeds 0 .. n_frames - 1, most of it
    pipelined) against the oracle rendering the same n_frames OnRuns, on every k-th pixel
    (k = 64 for configs 3/4, 1024 for config 5); bit-exact expected."""
    if last_accum is None:
        return None
    try:
        import oracle
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}
    stride = 1024 if args.config == 5 else 64
    npix = args.width * args.height
    pixels = np.arange(stride // 2, npix, stride, dtype=np.uint32)
    osc = oracle.OracleScene(desc)
    r = osc.render(spp=n_frames, max_depth=args.max_depth, pixels=pixels, threads=args.cpu_threads or usable_cpus())
    osc.close()
    gpu = last_accum.cpu().numpy().reshape(npix, 4)[pixels]
    exact = int(np.all(gpu.view(np.uint32) == r["accum"].view(np.uint32), axis=1).sum())
    return {"pixels": f"every {stride}th pixel from {stride // 2}", "frames": int(n_frames),
            "bit_exact": f"{exact}/{len(pixels)}"}

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
