"""Strong-scaling probe on ONE GPU: render each rank's tile share of the config-4
frame (tile t -> rank t % N) in turn and report its time, so the N-GPU frame time
(max over ranks, gather excluded) can be predicted before the driver's 8-GPU run.

Every window counts the rays its renders traced (the engine's running total, as
bench.py does), so the prediction is a ray rate -- sum of the ranks' rays over the
slowest rank's time -- and not only a time ratio: with frame groups one OnRun in G
carries a whole group's traversal, and a window's time alone could include or miss
part of such a burst.

usage: python tools/shard_probe.py [--worlds 1 2 4 8] [--frames 3] [--onrun 1] [--moving 1]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--spheres", type=int, default=500)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--progressive", type=int, default=0,
                    help="1: every frame continues the previous one (seeds 8k..8k+7, accumulating) with "
                         "PUPIL_HINT_CONTINUE, so frames are pipelined (one traversal launch per frame in the "
                         "steady state), as bench.py renders; 0: every frame re-renders seed 0")
    ap.add_argument("--warmup", type=int, default=4, help="untimed frames per rank (fill the frame pipeline)")
    ap.add_argument("--onrun", type=int, default=0,
                    help="1: the drop-in cadence -- a frame is 8 renders of 1 spp, each followed by a device "
                         "synchronisation (PTPass::OnRun, pt_pass.cpp:51-56), continuing one progressive render")
    ap.add_argument("--moving", type=int, default=0,
                    help="1 (implies --onrun 1): the interactive cadence -- the camera moves before every OnRun "
                         "(a CameraChange, world.cpp:15-43), so every OnRun restarts accumulation and renders a "
                         "fresh 1-spp frame (pt_pass.cpp:40-49) and no frame is started ahead")
    ap.add_argument("--only-rank", type=int, default=-1,
                    help="render only this rank's share (a kernel trace of one rank's cadence)")
    args = ap.parse_args()
    if args.moving:
        args.onrun = 1
    import numpy as np
    import torch

    from pupiloptixlab_amd import abi, scenes
    from pupiloptixlab_amd.pt_pass import PTPass

    desc = scenes.sphere_field(args.spheres, 1920, 1080, 4, seed=1).desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    s = torch.cuda.current_stream()
    c2w0 = np.array(list(desc.camera_to_world), np.float32)
    step = [0]

    def move_camera():
        step[0] += 1
        c2w = c2w0.copy()
        c2w[3] += 1e-4 * step[0]
        abi.check(pt._lib.pupil_pt_set_camera(pt._pt, desc.sample_to_camera, c2w.ctypes.data_as(abi.f32p)))
        pt.dirty = False
        pt.random_seed = pt.sample_cnt = 0

    base = None
    for n in args.worlds:
        per_rank, host_ms, rays_rank, onrun_all = [], [], [], []
        stage0 = None
        for r in (range(n) if args.only_rank < 0 else [args.only_rank]):
            pt.set_tiling(args.tile, r, n)
            pt.mark_dirty()
            onrun_ms = []

            def frame(timed):
                if args.onrun:
                    for _ in range(8):
                        if args.moving:
                            move_camera()
                        t0 = time.perf_counter()
                        pt.render(1, stream=s)
                        s.synchronize()
                        if timed:
                            onrun_ms.append((time.perf_counter() - t0) * 1e3)
                else:
                    if not args.progressive:
                        pt.mark_dirty()
                    pt.render(8, stream=s, continues=bool(args.progressive))

            for _ in range(max(1, args.warmup)):
                frame(False)
            torch.cuda.synchronize()
            r0 = pt.stats()["rays_traced_total"]
            t0 = time.perf_counter()
            host = 0.0
            for _ in range(args.frames):
                h0 = time.perf_counter()
                frame(True)
                host += time.perf_counter() - h0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            rays_rank.append(pt.stats()["rays_traced_total"] - r0)
            per_rank.append(dt / args.frames * 1e3)
            host_ms.append(host / args.frames * 1e3)
            onrun_all.append(onrun_ms)
            if r == 0:  # one more frame with stage events for the stage times
                pt.mark_dirty()
                pt.render(8, collect_stats=2, stream=s)
                torch.cuda.synchronize()
                st = pt.stats()
                stage0 = {"trace_ms": round(st["trace_ms"], 3), "trace_launches": st["trace_launches"],
                          "shade_ms": round(st["shade_ms"], 3),
                          "rays": st["primary_rays"] + st["extension_rays"] + st["shadow_rays"]}
        worst = max(per_rank)
        # the N-rank rate: every rank's rays in the time of the slowest rank's window
        mrays = sum(rays_rank) / (worst * 1e-3 * args.frames) / 1e6
        base = base or mrays
        rec = {"world": n, "ms_max": round(worst, 3), "ms_min": round(min(per_rank), 3),
               "mrays_per_s": round(mrays, 1), "pred_speedup": round(mrays / base, 3),
               "pred_eff": round(mrays / base / n, 3),
               "rays_per_frame": round(sum(rays_rank) / args.frames),
               "host_enqueue_ms": round(max(host_ms), 3), "rank0": stage0,
               "ms_per_rank": [round(x, 3) for x in per_rank]}
        if args.onrun:
            flat = [x for v in onrun_all for x in v]
            rec["onrun_ms"] = {"p50": round(pct(flat, 0.5), 3), "p99": round(pct(flat, 0.99), 3),
                               "max": round(max(flat), 3), "mean": round(sum(flat) / len(flat), 3)}
        rec["mode"] = "moving" if args.moving else ("onrun" if args.onrun else
                                                   ("progressive" if args.progressive else "batched"))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
