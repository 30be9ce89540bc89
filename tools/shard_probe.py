"""Strong-scaling probe on ONE GPU: render each rank's tile share of the config-4
frame (tile t -> rank t % N) in turn and report its ms/frame, so the N-GPU
frame time (max over ranks, gather excluded) can be predicted before the
driver's 8-GPU run.

usage: python tools/shard_probe.py [--worlds 1 2 4 8] [--frames 3]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


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
    ap.add_argument("--only-rank", type=int, default=-1,
                    help="render only this rank's share (a kernel trace of one rank's cadence)")
    args = ap.parse_args()
    import torch

    from pupiloptixlab_amd import scenes
    from pupiloptixlab_amd.pt_pass import PTPass

    desc = scenes.sphere_field(args.spheres, 1920, 1080, 4, seed=1).desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    s = torch.cuda.current_stream()
    base = None
    for n in args.worlds:
        per_rank = []
        host_ms = []
        for r in (range(n) if args.only_rank < 0 else [args.only_rank]):
            pt.set_tiling(args.tile, r, n)
            pt.mark_dirty()

            def frame():
                if args.onrun:
                    for _ in range(8):
                        pt.render(1, stream=s)
                        s.synchronize()
                else:
                    if not args.progressive:
                        pt.mark_dirty()
                    pt.render(8, stream=s, continues=bool(args.progressive))

            for _ in range(max(1, args.warmup)):
                frame()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            host = 0.0
            for _ in range(args.frames):
                h0 = time.perf_counter()
                frame()
                host += time.perf_counter() - h0
            torch.cuda.synchronize()
            per_rank.append((time.perf_counter() - t0) / args.frames * 1e3)
            host_ms.append(host / args.frames * 1e3)
            if r == 0:  # one more frame with stage events for the stage times
                pt.mark_dirty()
                pt.render(8, collect_stats=2, stream=s)
                torch.cuda.synchronize()
                st = pt.stats()
                stage0 = {"trace_ms": round(st["trace_ms"], 3), "trace_launches": st["trace_launches"],
                          "shade_ms": round(st["shade_ms"], 3),
                          "rays": st["primary_rays"] + st["extension_rays"] + st["shadow_rays"]}
        worst = max(per_rank)
        base = base or worst * 1.0
        print(json.dumps({"world": n, "ms_max": round(worst, 3), "ms_min": round(min(per_rank), 3),
                          "pred_speedup": round(base / worst, 3), "pred_eff": round(base / worst / n, 3),
                          "host_enqueue_ms": round(max(host_ms), 3), "rank0": stage0,
                          "ms_per_rank": [round(x, 3) for x in per_rank]}), flush=True)


if __name__ == "__main__":
    main()
