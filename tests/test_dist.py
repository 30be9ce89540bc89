"""Tile sharding + per-frame gather on CPU with the gloo backend (world_size 2 and 3).

The GPU path uses the same FrameGather over RCCL; here each rank fills its
compact buffer with a deterministic function of the global pixel index (what
the engine's compact output holds) and rank 0 must reassemble the exact image."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pupiloptixlab_amd.dist import FrameGather, local_pixels


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, tile, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = FrameGather(w, h, tile, rank, world, "cpu")
    pix = local_pixels(w, h, tile, rank, world)
    local = torch.from_numpy(np.stack([pix, pix * 2, pix * 3, np.ones_like(pix)], 1).astype(np.float32))
    full = g.gather(local)
    h = g.gather_async(local)  # CPU tensors: the synchronous path, same result
    assert h.done()
    again = h.synchronize()
    if rank == 0:
        assert torch.equal(full, again)
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h,tile", [(2, 70, 45, 16), (3, 64, 64, 32), (2, 33, 17, 8)])
def test_gather_reassembles_frame(tmp_path, world, w, h, tile):
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), w, h, tile, out), nprocs=world, join=True)
    full = np.load(out)
    idx = np.arange(w * h, dtype=np.float32)
    assert np.array_equal(full[:, 0], idx)
    assert np.array_equal(full[:, 1], idx * 2)
    assert np.array_equal(full[:, 3], np.ones(w * h, np.float32))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_tiles_partition_image_and_balance(world):
    w, h, tile = 1920, 1080, 32
    seen = np.zeros(w * h, np.int32)
    counts = []
    for r in range(world):
        p = local_pixels(w, h, tile, r, world)
        seen[p] += 1
        counts.append(len(p))
    assert (seen == 1).all()
    # interleaved tiles: every rank within 2 tiles of the mean
    assert max(counts) - min(counts) <= 2 * tile * tile


@pytest.mark.gpu
def test_gather_async_on_gpu_single_rank():
    """The overlapped gather's stream/event plumbing over RCCL (one rank): the side
    stream snapshots the tile buffer, the caller's stream may overwrite it at once,
    and the gathered image is the snapshot."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        w, h, tile = 96, 64, 32
        g = FrameGather(w, h, tile, 0, 1, dev)
        s = torch.cuda.current_stream(dev)
        pix = torch.arange(w * h, dtype=torch.float32, device=dev)
        local = torch.stack([pix, 2 * pix, 3 * pix, torch.ones_like(pix)], 1)
        h = g.gather_async(local, s)
        local.fill_(-1.0)  # the next frame overwrites the tile buffer on the render stream
        full = h.wait(s)  # the render stream waits for the scatter before reading the image
        full = full.clone()
        torch.cuda.synchronize(dev)
        assert h.done()
        assert torch.equal(full[:, 1], 2 * pix)
        assert torch.equal(full[:, 3], torch.ones_like(pix))
    finally:
        dist.destroy_process_group()


def _report_worker(rank, world, port, out_path):
    import json
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a real gather per "step" through FrameGather's synchronous (gloo) path, timed by its handle
    g = FrameGather(64, 48, 16, rank, world, "cpu")
    local = torch.zeros((g.n_local, 4), dtype=torch.float32)
    handles = [g.gather_async(local) for _ in range(3)]
    per_rank, comm = bench.rank_report(0.5 + 0.1 * rank, 1000 * (rank + 1), [h.elapsed_ms() for h in handles], "cpu")
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"ranks": per_rank, "comm": comm}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_rank_report_names_every_rank(tmp_path, world):
    """bench.py --gpus N (N > 1) reports each rank's elapsed time, rays and gather time per step
    and the communicator's world size, so a scaling run shows which rank was slow and that the
    collective held N ranks."""
    import json

    out = str(tmp_path / "report.json")
    mp.spawn(_report_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rep = json.load(open(out))
    assert rep["comm"]["world_size"] == world and rep["comm"]["backend"] == "gloo"
    assert rep["comm"]["ranks_reporting"] == world and rep["comm"]["rccl_version"]
    assert [r["rank"] for r in rep["ranks"]] == list(range(world))
    for r in rep["ranks"]:
        assert r["elapsed_ms"] == pytest.approx(500 + 100 * r["rank"])
        assert r["rays"] == 1000 * (r["rank"] + 1)
        assert r["gather_ms_per_step"] is not None and r["gather_ms_per_step"] >= 0
