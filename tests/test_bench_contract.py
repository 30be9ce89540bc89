"""bench.py's roofline arithmetic (CPU): per-launch figures from the counter frame's
per-ray rates times the timed launches' rays per launch, the binding ceiling is the
highest fraction, and every reported fraction stays <= 1 -- on one GPU and for one
rank of an 8-way tile shard (whose launches carry 1/8 of the rays: r02 divided the
whole-frame PMC counts by the rank-local launch time and printed fractions > 1)."""
import bench


def _patch(monkeypatch):
    seen = {}

    def ceiling(footprint):
        seen["footprint"] = footprint
        return {"ceiling_gnodes_per_s": 150.0, "table_mb": 67.1, "per_waves_per_simd": {"7": 149.0}}

    monkeypatch.setattr(bench, "gather_ceiling", ceiling)
    # r02 config-4 PMC figures, per traced ray (11.7 GB and 2.63 G VALU per 26.6 M-ray launch)
    monkeypatch.setattr(bench, "pmc_record", lambda a: {"traffic_bytes_per_ray": 440.4, "round": "r03",
                                                        "valu_insts_per_ray": 98.7, "clock_ghz": 2.20})
    return seen


class A:
    config = 4


# counter frame: 98.4 M rays, 1.80 G node visits, 143.3 GB algorithmic
ST = {"primary_rays": 16588800, "extension_rays": 48300000, "shadow_rays": 33511200, "node_visits": 1.80e9,
      "unique_node_fetches": 0.92e9, "trace_bytes": 143.3e9, "bvh_nodes": 212619, "bvh_prims": 1000014}


def test_roofline_one_gpu_per_launch_and_binding_ceiling(monkeypatch):
    seen = _patch(monkeypatch)
    # 5 timed steps, one pipelined launch each carrying one frame's rays, 14.0 ms each
    timed = {"trace_ms": 70.0, "launches": 5, "rays": 5 * 98.4e6}
    r = bench.roofline(A, ST, timed)
    assert abs(r["ms_per_launch"] - 14.0) < 1e-9 and r["launches"] == 5
    assert abs(r["rays_per_launch"] - 98.4e6) < 1
    c = r["ceilings"]
    rays_cf = ST["primary_rays"] + ST["extension_rays"] + ST["shadow_rays"]
    f = 98.4e6 / rays_cf
    assert abs(c["node-gather"]["achieved"] - 0.92e9 * f / 14.0e-3 / 1e9) < 0.01
    assert abs(c["valu-issue"]["frac"] - 2 * 98.7 * 98.4e6 / (1024 * 2.20e9 * 14.0e-3)) < 1e-3
    assert abs(c["hbm"]["frac"] - 440.4 * 98.4e6 / 14.0e-3 / 8e12) < 1e-3
    assert abs(r["traffic"] - 440.4 * 98.4e6) < 1e3
    assert abs(r["algorithmic"]["bytes_per_launch"] - 143.3e9 * f) < 1e3
    assert all(0 < v["frac"] <= 1 for v in c.values())
    assert r["bound"] == max(c, key=lambda k: c[k]["frac"])
    assert r["frac"] == c[r["bound"]]["frac"]
    assert list(r)[:6] == ["bound", "achieved", "peak", "unit", "frac", "traffic"]
    # the gather ceiling is measured on a table no smaller than the node array
    assert seen["footprint"] == 64.0 * 212619


def test_roofline_rate_above_the_gather_table_is_not_a_ceiling(monkeypatch):
    """config 5: the traversal fetches its 137 MB node array faster than uniformly random
    gathers on a table of that size -- reported with a note, never chosen as the bound."""
    _patch(monkeypatch)
    monkeypatch.setattr(bench, "gather_ceiling", lambda footprint: {
        "ceiling_gnodes_per_s": 30.0, "table_mb": 268.4, "per_waves_per_simd": {"7": 30.0}})
    timed = {"trace_ms": 70.0, "launches": 5, "rays": 5 * 98.4e6}
    r = bench.roofline(A, ST, timed)
    c = r["ceilings"]
    assert c["node-gather"]["frac"] > 1 and "note" in c["node-gather"]
    assert r["bound"] != "node-gather" and r["frac"] <= 1


def test_roofline_rank_of_an_8_way_shard_stays_below_one(monkeypatch):
    _patch(monkeypatch)
    # one rank of 8: 1/8 of the rays per launch, launches longer than 1/8 (the launch tail)
    one = bench.roofline(A, ST, {"trace_ms": 70.0, "launches": 5, "rays": 5 * 98.4e6})
    rank = bench.roofline(A, ST, {"trace_ms": 5 * 2.2, "launches": 5, "rays": 5 * 98.4e6 / 8})
    for k, v in rank["ceilings"].items():
        assert 0 < v["frac"] <= 1, (k, v["frac"])
        assert v["frac"] < one["ceilings"][k]["frac"]  # the same work per ray, less of it per second
    assert abs(rank["traffic"] - one["traffic"] / 8) < 1e3


# ---------------------------------------------------------------- launcher (--gpus N)
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(HERE, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=env)


def test_plain_bench_gpus_2_spawns_two_ranks():
    """`python bench.py --gpus 2` with no launcher starts two rank processes (fresh
    interpreters, torchrun's environment) that form one group; rank 0 reports both."""
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2 and rec["gpus_requested"] == 2
    assert os.getpid() not in rec["pids"] and len(set(rec["pids"])) == 2


def test_bench_gpus_3_spawns_three_ranks():
    r = _run(["--gpus", "3", "--dry-run"])
    assert r.returncode == 0, r.stderr
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 3 and rec["ranks_seen"] == 3


def test_bench_world_size_disagreeing_with_gpus_fails():
    """Under a launcher, WORLD_SIZE must equal --gpus: a mismatch exits non-zero
    instead of printing an n_gpus the driver did not ask for."""
    r = _run(["--gpus", "1", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0


def test_failing_rank_fails_the_launch():
    """A rank that dies makes the whole launch fail and stops the rank still waiting
    for it in the rendezvous (no hang)."""
    import time

    t0 = time.time()
    r = _run(["--gpus", "2", "--dry-run"], {"PUPIL_BENCH_DRY_FAIL_RANK": "1"})
    assert r.returncode == 3 and time.time() - t0 < 120
    assert _run(["--gpus", "2", "--dry-run", "--config", "9"]).returncode != 0  # bad arguments
