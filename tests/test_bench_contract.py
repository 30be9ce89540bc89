"""bench.py's roofline arithmetic (CPU): per-launch normalisation over the timing
frame's traversal launches, the binding ceiling is the highest fraction, and every
reported fraction is <= 1 for the r02 config-4 figures."""
import bench


def test_roofline_normalises_per_launch_and_picks_the_binding_ceiling(monkeypatch):
    monkeypatch.setattr(bench, "gather_ceiling", lambda n: {"ceiling_gnodes_per_s": 146.9, "table_mb": 16.8,
                                                             "per_waves_per_simd": {"7": 145.9}})
    monkeypatch.setattr(bench, "pmc_record", lambda a: {"traffic_bytes_per_launch": 13.06e9, "round": "r02",
                                                        "valu_insts_per_launch": 2.78e9, "clock_ghz": 2.23})

    class A:
        config = 4

    # config 4, r02: 1.80 G node visits per frame over 4 traversal launches, 15.6 ms of traversal
    st = {"node_visits": 1.80e9, "unique_node_fetches": 1.80e9, "trace_bytes": 143.3e9, "bvh_nodes": 267580}
    r = bench.roofline(A, st, trace_ms=15.64, trace_launches=4)
    assert abs(r["ms_per_launch"] - 3.91) < 1e-9
    c = r["ceilings"]
    assert abs(c["node-gather"]["achieved"] - 1.80e9 / 4 / 3.91e-3 / 1e9) < 0.01
    assert all(0 < v["frac"] <= 1 for v in c.values())
    assert r["bound"] == max(c, key=lambda k: c[k]["frac"]) == "node-gather"
    assert r["frac"] == c["node-gather"]["frac"]
    assert abs(c["valu-issue"]["frac"] - 2 * 2.78e9 / (1024 * 2.23e9 * 3.91e-3)) < 1e-3
    assert abs(c["hbm"]["frac"] - 13.06e9 / 3.91e-3 / 8e12) < 1e-3
    assert list(r)[:6] == ["bound", "achieved", "peak", "unit", "frac", "traffic"]
