"""bench.py's CPU-baseline leg (the oracle timed on the host) for shard sizes below
its warm-up counts: H = 1 (the C2 row) and H = 3 on a tiny scan, both legs, no GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_cpu_leg_small_shards():
    import bench
    for H in (1, 3):
        r = bench.cpu_leg(64, H, 0.2)
        assert r["value"] > 0.0 and r["kind"] == "port"
        assert r["legs"]["single_process"]["scans_per_s"] > 0.0 and r["legs"]["pool"]["scans_per_s"] > 0.0
        assert ("%d hypotheses" % H) in r["sample"]
    assert "C2" not in r["sample"] and "H=3" in r["sample"]
