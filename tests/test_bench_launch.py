"""bench.py's rank launch (CPU): `bench.py --gpus N` run without a torch.distributed.run
environment re-launches itself with N ranks (one process per GPU), and the ranks agree on the
communicator id rank 0 broadcasts. --dry-run stops after that exchange, so no GPU is needed."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIST_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in DIST_ENV}
    env.update(extra)
    return env


def _json_lines(text):
    out = []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            out.append(json.loads(line))
    return out


def test_bench_gpus2_dry_run_spawns_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [d for d in _json_lines(r.stdout) if d.get("dry_run")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    d = lines[0]
    assert d["n_ranks"] == 2
    views = sorted(tuple(v) for v in d["ranks"])
    assert [v[:2] for v in views] == [(0, 2), (1, 2)]
    assert views[0][2] == views[1][2], "ranks hold different communicator ids"


def test_bench_rejects_gpus_world_size_mismatch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], cwd=ROOT,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "disagrees with WORLD_SIZE" in r.stderr


def test_workload_labels_name_the_config():
    """The bench line's config.workload names the BASELINE.json config it measures, and any other
    --hyps by its own shape (round 3 labelled a 32-hypothesis run "C3")."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.workload_label(256, 65536, 1) == "C3"
    assert bench.workload_label(256, 65536, 8).startswith("C4")
    assert bench.workload_label(1, 65536, 1) == "C2"
    assert bench.workload_label(32, 65536, 1).startswith("H=32 (one rank's shard of C4 at N=8)")
    assert bench.workload_label(100, 65536, 1) == "H=100, 65536 points"
