"""CPU tests of bench.py's multi-GPU launch contract: `--gpus N` without torch.distributed's
environment starts N ranks itself (one process per GPU on a real node), a launcher-provided
WORLD_SIZE must equal --gpus, and the rank plumbing (partition, record all-gather over gloo,
max-over-ranks timing) reports n_gpus = N.  --dry-run keeps all of it on the CPU."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return e


def _json_line(out: str):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_starts_its_own_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "3"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _json_line(p.stdout)
    assert line["n_gpus"] == 2 and line["dry_run"] is True
    assert line["config"]["rank0_shards"] == [0, 50] and line["config"]["shards_per_rank"] == 50


def test_bench_three_ranks_uneven_partition():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run", "--steps", "2"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _json_line(p.stdout)
    assert line["n_gpus"] == 3 and line["config"]["shards_per_rank"] == 34
    assert line["config"]["rank0_shards"] == [0, 33]


def test_bench_eight_ranks_configs3_geometry():
    """the driver's N = 8 run, rehearsed on the CPU: 100 shards over 8 ranks (12 or 13 per rank),
    records gathered in blocks padded to 13 over gloo and unpacked in shard order"""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run", "--steps", "2"], env=_env(),
                       capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _json_line(p.stdout)
    assert line["n_gpus"] == 8 and line["config"]["shards_per_rank"] == 13
    assert line["config"]["rank0_shards"] == [0, 12]


def test_world_size_must_match_gpus():
    e = _env()
    e.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run"], env=e, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in p.stderr
