"""bench.py's multi-rank launch (CPU only): `--gpus N` without a launcher
starts N rank processes itself and reports the ranks that joined; a WORLD_SIZE
that disagrees with --gpus is refused (`--gpus 8` must not
silently measure one GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env(**kw):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(kw)
    return e


def test_rank_envs():
    envs = bench.rank_envs(3, 12345, base_env={"X": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and
               e["MASTER_PORT"] == "12345" and e["X"] == "1" for e in envs)


def test_self_launch_two_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--launch-check"], env=_env(), capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                        # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks"] == [0, 1]


def test_world_size_mismatch_is_refused():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                          "--launch-check"], env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "WORLD_SIZE=1" in out.stderr


def test_bench_defaults_match_the_driver_contract():
    """With no flags: one GPU, a K/W that finishes in minutes, the headline on
    two result sets per queue, and c4tx's end-to-end loop over at least
    TX_LAUNCHES launches (its fill and drain under 1 %)."""
    a = bench.parse_args([])
    assert a.gpus == 1 and a.config == "c5"
    assert a.steps == 40 and a.warmup == 5
    assert a.result_rounds == 2
    assert a.tx_launches == bench.TX_LAUNCHES >= 50
    assert a.tx_rings == 8
    assert set(a.host_inclusive.split(",")) == {"c5", "c2"}
    assert bench.parse_args(["--tx-launches", "13"]).tx_launches == 13
