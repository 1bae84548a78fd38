"""bench.py --gpus 2 without a launcher on the one-GPU box:
it starts two rank processes itself, both classify on device 0 (more ranks
than GPUs: round-robin), and the line reports the two ranks that ran."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launched_two_ranks():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c2",
                        "--frames", "262144", "--queues", "2", "--steps", "4", "--warmup", "1",
                        "--ramp", "2", "--launch-probe", "3", "--rotate-mib", "32",
                        "--no-cpu-baseline", "--no-extra"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                     # rank 0's line only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "replicas2"
    assert d["config"]["rank_devices"] == [0, 0]
    assert d["value"] > 0 and d["steps"] == 4
