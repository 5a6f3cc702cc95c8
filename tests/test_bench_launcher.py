"""bench.py --gpus N started without a launcher spawns N ranks itself (one
process per GPU, torch.distributed.run on 127.0.0.1) before anything touches
the GPU; --dry-run makes each rank report its place and stop there."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,extra", [(2, []), (3, []), (2, ["--n", "1024"]), (2, ["--n=512"])])
def test_bench_spawns_ranks(n, extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *extra, "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == list(range(n))
    assert sorted(x["local_rank"] for x in lines) == list(range(n))
    assert all(x["world_size"] == n and x["gpus"] == n for x in lines)
    assert all(x["master"].startswith("127.0.0.1:") for x in lines)
    want_n = int(extra[-1].split("=")[-1]) if extra else 2048  # --n passes through the launcher
    assert all(x["n"] == want_n for x in lines)


def test_bench_dry_run_single():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], capture_output=True, text=True,
                       timeout=120, cwd=ROOT)
    assert r.returncode == 0
    (x,) = [json.loads(v) for v in r.stdout.splitlines() if v.startswith("{")]
    assert x["rank"] == 0 and x["world_size"] == 1
