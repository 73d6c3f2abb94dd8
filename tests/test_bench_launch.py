"""bench.py's rank bookkeeping on the CPU (no GPU): `--gpus N` without a launcher starts N ranks
itself (torch.distributed.run on 127.0.0.1, gloo here), a launcher's WORLD_SIZE must agree with
--gpus, and --gpus 1 stays one process. `--launch-check` stops each rank before any GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 alone prints
    return json.loads(lines[0])


def test_gpus_2_without_launcher_spawns_two_ranks():
    p = _run(["--gpus", "2", "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    j = _line(p.stdout)
    assert j["n_gpus"] == 2 and j["gpus_flag"] == 2
    assert sorted(r["rank"] for r in j["ranks"]) == [0, 1]
    assert len({r["pid"] for r in j["ranks"]}) == 2


def test_gpus_1_stays_one_process():
    p = _run(["--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    j = _line(p.stdout)
    assert j["n_gpus"] == 1 and [r["rank"] for r in j["ranks"]] == [0]


def test_gpus_disagreeing_with_world_size_is_refused():
    p = _run(["--gpus", "3", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, drop=())
    assert p.returncode != 0
    assert "disagrees with WORLD_SIZE" in p.stderr
