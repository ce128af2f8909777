"""bench.py --gpus N: one command starts N ranks (the reference's benchmark starts one
worker per GPU itself, benchmarks/python_e2e/main.py:72-79).

CPU: the dispatch logic (child launch when WORLD_SIZE is unset, the WORLD_SIZE /
--gpus consistency check, the torch.distributed.run command line).
GPU: a real 4-rank run from one command on the single test GPU over the
torch.distributed callbacks (RCCL refuses two ranks per GPU), small scales.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_gpus_n_starts_child_launcher(monkeypatch):
    bench = _bench()
    seen = {}

    def fake(n, argv):
        seen["n"], seen["argv"] = n, list(argv)
        return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", fake)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    assert seen == {"n": 4, "argv": ["--gpus", "4", "--steps", "3"]}


def test_world_size_must_match_gpus(monkeypatch):
    bench = _bench()
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=2" in str(e.value.code)


def test_launch_command_line():
    bench = _bench()
    cmd = bench.launch_command(8, ["--gpus", "8", "--steps", "2"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "2"]
    assert cmd[cmd.index("--master-port") + 2].endswith("bench.py")


@pytest.mark.gpu
def test_bench_gpus4_one_command_rehearsal():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--comm", "torch", "--scale", "17",
           "--bfs-scale", "15", "--bfs-roots", "2", "--louvain-scale", "12", "--no-secondary", "--no-traffic",
           "--no-cpu-baseline", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=240)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    lines = [x for x in r.stdout.decode().splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout.decode()[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4
    assert out["config"]["parallelism"].startswith("mg4: 2D ")
    assert out["value"] > 0
    assert out["bfs"]["n_gpus"] == 4 and out["bfs"]["mteps_harmonic_mean"] > 0
    assert out["louvain"]["n_gpus"] == 4 and out["louvain"]["modularity"] > 0
