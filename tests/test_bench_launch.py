"""bench.py's N > 1 entry: `python bench.py --gpus N` started as a plain
process launches torch.distributed.run itself (child process, before torch
is imported) and relays rank 0's JSON line; the N > 1 line carries roofline,
cpu_baseline and both exchanges (VERDICT r05 "next" item 1)."""
import io
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_module():
    sys.path.insert(0, ROOT)
    import importlib
    import bench
    return importlib.reload(bench)


def test_self_launch_command_and_relay(monkeypatch, capsys):
    bench = _bench_module()
    seen = {}

    class FakeProc:
        def __init__(self, cmd, stdout=None, text=None, env=None):
            seen["cmd"], seen["env"] = cmd, env
            self.stdout = io.StringIO("[Gloo] Rank 0 is connected to 1 peer ranks.\n"
                                      '{"metric": "m", "value": 1.0, "n_gpus": 2}\n'
                                      "{not json\n")

        def wait(self):
            return 0

    monkeypatch.setattr(bench.subprocess, "Popen", FakeProc)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    assert bench.self_launch(2) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]
    assert seen["env"]["PM_BENCH_LAUNCHED"] == "1"
    out, err = capsys.readouterr()
    assert out.strip().splitlines() == ['{"metric": "m", "value": 1.0, "n_gpus": 2}']   # only the JSON line
    assert "Gloo" in err and "{not json" in err


def test_self_launched_rank_without_world_fails(monkeypatch):
    bench = _bench_module()
    monkeypatch.setenv("PM_BENCH_LAUNCHED", "1")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE" in str(e.value.code)


@pytest.mark.gpu
def test_bench_gpus2_self_launch_one_device():
    """Two ranks on the test box's one GPU over gloo (PM_BENCH_ONE_DEVICE /
    PM_BENCH_BACKEND: rehearsal knobs — the times are not measurements)."""
    env = dict(os.environ, PM_BENCH_ONE_DEVICE="1", PM_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c1",
                        "--steps", "3", "--warmup", "1", "--cpu-threads", "4"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0
    assert d["roofline"] is not None and d["roofline"]["frac"] > 0
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] == 4
    assert d["config"]["exchange"] == "reduce"
    assert d["alt_exchange"]["exchange"] == "allgather" and d["alt_exchange"]["value"] > 0
    assert d["exchange"]["bytes_per_pass"] > 0
