"""bench.py --gpus N self-launch (CPU): N rank processes with the torch.distributed.run environment, one per
GPU, started before the launcher touches the GPU (the reference launches one process per GPU itself:
/root/reference/examples/distributed_mp.py:77-84). The rank processes are faked here; their GPU work is
the driver's multi-GPU run."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


class FakeProc:
    def __init__(self, args, env, codes, log):
        self.args, self.env = args, env
        self.rank = int(env["RANK"])
        self.codes = codes  # rank -> exit code (None: runs until terminated)
        self.code = codes.get(self.rank, 0)
        self.log = log
        log.append(("start", self.rank))

    def poll(self):
        return self.code

    def terminate(self):
        self.log.append(("terminate", self.rank))
        self.code = -15

    def kill(self):
        self.log.append(("kill", self.rank))
        self.code = -9

    def wait(self):
        return self.code


def _run(monkeypatch, argv, codes):
    log, procs = [], []

    def popen(args, env=None, stdout=None, **kw):
        p = FakeProc(args, env, codes, log)
        p.stdout = None if stdout is not subprocess.PIPE else iter(
            ['[Gloo] Rank 0 is connected to 1 peer ranks\n', '{"metric": "m", "value": 1}\n'])
        procs.append(p)
        return p
    monkeypatch.setattr(subprocess, "Popen", popen)
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    rc = bench.launch_ranks(bench.parse())
    return rc, procs, log


def test_launch_ranks_environment(monkeypatch):
    rc, procs, _ = _run(monkeypatch, ["--gpus", "4", "--steps", "3", "--warmup", "1"], {})
    assert rc == 0 and len(procs) == 4
    ports = {p.env["MASTER_PORT"] for p in procs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, p in enumerate(procs):
        assert p.env["RANK"] == p.env["LOCAL_RANK"] == str(r)
        assert p.env["WORLD_SIZE"] == p.env["LOCAL_WORLD_SIZE"] == "4"
        assert p.env["MASTER_ADDR"] == "127.0.0.1"
        assert p.args[0] == sys.executable and p.args[1].endswith("bench.py")
        assert p.args[2:] == ["--gpus", "4", "--steps", "3", "--warmup", "1"]


def test_launch_ranks_failure_stops_the_others(monkeypatch):
    rc, procs, log = _run(monkeypatch, ["--gpus", "3"], {0: None, 1: 7, 2: None})
    assert rc == 7
    assert ("terminate", 0) in log and ("terminate", 2) in log


def test_main_launches_before_touching_the_gpu(monkeypatch):
    """Without WORLD_SIZE, main() hands --gpus N > 1 to the launcher and exits with its code; it neither
    runs the CPU baseline nor imports torch.cuda state on the way."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    seen = []
    monkeypatch.setattr(bench, "launch_ranks", lambda a: seen.append(a.gpus) or 5)
    monkeypatch.setattr(bench, "cpu_baseline", lambda *x: pytest.fail("cpu baseline in the launcher"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 5 and seen == [2]


def test_rank_rejects_mismatched_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()


def test_launcher_forwards_only_rank0_json_line(monkeypatch, capsys):
    rc, procs, _ = _run(monkeypatch, ["--gpus", "2"], {})
    out, err = capsys.readouterr()
    assert rc == 0
    assert out == '{"metric": "m", "value": 1}\n'  # the library's status line went to stderr
    assert "[Gloo]" in err
