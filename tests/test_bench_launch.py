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


def _launch_real(argv, timeout):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def test_real_launch_of_four_ranks_plumbs_the_environment():
    """A real `bench.py --gpus 4` launch (rank processes, not fakes) on the CPU: the 4 ranks rendezvous over gloo
    with the launcher's MASTER_ADDR / MASTER_PORT and report RANK / LOCAL_RANK / WORLD_SIZE 0..3 / 4."""
    import json
    r = _launch_real(["--gpus", "4", "--launch-check"], timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["ranks"] == [[i, i, 4] for i in range(4)]
    assert d["rank_ms_per_step"] == {"min": 10.0, "max": 40.0, "per_rank": [10.0, 20.0, 30.0, 40.0]}
    assert d["master"][0] == "127.0.0.1" and int(d["master"][1]) > 0


def test_real_launch_fails_fast_when_one_rank_fails():
    """Rank 2 exits with code 3 before the rendezvous; ranks 0, 1, 3 would wait in init_process_group forever.
    The launcher returns rank 2's code and stops the others well before the rendezvous timeout."""
    import time
    t0 = time.perf_counter()
    r = _launch_real(["--gpus", "4", "--launch-check", "--launch-check-fail", "2"], timeout=240)
    assert r.returncode == 3, r.stderr[-2000:]
    assert time.perf_counter() - t0 < 120


def test_rank_spread_and_gather_single_rank():
    assert bench.gather_elapsed(1.5, 1, None) == [1.5]
    assert bench.rank_spread([1.5], 10) is None
    s = bench.rank_spread([0.02, 0.03, 0.025], 10)
    assert s["min"] == 2.0 and s["max"] == 3.0 and s["per_rank"] == [2.0, 3.0, 2.5]


def test_pmc_traffic_only_for_one_gpu(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    traffic1, _ = bench.pmc_traffic("k_scan", "C3", a, bench.SPLIT, world=1)
    traffic8, src8 = bench.pmc_traffic("k_scan", "C3", a, bench.SPLIT, world=8)
    assert traffic8 is None and src8 is None
    assert traffic1 is not None  # the committed one-GPU summary
