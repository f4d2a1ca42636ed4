"""Host-side helpers of bench.py (no GPU): CPU placement picks whole cores."""
import os

import bench


def _core(c):
    try:
        return open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
    except OSError:
        return str(c)


def test_idlest_picks_distinct_cores():
    cpus = sorted(os.sched_getaffinity(0))
    k = min(4, len(cpus))
    got = bench.idlest(cpus, k, window=0.05)
    assert len(got) == k and len(set(got)) == k and set(got) <= set(cpus)
    ncores = len({_core(c) for c in cpus})
    if ncores >= k:  # one CPU per core whenever there are enough cores
        assert len({_core(c) for c in got}) == k


def test_idlest_fills_when_cores_are_few():
    cpus = sorted(os.sched_getaffinity(0))[:2]
    got = bench.idlest(cpus, 2, window=0.01)
    assert sorted(got) == sorted(cpus)


def _args(*argv):
    import sys
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_rank_env_from_torchrun():
    """Under torchrun the environment names the rank; --gpus must agree with the world."""
    a = _args("--gpus", "4")
    assert bench.rank_env(a, {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}) == (2, 4, 2)
    assert bench.rank_env(_args(), {"WORLD_SIZE": "8", "RANK": "7", "LOCAL_RANK": "7"}) == (7, 8, 7)
    import pytest
    with pytest.raises(SystemExit):
        bench.rank_env(a, {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})


def test_rank_env_single_and_launcher():
    assert bench.rank_env(_args(), {}) == (0, 1, 0)
    assert bench.rank_env(_args("--gpus", "1"), {}) == (0, 1, 0)
    assert bench.rank_env(_args("--gpus", "2"), {}) is None  # this process starts the ranks


def test_launch_fails_without_enough_gpus(capsys):
    """`bench.py --gpus 2` on a box with fewer GPUs exits non-zero with a clear message,
    before anything is started."""
    rc = bench.launch_ranks(_args("--gpus", "2"), ["--gpus", "2"], device_count=1)
    assert rc == 2
    assert "needs 2 visible GPUs, found 1" in capsys.readouterr().err


def test_launch_cmd_is_torchrun_on_loopback():
    cmd = bench.launch_cmd(["--gpus", "8", "--steps", "20"], 8, 29511)
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and "--master-port=29511" in cmd
    assert cmd[-5:] == [os.path.abspath(bench.__file__), "--gpus", "8", "--steps", "20"]


def test_launch_runs_ranks_with_rank_environment(tmp_path):
    """The launcher's children see torchrun's rank environment (gloo world of 2 on the CPU:
    a stand-in script that reports what bench.rank_env reads)."""
    import subprocess
    import sys
    script = tmp_path / "probe.py"
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {os.path.dirname(os.path.abspath(bench.__file__))!r})\n"
        "import bench\n"
        "a = bench.parse()\n"
        "r = bench.rank_env(a)\n"
        f"open(os.path.join({str(tmp_path)!r}, 'rank%d' % r[0]), 'w').write('%d %d %d' % r)\n")
    cmd = bench.launch_cmd(["--gpus", "2"], 2, bench.free_port())
    cmd[cmd.index(os.path.abspath(bench.__file__))] = str(script)
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    assert subprocess.call(cmd, env=env, timeout=120) == 0
    got = sorted((tmp_path / f).read_text() for f in ("rank0", "rank1"))
    assert got == ["0 2 0", "1 2 1"]
