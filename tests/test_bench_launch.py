"""bench.py's launch contract, CPU only: `bench.py --gpus N` with no launcher
must start the N ranks itself — torch.distributed.run as a CHILD process (never exec), the JSON line
passed through, the child's exit code returned — and a launcher whose WORLD_SIZE disagrees with
--gpus must be an error, so an N-GPU line can never silently time one rank. Anchor: the
reference's only parallel stage, the chunked decompression of preprocess-kgz.rs:105-110."""
import importlib.util
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_check_launch_decisions():
    b = load_bench()
    assert b.check_launch(1, {}) is None                        # N = 1: run here
    assert b.check_launch(8, {}) == "spawn"                     # N > 1, no launcher: start the ranks
    assert b.check_launch(8, {"WORLD_SIZE": "8"}) is None       # under the driver's torch.distributed.run
    assert b.check_launch(1, {"WORLD_SIZE": "1"}) is None
    err = b.check_launch(8, {"WORLD_SIZE": "1"})                # the silent one-rank case: an error now
    assert err and "WORLD_SIZE 1" in err


def test_spawn_argv_is_the_drivers_launch():
    b = load_bench()
    cmd = b.spawn_argv(4, 29511, ["--gpus", "4", "--steps", "2"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"] and cmd[-5] == os.path.abspath(BENCH)


def test_spawn_forwards_json_and_exit_code(monkeypatch, capsys):
    """The child's rank-0 JSON line reaches stdout alone; other output goes to stderr; the child's
    exit code is returned (a failing rank fails the bench)."""
    b = load_bench()
    script = "import sys; print('rccl banner'); print('{\"metric\": \"m\", \"value\": 1}'); sys.exit(3)"
    monkeypatch.setattr(b, "spawn_argv", lambda n, port, argv: [sys.executable, "-c", script])

    class A:
        gpus = 2

    assert b.spawn_ranks(A()) == 3
    out, err = capsys.readouterr()
    assert out.strip() == '{"metric": "m", "value": 1}'
    assert "rccl banner" in err and "torch.distributed.run" not in out


def _alive(pid):
    """True while pid runs: a zombie (killed but not yet reaped, e.g. when PID 1 does not reap
    orphans) or a vanished pid counts as dead."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            state = f.read().rsplit(")", 1)[1].split()[0]
    except (FileNotFoundError, ProcessLookupError, IndexError):
        return False
    return state not in ("Z", "X")


def test_rank_failure_after_timed_region_fails_the_bench(capsys, tmp_path):
    """A real torch.distributed.run with 2 ranks: rank 0 prints its JSON line and exits 0, rank 1
    fails afterwards (as a rank could in the rows after the timed region). bench.py still forwards
    the line, and its exit code is the launcher's non-zero one, so the driver sees the failure."""
    b = load_bench()
    script = ("import os, sys, time\n"
              "r = int(os.environ['RANK'])\n"
              "if r == 0:\n"
              "    print('{\"metric\": \"m\", \"value\": 1}', flush=True)\n"
              "    time.sleep(20)\n"
              "    sys.exit(0)\n"
              "time.sleep(1)\n"
              "sys.exit(7)\n")
    rank_py = tmp_path / "rank.py"
    rank_py.write_text(script)
    real = b.spawn_argv
    b.spawn_argv = lambda n, port, argv: real(n, port, [])[:-1] + [str(rank_py)]

    class A:
        gpus = 2

    assert b.spawn_argv(2, 1, [])[-1] == str(rank_py) and "torch.distributed.run" in b.spawn_argv(2, 1, [])
    t = __import__("time").perf_counter()
    rc = b.spawn_ranks(A())
    out, _ = capsys.readouterr()
    assert rc != 0
    assert out.strip() == '{"metric": "m", "value": 1}'
    assert __import__("time").perf_counter() - t < 18  # the launcher stopped rank 0 instead of waiting for it


def test_spawned_launcher_dies_with_the_bench(tmp_path):
    """A driver timeout kills bench.py: the launcher it started must not outlive it (it would keep
    the ranks on the GPUs). The child is started with PR_SET_PDEATHSIG = SIGTERM."""
    import signal
    import time

    pidfile = tmp_path / "child.pid"
    stub = ("import os, sys, time; open(sys.argv[1], 'w').write(str(os.getpid())); time.sleep(120)")
    driver = (
        "import importlib.util, sys\n"
        f"spec = importlib.util.spec_from_file_location('b', {BENCH!r}); b = importlib.util.module_from_spec(spec)\n"
        "spec.loader.exec_module(b)\n"
        f"b.spawn_argv = lambda n, port, argv: [sys.executable, '-c', {stub!r}, {str(pidfile)!r}]\n"
        "class A: gpus = 2\n"
        "sys.exit(b.spawn_ranks(A()))\n")
    parent = subprocess.Popen([sys.executable, "-c", driver])
    for _ in range(200):
        if pidfile.exists() and pidfile.read_text():
            break
        time.sleep(0.05)
    child = int(pidfile.read_text())
    parent.send_signal(signal.SIGKILL)  # no chance to forward anything: only the death signal helps
    parent.wait()
    for _ in range(100):
        if not _alive(child):
            break
        time.sleep(0.05)
    else:
        os.kill(child, signal.SIGKILL)
        raise AssertionError("the spawned launcher outlived bench.py")


def test_world_size_mismatch_exits_nonzero_before_torch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "8"], env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode == 2
    assert "WORLD_SIZE 1" in p.stderr and p.stdout == ""


def test_num_cpus_follows_num_cpus_1_13(tmp_path):
    """cpu_baseline's decompress thread count is what the reference's num_cpus::get() (1.13.0,
    /root/reference/Cargo.lock) returns: ceil(cgroup-v1 CFS quota / period), capped by the affinity
    CPUs, when a v1 cpu controller has a quota; otherwise the affinity count (cgroup v2's cpu.max
    is not read by that version)."""
    b = load_bench()
    mnt = tmp_path / "cg" / "cpu,cpuacct"
    d = mnt / "job"
    d.mkdir(parents=True)
    (d / "cpu.cfs_quota_us").write_text("150000\n")
    (d / "cpu.cfs_period_us").write_text("100000\n")
    cg = tmp_path / "cgroup"
    cg.write_text("12:memory:/job\n3:cpu,cpuacct:/job\n0::/\n")
    mi = tmp_path / "mountinfo"
    mi.write_text(f"30 25 0:26 / {mnt} rw,nosuid - cgroup cgroup rw,cpu,cpuacct\n"
                  f"31 25 0:27 / {tmp_path}/cg/memory rw - cgroup cgroup rw,memory\n")
    assert b.cgroup_v1_cpu_quota(str(cg), str(mi)) == 2
    (d / "cpu.cfs_quota_us").write_text("-1\n")  # no quota
    assert b.cgroup_v1_cpu_quota(str(cg), str(mi)) is None
    cg.write_text("0::/\n")  # cgroup v2 only
    assert b.cgroup_v1_cpu_quota(str(cg), str(mi)) is None
    assert b.num_cpus() == min(b.cgroup_v1_cpu_quota() or b.affinity_cpus(), b.affinity_cpus())
