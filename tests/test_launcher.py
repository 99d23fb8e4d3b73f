"""The multi-GPU entry point: `python bench.py --gpus N` runs N ranks.

Rehearsed on the CPU with gloo (the launcher parent spawns fresh child
processes with RANK/LOCAL_RANK/WORLD_SIZE set; rank 0 prints the slowest
rank's time). On the GPU box the same launcher starts one rank per GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(n, rows=4096, extra=()):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--device", "cpu",
                        "--rows", str(rows), "--steps", "2", "--warmup", "1", *extra],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    out = json.loads(lines[0])
    out["_rank_lines"] = [json.loads(ln) for ln in p.stderr.splitlines() if ln.startswith('{"bench_rank"')]
    return out


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_bench_spawns_n_ranks(n):
    out = _run_bench(n)
    assert out["n_gpus"] == n
    assert out["config"]["parallelism"] == f"dp{n}"
    assert out["config"]["rows"] == 4096 and out["config"]["partitions"] == 4 * n
    assert out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["max_abs_err"] < 1e-3
    assert out["scaling"] == "strong"
    # one stderr diagnostic line per rank: rank, world, backend, own time, its partitions
    ranks = sorted(out["_rank_lines"], key=lambda d: d["bench_rank"])
    assert [d["bench_rank"] for d in ranks] == list(range(n))
    assert all(d["world_size"] == n and d["own_ms_per_step"] > 0 for d in ranks)
    assert all(d["backend"] == ("gloo" if n > 1 else None) for d in ranks)
    assert sorted(p for d in ranks for p in d["partitions"]) == list(range(4 * n))
    assert all(p % n == d["bench_rank"] for d in ranks for p in d["partitions"])
    assert sum(d["rows"] for d in ranks) == 4096


def test_launcher_propagates_failure(tmp_path):
    sys.path.insert(0, REPO)
    from tensorframes_amd.parallel import launch
    script = tmp_path / "fail.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "sys.exit(3) if r == 1 else time.sleep(60)\n")
    rc = launch.spawn([str(script)], 3)
    assert rc == 3  # the failing rank's code; the sleeping ranks were taken down


def test_launcher_sets_rank_env(tmp_path):
    sys.path.insert(0, REPO)
    from tensorframes_amd.parallel import launch
    out = tmp_path / "out"
    out.mkdir()
    script = tmp_path / "env.py"
    script.write_text("import os\n"
                      f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write(\n"
                      "  ','.join(os.environ[k] for k in ('LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR')))\n")
    assert launch.spawn([str(script)], 4) == 0
    got = {p.name: p.read_text() for p in out.iterdir()}
    assert got == {str(r): f"{r},4,127.0.0.1" for r in range(4)}


def _fault_script(tmp_path, fail_attempts):
    """Rank 1 loses its 'GPU context' (a sticky-classified error) on the first
    `fail_attempts` attempts of the job; every rank records its attempt."""
    script = tmp_path / "sticky.py"
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {REPO!r})\n"
        "from tensorframes_amd.utils import faults\n"
        "@faults.exit_on_device_fault\n"
        "def main():\n"
        "    k = faults.restart_count()\n"
        f"    open(os.path.join({str(tmp_path)!r}, f\"r{{os.environ['RANK']}}_a{{k}}\"), 'w').close()\n"
        f"    if os.environ['RANK'] == '1' and k < {fail_attempts}:\n"
        "        raise RuntimeError('HIP error: an illegal memory access was encountered (illegal address)')\n"
        "main()\n")
    return script


def test_launcher_restarts_job_after_device_fault(tmp_path):
    """A sticky GPU fault is never retried in-process: the rank exits with
    EXIT_DEVICE_FAULT and the launcher re-runs the whole job in fresh
    processes (new HIP contexts), up to max_restarts times."""
    sys.path.insert(0, REPO)
    from tensorframes_amd.parallel import launch
    from tensorframes_amd.utils import faults
    assert launch.EXIT_DEVICE_FAULT == faults.EXIT_DEVICE_FAULT
    script = _fault_script(tmp_path, fail_attempts=1)
    assert launch.spawn([str(script)], 2, max_restarts=1) == 0
    names = {p.name for p in tmp_path.iterdir() if p.name.startswith("r")}
    assert {"r0_a0", "r1_a0", "r0_a1", "r1_a1"} <= names


def test_launcher_gives_up_after_max_restarts(tmp_path):
    sys.path.insert(0, REPO)
    from tensorframes_amd.parallel import launch
    from tensorframes_amd.utils import faults
    script = _fault_script(tmp_path, fail_attempts=5)
    assert launch.spawn([str(script)], 2, max_restarts=1) == faults.EXIT_DEVICE_FAULT
    assert launch.spawn([str(script)], 2, max_restarts=0) == faults.EXIT_DEVICE_FAULT


def test_non_sticky_errors_are_not_turned_into_restarts(tmp_path):
    sys.path.insert(0, REPO)
    from tensorframes_amd.utils import faults

    @faults.exit_on_device_fault
    def bad():
        raise ValueError("a validation error")
    with pytest.raises(ValueError):
        bad()

    @faults.exit_on_device_fault
    def sticky():
        raise faults.DeviceFaultError("context lost")
    with pytest.raises(SystemExit) as ei:
        sticky()
    assert ei.value.code == faults.EXIT_DEVICE_FAULT
