"""bench.py's GPU-count rules (CPU): which devices a run drives, and that a
run asking for more GPUs than are visible fails loudly instead of timing
fewer (BASELINE config 5)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("gpus,world,local,ndev,rehearse,want", [
    (1, 1, 0, 1, False, ("single", [0])),
    (1, 1, 0, 8, False, ("single", [0])),
    (8, 1, 0, 8, False, ("one_process", list(range(8)))),
    (4, 1, 0, 8, False, ("one_process", [0, 1, 2, 3])),
    (2, 1, 0, 1, True, ("one_process", [0, 0])),
    (3, 1, 0, 2, True, ("one_process", [0, 1, 0])),
    (2, 2, 1, 8, False, ("ranks", [1])),
    (8, 8, 7, 8, False, ("ranks", [7])),
    (2, 2, 1, 1, True, ("ranks", [0])),
])
def test_plan_devices(gpus, world, local, ndev, rehearse, want):
    assert bench.plan_devices(gpus, world, local, ndev, rehearse) == want


@pytest.mark.parametrize("gpus,world,local,ndev,rehearse,msg", [
    (2, 1, 0, 1, False, "only 1 GPU"),        # one process, too few devices
    (8, 1, 0, 4, False, "only 4 GPU"),
    (2, 2, 1, 1, False, "needs device 1"),    # a launcher rank without its GPU
    (4, 2, 0, 8, False, "must match"),        # --gpus vs WORLD_SIZE
    (1, 1, 0, 0, True, "no GPU"),             # nothing visible, even rehearsing
    (0, 1, 0, 8, False, "at least 1"),
])
def test_plan_devices_rejects(gpus, world, local, ndev, rehearse, msg):
    with pytest.raises(ValueError, match=msg):
        bench.plan_devices(gpus, world, local, ndev, rehearse)


def test_bench_exits_nonzero_without_enough_gpus():
    """Fewer than 2 GPUs visible (none in this container): `bench.py --gpus 2`
    must exit 2 with the reason, never print a bench line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("GPUs visible: the refusal is covered by the gpu test")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "bench.py:" in p.stderr and not p.stdout.strip()


def test_cpu_baseline_cores_are_labelled(monkeypatch):
    """the CPU baselines' thread count is the job's core
    share (job_cores), never more than the affinity mask allows, and the
    line records what it ran on (affinity size, OMP_NUM_THREADS, nproc)."""
    aff = len(os.sched_getaffinity(0))
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.job_cores() == min(3, aff)
    monkeypatch.setenv("OMP_NUM_THREADS", str(aff + 100))
    assert bench.job_cores() == aff
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.job_cores() == aff
    info = bench.core_info()
    assert set(info) == {"job_cores", "sched_affinity", "OMP_NUM_THREADS", "nproc"}
    assert info["sched_affinity"] == aff and info["nproc"] == os.cpu_count()


def test_fused_reruns_fail_the_run():
    """the bench line reports re-runs of failed one-launch
    split posts per timed leg and a non-zero count fails the run."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert src.count('out["fused_reruns"] = reruns') == 2     # both modes
    assert src.count("glfsx_fused_failures()") >= 6
    assert src.count("sys.exit(3)") == 2
