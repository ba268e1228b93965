"""CPU: bench.py's rank launcher.  ``python bench.py --gpus N`` without a torch.distributed
launcher must start N ranks itself (the driver's scaling run uses that command shape), and a
launcher whose WORLD_SIZE differs from --gpus must fail instead of printing a line for the wrong
number of GPUs.  ``--launch-probe`` runs the rank flow up to the (gloo) process group only, no GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update({k: str(v) for k, v in kw.items()})
    return env


def test_gpus_n_spawns_n_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"], capture_output=True, text=True,
                       env=_env(), timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, p.stdout
    rec = json.loads(line[0])
    assert rec == {"n_gpus": 2, "ranks_answered": 2, "launched_by_bench": True}


def test_single_gpu_runs_in_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-probe"], capture_output=True, text=True,
                       env=_env(), timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1]) == {"n_gpus": 1, "ranks_answered": 1,
                                                             "launched_by_bench": False}


def test_world_size_mismatch_fails():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE=3, RANK=0, LOCAL_RANK=0), timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=3" in p.stderr
    assert not p.stdout.strip()
