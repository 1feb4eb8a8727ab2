"""The examples run end to end on CPU (gloo for the multi-rank ones) and
resume from their own snapshots -- the flows of the reference's
examples/ (simple train/resume, DDP, FSDP with an elastic resume, DLRM)."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


def _env():
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="2")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    return env


def _run(args, timeout=300):
    proc = subprocess.run(args, capture_output=True, text=True, env=_env(), timeout=timeout,
                          cwd=ROOT)
    assert proc.returncode == 0, proc.stdout[-2000:] + proc.stderr[-4000:]
    return proc.stdout


def _torchrun(n, script, *args, port):
    return _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                 f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
                 os.path.join(EX, script), *args])


def test_simple_example_trains_and_resumes(tmp_path):
    wd = str(tmp_path / "run")
    out = _run([sys.executable, os.path.join(EX, "simple_example.py"), "--work-dir", wd,
                "--epochs", "2"])
    assert "epoch 2" in out
    out = _run([sys.executable, os.path.join(EX, "simple_example.py"), "--work-dir", wd,
                "--epochs", "3", "--resume"])
    assert "resumed at epoch 2" in out and "epoch 3" in out


def test_ddp_example_resumes_from_its_snapshot(tmp_path):
    wd = str(tmp_path / "ddp")
    out = _torchrun(2, "ddp_example.py", "--work-dir", wd, "--steps", "20", port=29641)
    assert "step 20: snapshot committed" in out
    out = _torchrun(2, "ddp_example.py", "--work-dir", wd, "--steps", "30", port=29642)
    # restored at step 20: only steps 21-30 ran, one snapshot at 30
    assert "step 30: snapshot committed" in out and "step 10:" not in out


def test_fsdp_example_elastic_resume(tmp_path):
    wd = str(tmp_path / "fsdp")
    out = _torchrun(2, "fsdp_example.py", "--work-dir", wd, "--steps", "10", port=29643)
    assert "done at step 10" in out
    # 2 ranks saved the sharded state; 1 rank restores it (reshards) and goes on
    out = _torchrun(1, "fsdp_example.py", "--work-dir", wd, "--steps", "15", "--resume",
                    port=29644)
    assert "done at step 15" in out


@pytest.mark.parametrize("restore_ranks", [2])
def test_dlrm_example_restores_sharded_tables(tmp_path, restore_ranks):
    sp = str(tmp_path / "dlrm")
    out = _torchrun(2, "dlrm_example.py", "--snapshot-path", sp, "--epochs", "1",
                    "--steps-per-epoch", "3", port=29645)
    assert "snapshot ->" in out
    out = _torchrun(restore_ranks, "dlrm_example.py", "--snapshot-path", str(tmp_path / "d2"),
                    "--restore-path", os.path.join(sp, "epoch_1"), "--epochs", "2",
                    "--steps-per-epoch", "3", port=29646)
    assert "restored from" in out and "at epoch 1" in out
