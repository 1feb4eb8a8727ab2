"""bench.py's self-launcher: ``--gpus N`` without torchrun starts N ranks,
forwards rank 0's JSON line and fails the run when any rank fails."""

import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra, timeout=120):
    env = dict(os.environ, **env_extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    return p, time.monotonic() - t0


def test_launcher_forwards_rank0_json():
    p, _ = _run(["--gpus", "3"], {"HSBENCH_SELFTEST": "ok"})
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 3


def test_launcher_propagates_rank_failure_and_stops_the_others():
    # rank 1 fails at once; ranks 0 and 2 would block forever (as in a
    # rendezvous waiting for rank 1): the launcher must end them and fail
    p, dt = _run(["--gpus", "3"], {"HSBENCH_SELFTEST": "fail:1"})
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert "rank 1 exited with 3" in p.stderr
    assert dt < 60


def test_launcher_timeout_fails_the_run():
    p, dt = _run(["--gpus", "2", "--launch-timeout", "3"],
                 {"HSBENCH_SELFTEST": "fail:9"})
    assert p.returncode == 124 and "timed out" in p.stderr
    assert dt < 60


def test_torchrun_world_size_mismatch_is_an_error():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    env.pop("HSBENCH_SELFTEST", None)
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 2 and "WORLD_SIZE is 1" in p.stderr


@pytest.mark.gpu
def test_self_launched_two_rank_bench_on_one_gpu(tmp_path):
    """Two gloo ranks sharing the GPU, launched by bench.py itself, with the
    DDP (config 2) and elastic 2 -> 1 (config 3) phases, all bitwise."""
    p, _ = _run(["--gpus", "2", "--backend", "gloo", "--model", "tiny", "--steps", "2",
                 "--warmup", "1", "--async-iters", "1", "--restore-iters", "1",
                 "--raw-steps", "1", "--fresh-steps", "0", "--ddp-steps", "0",
                 "--no-numa-bind", "--path", str(tmp_path / "b")], {}, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["world_size"] == 2 and out["backend"] == "gloo"
    assert out["restore_bitwise_ok"] is True
    assert out["ddp_llama_restore_bitwise_ok"] is True
    assert len(out["ddp_llama_rank_written_bytes"]) == 2
    assert out["elastic_bitwise_ok"] is True and out["elastic_to_ranks"] == 1
    assert out["vs_baseline"] is None  # no reference number at 2 GPUs
