"""Multi-process CPU (gloo) tests: DDP replication + partitioning + elastic
upscale, FSDP2/DTensor resharding across world sizes, async take with fault
injection, store barrier, object collectives."""

import pytest

import dist_workers as W
from hipsnapshot.utils.test_utils import run_distributed
from hipsnapshot.verify import verify_snapshot

pytestmark = pytest.mark.multiproc


def test_comm_collectives():
    run_distributed(W.comm_collectives, 3)


@pytest.mark.parametrize("chunk", [None, pytest.param(700, marks=pytest.mark.slow)])
def test_ddp_take_restore_and_upscale(tmp_path, chunk):
    p = str(tmp_path / f"ddp_{chunk}")
    run_distributed(W.ddp_take, 2, p, chunk)
    rep = verify_snapshot(p)  # replicated + per-rank blobs, both rank files
    assert rep.ok and rep.checked == rep.blobs > 0, rep
    run_distributed(W.ddp_restore, 2, p, 2)
    run_distributed(W.ddp_restore, 3, p, 2)  # elastic: a new rank joins


def test_replicated_write_load_balance(tmp_path):
    run_distributed(W.write_load_balance, 3, str(tmp_path / "lb"))


def test_partition_plan():
    run_distributed(W.partition_plan_check, 4)


@pytest.mark.parametrize("save_ws,load_ws", [(2, 2), (2, 1), pytest.param(2, 3, marks=pytest.mark.slow),
                                              (4, 2)])
def test_fsdp2_dtensor_resharding(tmp_path, save_ws, load_ws):
    p = str(tmp_path / "fsdp")
    run_distributed(W.fsdp_take, save_ws, p)
    assert verify_snapshot(p).ok
    run_distributed(W.fsdp_restore, load_ws, p)


@pytest.mark.parametrize("load_ws", [1, 2])
def test_fsdp2_optimizer_state_restores_into_a_fresh_optimizer(tmp_path, load_ws):
    p = str(tmp_path / "opt")
    run_distributed(W.fsdp_optim_take, 2, p)
    run_distributed(W.fsdp_optim_restore_fresh, load_ws, p)


def test_fsdp2_takes_reuse_plan_on_every_rank(tmp_path):
    run_distributed(W.fsdp_take_reusing_plan, 2, str(tmp_path / "pc"))


def test_async_take(tmp_path):
    run_distributed(W.async_take_ok, 2, str(tmp_path / "a"))


def test_async_take_fault_injection(tmp_path):
    run_distributed(W.async_take_faulty, 2, str(tmp_path / "f"))


def test_async_take_staging_fault_fails_peers_promptly(tmp_path):
    run_distributed(W.async_take_staging_fault, 2, str(tmp_path / "sf"))


def test_linear_barrier():
    run_distributed(W.linear_barrier, 3, "lb_ok")


def test_linear_barrier_error_propagation():
    run_distributed(W.linear_barrier, 3, "lb_err", -1, 1)


def test_linear_barrier_timeout():
    run_distributed(W.linear_barrier, 2, "lb_to", 1, -1)


def test_replication_glob_semantics(tmp_path):
    run_distributed(W.replication_globs, 2, str(tmp_path / "g"))


@pytest.mark.parametrize("ignore", [False, True])
def test_ddp_replication_inference(tmp_path, ignore):
    run_distributed(W.ddp_infer_replication, 2, str(tmp_path / f"d{ignore}"), ignore)


def test_take_returns_after_commit_on_every_rank(tmp_path):
    # reference quirk: take() returned before rank 0 wrote the metadata, so a
    # rank that read the snapshot at once could find nothing
    run_distributed(W.committed_on_return, 3, str(tmp_path / "c"))


def test_distributed_verify(tmp_path):
    run_distributed(W.distributed_verify, 3, str(tmp_path / "dv"))


def test_async_take_metadata_through_store(tmp_path):
    run_distributed(W.async_metadata_via_store, 3, str(tmp_path / "a"))


def test_state_dict_barriers_only_when_needed():
    run_distributed(W.state_dict_barriers, 2)


def test_write_load_rebalancing(tmp_path):
    run_distributed(W.rebalance_take, 3, str(tmp_path / "rb"))


def test_rebalance_plan_math():
    from hipsnapshot.parallel.rebalance import plan_moves

    cands = [[(i, 100, f"a{i}") for i in range(8)], [], [(0, 50, "c0")]]
    moves = plan_moves([800, 0, 50], cands, 0.1, 12)
    loads = [800, 0, 50]
    for src, _i, dst, n, _p in moves:
        loads[src] -= n
        loads[dst] += n
    assert max(loads) - min(loads) <= 100 and loads[0] <= 350, (moves, loads)
    assert plan_moves([100, 100], [[(0, 10, "x")], []], 0.1, 4) == []


def test_rewrite_of_committed_path_uncommits_before_any_blob_write(tmp_path):
    # rank 0 deletes the old .snapshot_metadata before its part of the first
    # collective; a blob written while it still exists fails the take
    run_distributed(W.rewrite_never_overlaps_commit, 3, str(tmp_path / "rw"))


def test_forced_collectives_at_world_size_one(tmp_path):
    # HIPSNAPSHOT_FORCE_COLLECTIVES: a one-rank group issues every collective
    # (the GPU suite runs the same worker on RCCL and compares)
    run_distributed(W.forced_collectives, 1, str(tmp_path / "s"), str(tmp_path / "o.json"),
                    False)
