#!/usr/bin/env python3
"""Restore-pool trim probe with 4 processes sharing one GPU (gloo): every
rank read_objects the 2-D DTensor test snapshot with a 2048-byte budget,
trimming the restore pools after every job in a given mode (none / both /
upload / scratch), half of the reads with verify=True (the job hashes the
uploaded bytes in HBM: a mismatch means the upload, not the copy, is wrong)."""

import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

MODES = {"none": None, "both0": (0, 0), "upload0": (0, 1 << 40), "scratch0": (1 << 40, 0)}


def worker(tmp, mode, out_dir):
    import torch
    import torch.distributed as dist

    from hipsnapshot import Snapshot
    from hipsnapshot.engine import native_restore
    from hipsnapshot.ops import native

    lib = native.require_gpu_lib()
    keeps = MODES[mode]
    if keeps is None:
        native_restore.native.restore_trim = lambda d, k: 0
    else:
        native_restore.native.restore_trim = \
            lambda d, k, _k=keeps: int(lib.hsg_restore_trim_pools(d, _k[0], _k[1]))
    ref = torch.load(f"{tmp}/ref.pt", weights_only=True)
    bad = corrupt = total = 0
    for it in range(6):
        for name in ("layers.0.attention.wq.weight", "layers.1.feed_forward.w2.weight",
                     "tok_embeddings.weight"):
            for budget in (None, 2048):
                total += 1
                plain = torch.zeros_like(ref[f"m/{name}"]).to("cuda:0")
                try:
                    Snapshot(f"{tmp}/async").read_object(f"0/model/{name}", obj_out=plain,
                                                         memory_budget_bytes=budget,
                                                         verify=bool(it % 2))
                except native.CorruptBlobError:
                    corrupt += 1
                torch.cuda.synchronize()
                if not torch.equal(plain.cpu(), ref[f"m/{name}"]):
                    bad += 1
    with open(os.path.join(out_dir, f"{mode}.{dist.get_rank()}"), "w") as f:
        f.write(f"{bad} {corrupt} {total}\n")


def main():
    import test_dtensor_2d as T

    from hipsnapshot.utils.test_utils import run_distributed

    tmp = tempfile.mkdtemp(dir=os.environ.get("HSBENCH_DIR", "/tmp"))
    run_distributed(T._save_worker, 4, tmp, "cuda:0", timeout=600)
    out = tempfile.mkdtemp(dir=os.environ.get("HSBENCH_DIR", "/tmp"))
    for mode in sys.argv[1:] or list(MODES):
        try:
            run_distributed(worker, 4, tmp, mode, out, timeout=600)
        except Exception as e:  # noqa: BLE001
            print(f"mode={mode}: worker failed {str(e)[-300:]}", flush=True)
            continue
        res = [open(os.path.join(out, f"{mode}.{r}")).read().split() for r in range(4)]
        print(f"mode={mode}: wrong reads / failed verification / reads per rank: {res}",
              flush=True)


if __name__ == "__main__":
    main()
