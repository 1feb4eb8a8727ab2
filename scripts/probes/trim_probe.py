#!/usr/bin/env python3
"""Restore-pool trim probe: read_object of raw fp32 tensors into HBM with a
2048-byte budget (many tiny native items), trimming the restore pools after
every job -- both pools, only the uncached upload pool, only the scratch
pool, or none -- and checking the bytes each time."""

import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from hipsnapshot import Snapshot, StateDict  # noqa: E402
from hipsnapshot.engine import native_restore  # noqa: E402
from hipsnapshot.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
tmp = tempfile.mkdtemp(dir=os.environ.get("HSBENCH_DIR", "/tmp"))
torch.manual_seed(0)
sd = StateDict(a=torch.randn(256, 96, device=dev), b=torch.randn(1000, 33, device=dev),
               c=torch.randn(64, 64, device=dev))
Snapshot.take(os.path.join(tmp, "s"), {"sd": sd})
lib = native.require_gpu_lib()
modes = {"none": None, "both0": (0, 0), "upload0": (0, 1 << 40), "scratch0": (1 << 40, 0)}
for mode, keeps in modes.items():
    if keeps is None:
        native_restore.native.restore_trim = lambda d, k: 0
    else:
        native_restore.native.restore_trim = \
            lambda d, k, _k=keeps: int(lib.hsg_restore_trim_pools(d, _k[0], _k[1]))
    bad = corrupt = 0
    for it in range(12):
        for name, ref in sd.items():
            for budget in (None, 2048):
                out = torch.full_like(ref, -7.0)
                try:
                    # verify: the job hashes the uploaded bytes in HBM -- a
                    # mismatch means the upload (not the copy kernel) is wrong
                    Snapshot(os.path.join(tmp, "s")).read_object(
                        f"0/sd/{name}", obj_out=out, memory_budget_bytes=budget,
                        verify=(it % 2 == 1))
                except native.CorruptBlobError as e:
                    corrupt += 1
                    if corrupt <= 3:
                        print(f"  {mode} it={it} {name} budget={budget}: {e}", flush=True)
                torch.cuda.synchronize()
                if not torch.equal(out, ref):
                    bad += 1
                    if bad <= 3:
                        diff = (out != ref).nonzero()
                        print(f"  {mode} it={it} {name} budget={budget}: {diff.shape[0]} wrong "
                              f"elements, first {diff[0].tolist()}", flush=True)
    print(f"mode={mode}: {bad} bad reads of {12 * 3 * 2}, {corrupt} failed verification",
          flush=True)
