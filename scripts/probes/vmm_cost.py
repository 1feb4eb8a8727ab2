#!/usr/bin/env python3
"""Cost of the restore pools' VMM blocks (hshost.hip hsg_rt_vmm_alloc/free)
against hipMalloc / hipExtMallocWithFlags + hipFree, per size and kind: what
a restore pays when its pools were trimmed to 0 and it allocates its rings
again.  Prints one JSON object (milliseconds, median of 5)."""

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from hipsnapshot.ops import native

    lib = native.require_gpu_lib()
    torch.cuda.init()
    out = {}
    for size in (2 << 20, 64 << 20, 512 << 20, 2 << 30):
        for uncached in (1, 0):
            for name, alloc, free in (("vmm", lib.hsg_rt_vmm_alloc, lib.hsg_rt_vmm_free),
                                      ("malloc", lib.hsg_rt_dev_alloc, lib.hsg_rt_dev_free)):
                ta, tf = [], []
                for _ in range(5):
                    t0 = time.perf_counter()
                    p = alloc(0, size, uncached)
                    t1 = time.perf_counter()
                    assert p, lib.hsg_rt_last_error()
                    free(p)
                    t2 = time.perf_counter()
                    ta.append((t1 - t0) * 1e3)
                    tf.append((t2 - t1) * 1e3)
                key = f"{name}_{'uc' if uncached else 'plain'}_{size >> 20}MiB"
                out[key] = {"alloc_ms": round(statistics.median(ta), 3),
                            "free_ms": round(statistics.median(tf), 3)}
    out["vmm_retired_bytes"] = int(lib.hsg_rt_vmm_retired_bytes())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
