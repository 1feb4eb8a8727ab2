#!/usr/bin/env python3
"""Device-memory churn across processes sharing one GPU, outside the restore
engine: does data that one process writes into freshly allocated HBM ever
come back wrong when other processes allocate and free HBM at the same time?

Every process loops: allocate an uncached block U (the restore's SDMA upload
target) and a plain block S (decode scratch), SDMA-upload a tagged pattern
into U, copy U -> S -> a torch tensor with the copy kernel (hs_copy_nd), read
S and the tensor back and compare, then free U and S.  Words carry
(process, iteration, index), so a wrong word names who wrote it.

    python scripts/probes/pool_churn_mp.py [--procs 4] [--iters 200]
        [--mode both|uc|plain|none] [--alloc malloc|vmm|mixed] [--out FILE]

mode: which kinds are allocated and freed every iteration (``none``: both
blocks are allocated once and kept, the restore's default).
"""

import argparse
import json
import multiprocessing as mp
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

MiB = 1 << 20


def pattern(np, r, k, nwords):
    i = np.arange(nwords, dtype=np.uint32)
    return (np.uint32(r & 0xF) << np.uint32(28)) | (np.uint32(k & 0xFFF) << np.uint32(16)) | \
        (i & np.uint32(0xFFFF))


def classify(np, got, want, r, k):
    bad = np.nonzero(got != want)[0]
    if not len(bad):
        return None
    g = got[bad]
    procs = (g >> 28) & 0xF
    iters = (g >> 16) & 0xFFF
    zero = int((g == 0).sum())
    own_stale = int(((procs == (r & 0xF)) & (iters != (k & 0xFFF))).sum())
    foreign = int((procs != (r & 0xF)).sum()) - zero
    return {"bad_words": int(len(bad)), "first": int(bad[0]), "last": int(bad[-1]),
            "zero": zero, "own_stale": own_stale, "foreign_or_other": foreign,
            "sample": [hex(int(x)) for x in g[:8]]}


def worker(r, args, q):
    import numpy as np
    import torch

    from hipsnapshot.ops import native

    lib = native.require_gpu_lib()
    torch.cuda.set_device(0)
    if args.alloc == "vmm":
        alloc, free = lib.hsg_rt_vmm_alloc, lib.hsg_rt_vmm_free
    elif args.alloc == "mixed":
        # uncached blocks from the VMM hooks, plain ones from hipMalloc (as
        # torch's allocator frees and re-allocates them beside the pools)
        def alloc(dev, n, uncached):
            return (lib.hsg_rt_vmm_alloc if uncached else lib.hsg_rt_dev_alloc)(dev, n, uncached)

        def free(p):
            if lib.hsg_rt_vmm_free(p) == -1:  # not a VMM block
                lib.hsg_rt_dev_free(p)
    else:
        alloc, free = lib.hsg_rt_dev_alloc, lib.hsg_rt_dev_free
    rng = random.Random(1000 + r)
    stream = native.copy_stream(0, 77)
    sizes = [2 * MiB, 4 * MiB, 8 * MiB]
    maxn = max(sizes)
    src = native.PinnedBuffer(maxn)
    back = native.PinnedBuffer(maxn)
    dest = torch.empty(maxn, dtype=torch.uint8, device="cuda:0")
    kept_u = kept_s = None
    if args.mode in ("plain", "none"):
        kept_u = alloc(0, maxn, 1)
    if args.mode in ("uc", "none"):
        kept_s = alloc(0, maxn, 0)
    res = {"rank": r, "iters": 0, "bad_iters": 0, "errors": [], "details": []}
    t0 = time.time()
    for k in range(args.iters):
        n = rng.choice(sizes)
        nu, ns = (rng.choice(sizes), rng.choice(sizes))
        nu = max(nu, n)
        ns = max(ns, n)
        order = rng.random() < 0.5
        u = kept_u
        s = kept_s
        if u is None and order:
            u = alloc(0, nu, 1)
        if s is None:
            s = alloc(0, ns, 0)
        if u is None:
            u = alloc(0, nu, 1)
        if not u or not s:
            res["errors"].append(f"iter {k}: alloc failed")
            break
        want = pattern(np, r, k, n // 4)
        np.frombuffer(src.view, dtype=np.uint32, count=n // 4)[:] = want
        rc = lib.hsg_sdma_h2d(0, u, src.ptr, n)
        if rc != 0:
            res["errors"].append(f"iter {k}: sdma {rc}")
            break
        b = native.CopyBatch()
        b.add_bytes(u, s, n)
        b.launch(0, stream, sync=True)
        b = native.CopyBatch()
        b.add_bytes(s, dest.data_ptr(), n)
        b.launch(0, stream, sync=True)
        checks = {}
        if lib.hsg_rt_memcpy_d2h(back.ptr, u, n) != 0:
            res["errors"].append(f"iter {k}: d2h U {lib.hsg_rt_last_error()}")
            break
        checks["U"] = classify(np, np.frombuffer(back.view, dtype=np.uint32, count=n // 4).copy(),
                               want, r, k)
        if lib.hsg_rt_memcpy_d2h(back.ptr, s, n) != 0:
            res["errors"].append(f"iter {k}: d2h S {lib.hsg_rt_last_error()}")
            break
        checks["S"] = classify(np, np.frombuffer(back.view, dtype=np.uint32, count=n // 4).copy(),
                               want, r, k)
        got = dest[:n].cpu().numpy().view(np.uint32)
        checks["T"] = classify(np, got, want, r, k)
        res["iters"] += 1
        res.setdefault("log", []).append([k, hex(u), hex(s), sorted(kk for kk, v in checks.items()
                                                                   if v)])
        if any(v is not None for v in checks.values()):
            res["bad_iters"] += 1
            if len(res["details"]) < 20:
                res["details"].append({"iter": k, "n": n, "u": hex(u), "s": hex(s),
                                       **{kk: v for kk, v in checks.items() if v}})
        frees = [p for p, kept in ((u, kept_u), (s, kept_s)) if p != kept]
        if rng.random() < 0.5:
            frees.reverse()
        for p in frees:
            free(p)
    res["seconds"] = round(time.time() - t0, 2)
    q.put(res)


def previous_kind_table(ranks):
    """Per block role (U uncached / S plain): how many iterations had a bad
    check, split by what the block's address was last allocated as in this
    process (same kind, the other kind, never).  A stale translation of a
    re-used address shows as bad iterations in the "other" rows only."""
    table = {}
    for r in ranks:
        last = {}
        for k, u, s, bad in r.get("log", []):
            for role, addr, kind in (("U", u, 1), ("S", s, 0)):
                prev = last.get(addr)
                key = f"{role}:{'never' if prev is None else 'same' if prev == kind else 'other'}"
                row = table.setdefault(key, [0, 0])
                row[0] += 1
                row[1] += int(bool(bad))
            last[u], last[s] = 1, 0
    return {k: {"iters": v[0], "bad": v[1]} for k, v in sorted(table.items())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--mode", default="both", choices=["both", "uc", "plain", "none"])
    ap.add_argument("--alloc", default="malloc", choices=["malloc", "vmm", "mixed"],
                    help="hipMalloc / hipExtMallocWithFlags, the VMM blocks of hshost.hip, "
                         "or VMM uncached blocks beside hipMalloc plain ones")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, args, q)) for r in range(args.procs)]
    for p in ps:
        p.start()
    out = []
    for _ in ps:
        out.append(q.get(timeout=200))
    for p in ps:
        p.join(timeout=60)
    summary = {"mode": args.mode, "alloc": args.alloc, "procs": args.procs, "iters": args.iters,
               "bad_iters": sum(o["bad_iters"] for o in out),
               "errors": sum(len(o["errors"]) for o in out),
               "exitcodes": [p.exitcode for p in ps],
               "ranks": sorted(out, key=lambda o: o["rank"])}
    summary["by_previous_kind"] = previous_kind_table(summary["ranks"])
    print(json.dumps({k: v for k, v in summary.items() if k != "ranks"}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
