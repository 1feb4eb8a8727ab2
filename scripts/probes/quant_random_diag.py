"""Diagnose tests/test_quant_random.py GPU mismatches: for each failing seed,
where the restored tensor differs from the fp32 reference of its format --
per block: does the block hold a non-finite value, a subnormal-scale amax,
and how far apart are the values."""

import os
import random
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import test_quant_random as t  # noqa: E402
from hipsnapshot import Snapshot, StateDict  # noqa: E402
from hipsnapshot.utils.test_utils import env  # noqa: E402

seeds = [int(s) for s in sys.argv[1:]] or list(range(100, 130))
for seed in seeds:
    rng = random.Random(seed)
    g = torch.Generator().manual_seed(seed)
    fmt = rng.choice(t.FORMATS)
    # the same draws as _round_trip
    state = {}
    import math
    for i in range(rng.randint(1, 5)):
        dtype = rng.choice([torch.float32, torch.bfloat16, torch.float16])
        n = rng.choice([1, 31, 32, 33, 127, 129, 4096, rng.randint(1, 300_000)])
        shape = [n] if rng.random() < 0.5 or n < 4 else [n // 2, 2]
        x = t._values(rng, math.prod(shape), g).view(shape)
        if dtype == torch.float16:
            x = x.clamp(-6e4, 6e4)
        state[f"w{i}"] = x.to(dtype).to("cuda:0")
    d = tempfile.mkdtemp()
    with env(HIPSNAPSHOT_FP8_FORMAT=fmt):
        Snapshot.take(d, {"sd": StateDict(**state)}, quantize=["sd/**"])
    snap = Snapshot(d)
    man = snap.get_manifest()
    out = StateDict(**{k: torch.zeros_like(v) for k, v in state.items()})
    snap.restore({"sd": out})
    for k, v in state.items():
        quant = man[f"0/sd/{k}"].quant
        ref = t._reference(v.cpu(), quant).float().reshape(-1)
        got = out[k].cpu().float().reshape(-1)
        x = v.cpu().float().reshape(-1)
        nan_r, nan_g = torch.isnan(ref), torch.isnan(got)
        bad = (nan_r != nan_g) | (~nan_r & ~nan_g & (ref != got))
        if not bad.any():
            continue
        blk = quant["block"]
        n = x.numel()
        bad_blocks = sorted(set((bad.nonzero().flatten() // blk).tolist()))
        info = []
        for b in bad_blocks[:4]:
            xs = x[b * blk:(b + 1) * blk]
            nonfinite = int((~torch.isfinite(xs)).sum())
            amax = float(xs[torch.isfinite(xs)].abs().max()) if torch.isfinite(xs).any() else None
            i0 = int(bad.nonzero()[0])
            info.append(dict(block=b, nonfinite=nonfinite, amax=amax,
                             nbad=int(bad[b * blk:(b + 1) * blk].sum())))
        i0 = int(bad.nonzero()[0])
        print(dict(seed=seed, fmt=fmt, key=k, dtype=str(v.dtype), n=n, rot=quant.get("rotation"),
                   nbad=int(bad.sum()), nblocks_bad=len(bad_blocks), first=i0,
                   x=float(x[i0]), ref=float(ref[i0]), got=float(got[i0]), blocks=info),
              flush=True)
