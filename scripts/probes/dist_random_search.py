"""Widen tests/test_dist_random.py's search: ``--seeds A B`` cases of
``--cases`` random DTensor layouts each, 4 gloo ranks, on ``--device``.
One line per seed; stops at the first failing seed."""

import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs=2, default=[20, 30])
    ap.add_argument("--cases", type=int, default=24)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--strided", action="store_true", help="mix _StridedShard placements in")
    a = ap.parse_args()
    import test_dist_random as t

    from hipsnapshot.utils.test_utils import run_distributed

    for seed in range(*a.seeds):
        with tempfile.TemporaryDirectory() as d:
            run_distributed(t._worker, 4, d, a.cases, seed, a.device, a.strided, timeout=600)
        print(f"seed {seed}: {a.cases} cases ok", flush=True)
