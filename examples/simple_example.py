#!/usr/bin/env python3
"""Single-process training loop with periodic snapshots and resume.

    python examples/simple_example.py --work-dir /tmp/run1            # train + snapshot
    python examples/simple_example.py --work-dir /tmp/run1 --resume    # resume from latest

(Same flow as the reference's examples/simple_example.py:60-82.)
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipsnapshot import RNGState, Snapshot, StateDict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work-dir", default="/tmp/hipsnapshot_simple")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--resume", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(128, 256), torch.nn.ReLU(),
                                torch.nn.Linear(256, 10)).to(dev)
    optim = torch.optim.AdamW(model.parameters(), lr=1e-3)
    progress = StateDict(epoch=0)
    app_state = {"model": model, "optim": optim, "progress": progress, "rng": RNGState()}
    latest = os.path.join(args.work_dir, "latest")
    if args.resume and os.path.exists(os.path.join(latest, ".snapshot_metadata")):
        Snapshot(latest).restore(app_state)
        print(f"resumed at epoch {progress['epoch']}")
    while progress["epoch"] < args.epochs:
        for _ in range(20):
            x = torch.randn(64, 128, device=dev)
            loss = torch.nn.functional.cross_entropy(model(x), torch.randint(0, 10, (64,),
                                                                              device=dev))
            optim.zero_grad()
            loss.backward()
            optim.step()
        progress["epoch"] += 1
        Snapshot.take(latest, app_state)
        print(f"epoch {progress['epoch']}: loss {loss.item():.4f} (snapshot -> {latest})")


if __name__ == "__main__":
    main()
