"""Command line tools.

    python -m hipsnapshot verify PATH [--json] [--concurrency N]
        re-read every blob of the snapshot at PATH and check its recorded
        hs64 checksum (hipsnapshot/verify.py); exit status 0 iff all match
    torchrun --nproc-per-node N -m hipsnapshot verify PATH --distributed
        the same, each rank checking 1/N of the blobs
    python -m hipsnapshot info PATH
        print the snapshot's version, world size and entry counts
"""

from __future__ import annotations

import argparse
import json
import sys
from collections import Counter


def _verify(args) -> int:
    from .verify import verify_snapshot

    if args.distributed:
        # under torchrun: every rank checks its share of the blobs (gloo;
        # only the report crosses the network)
        import torch.distributed as dist

        dist.init_process_group("gloo")
    rep = verify_snapshot(args.path, concurrency=args.concurrency,
                          distributed=args.distributed)
    if args.distributed:
        import torch.distributed as dist

        rank = dist.get_rank()
        dist.destroy_process_group()
        if rank != 0:
            return 0 if rep.ok else 1
    if args.json:
        print(json.dumps(rep.as_dict()))
    else:
        if not rep.has_checksums:
            print(f"{args.path}: no checksums recorded (taken with HIPSNAPSHOT_CHECKSUM=0?)")
        else:
            print(f"{args.path}: {rep.checked}/{rep.blobs} blobs, {rep.bytes / 1e9:.3f} GB "
                  f"in {rep.seconds:.2f} s -> {'OK' if rep.ok else 'FAILED'}")
        for what in ("mismatched", "missing_blobs", "missing_checksums"):
            for p in getattr(rep, what):
                print(f"  {what}: {p}")
    return 0 if rep.ok else 1


def _info(args) -> int:
    from .snapshot import Snapshot

    md = Snapshot(args.path).metadata
    kinds = Counter(type(e).__name__ for e in md.manifest.values())
    print(json.dumps({"version": md.version, "world_size": md.world_size,
                      "entries": len(md.manifest), "by_type": dict(kinds)}))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m hipsnapshot")
    sub = ap.add_subparsers(dest="cmd", required=True)
    v = sub.add_parser("verify", help="check every blob against its recorded checksum")
    v.add_argument("path")
    v.add_argument("--json", action="store_true")
    v.add_argument("--concurrency", type=int, default=4)
    v.add_argument("--distributed", action="store_true",
                   help="split the blobs over the ranks of a torchrun launch")
    v.set_defaults(fn=_verify)
    i = sub.add_parser("info", help="summarise a snapshot's metadata")
    i.add_argument("path")
    i.set_defaults(fn=_info)
    args = ap.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
