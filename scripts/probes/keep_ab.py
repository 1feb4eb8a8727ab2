#!/usr/bin/env python3
"""A/B of the restore pools' kept bytes on the 2-D DTensor GPU test
(tests/test_dtensor_2d.py, read_object with a 2048-byte budget)."""

import os
import sys
import tempfile
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def restore(tmp, target, keep, trim_mode):
    from hipsnapshot import knobs

    knobs.TUNING.restore_keep_bytes = keep
    import test_dtensor_2d as T

    T._restore_worker(tmp, target, "cuda:0")


def main():
    import test_dtensor_2d as T

    from hipsnapshot.utils.test_utils import run_distributed

    tmp = tempfile.mkdtemp(dir=os.environ.get("HSBENCH_DIR", "/tmp"))
    run_distributed(T._save_worker, 4, tmp, "cuda:0", timeout=600)
    for keep in (int(sys.argv[1]) if len(sys.argv) > 1 else 0, (2 << 30) + (256 << 20)):
        for target in ("2d_swapped", "fsdp"):
            try:
                run_distributed(restore, 4, tmp, target, keep, 0, timeout=600)
                print(f"keep={keep} target={target}: OK", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"keep={keep} target={target}: FAIL {str(e)[-600:]}", flush=True)


if __name__ == "__main__":
    main()
