import sys, random, tempfile, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tests")]
import test_e2e_random as t
from hipsnapshot.engine import native_restore, native_drain
used_r = used_d = 0
for seed in range(100, 130):
    native_restore.last_stats.clear(); native_drain.last_stats.clear()
    t._round_trip(tempfile.mkdtemp(), seed, "cuda:0", tuning=seed % 2 == 0)
    r = bool(native_restore.last_stats); d = bool(native_drain.last_stats)
    used_r += r; used_d += d
    print(seed, "native_restore", r, "native_drain", d, native_restore.last_stats.get("items"), flush=True)
print("totals", used_r, used_d)
