"""Aggregate page-cache write bandwidth of P processes x T threads (no GPU).

Emulates the storage side of an N-rank take: each process writes S bytes as
64 MB files with T threads (buffered pwrite from an anonymous buffer, like
the native I/O engine), all processes starting together.  Prints one JSON
line per P with the aggregate GB/s.  Files are rewritten in place (same
paths every round, as the benchmark's repeated takes do) after one warm-up
round.
"""

import json
import multiprocessing as mp
import os
import sys
import threading
import time


def worker(rank, d, total, nthreads, barrier, out_q):
    blob = 64 << 20
    buf = bytearray(os.urandom(1 << 20)) * 64
    n = total // blob
    paths = [os.path.join(d, f"r{rank}_{i}") for i in range(n)]

    def run_round():
        idx = [0]
        lock = threading.Lock()

        def th():
            while True:
                with lock:
                    i = idx[0]
                    idx[0] += 1
                if i >= n:
                    return
                fd = os.open(paths[i], os.O_WRONLY | os.O_CREAT, 0o644)
                os.pwrite(fd, buf, 0)
                os.close(fd)

        ts = [threading.Thread(target=th) for _ in range(nthreads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    run_round()
    barrier.wait()
    t0 = time.perf_counter()
    run_round()
    out_q.put((rank, t0, time.perf_counter()))
    for p in paths:
        os.remove(p)


def main():
    d = sys.argv[1]
    total = int(float(sys.argv[2]) * (1 << 30)) if len(sys.argv) > 2 else 2 << 30
    nthreads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    os.makedirs(d, exist_ok=True)
    ctx = mp.get_context("spawn")
    configs = [(1, nthreads), (2, nthreads), (4, nthreads), (8, nthreads),
               (4, max(1, nthreads // 4)), (8, max(1, nthreads // 8))]
    for p, nthreads in configs:
        os.sync()  # no dirty pages left from the previous configuration
        barrier = ctx.Barrier(p)
        q = ctx.Queue()
        procs = [ctx.Process(target=worker, args=(r, d, total, nthreads, barrier, q))
                 for r in range(p)]
        for pr in procs:
            pr.start()
        res = [q.get() for _ in range(p)]
        for pr in procs:
            pr.join()
        t0 = min(r[1] for r in res)
        t1 = max(r[2] for r in res)
        print(json.dumps({"probe": "pagecache_write", "procs": p, "threads": nthreads,
                          "GB_per_proc": round(total / 1e9, 2),
                          "aggregate_GBps": round(p * total / (t1 - t0) / 1e9, 1),
                          "per_proc_GBps": round(total / (t1 - t0) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
