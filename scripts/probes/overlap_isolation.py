"""Where does a background snapshot drain slow training down?

Two processes share the one GPU:

* ``--role train``: Llama-3-8B FSDP2 + AdamW training steps (stream-local
  sync, like ``loss.item()``), each step's end time and duration appended to
  ``<out>/train.jsonl``; it writes ``<out>/ready`` after warm-up and stops
  after ``--seconds``.
* ``--role drain --what X``: waits for ``ready``, idles ``--lead`` seconds,
  then runs ONE kind of load for ``--seconds`` and records its window in
  ``<out>/drain_X.json``:
    - ``take_hsz1`` / ``take_raw``: back-to-back Snapshot.take of a 16 GB bf16
      state of its own (codec / no codec);
    - ``d2h``: 256 MiB device -> pinned host copies (SDMA), nothing written;
    - ``write``: 16 threads pwrite() pinned buffers to the page cache, no GPU;
    - ``encode``: HSZ1 encode kernels on 256 MiB, nothing leaves the GPU;
    - ``encode_capped``: the same with the drain's grid cap (HIPSNAPSHOT_DRAIN_CUS);
    - ``none``: nothing (the trainer's quiet baseline window).

Comparing the trainer's step time inside vs outside each window separates
GPU-side contention (kernels, DMA) from host-side contention (page-cache
copies, memory bandwidth) -- with no in-process effect (GIL, runtime locks),
which the in-process benchmark (benchmarks/train_overlap) includes.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def train(args) -> None:
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(args.port), RANK="0",
                      WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    cfg = LlamaConfig.llama3_8b()
    model = build_fsdp_llama(cfg, dev, torch.bfloat16, mesh=init_device_mesh("cuda", (1,)),
                             compute_dtype=torch.bfloat16)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5, foreach=True)
    gen = torch.Generator(device=dev).manual_seed(1)
    stream = torch.cuda.current_stream(dev)

    def step() -> None:
        tok = torch.randint(0, cfg.vocab_size, (1, args.seq + 1), device=dev, generator=gen)
        loss = F.cross_entropy(model(tok[:, :-1]).float().flatten(0, 1), tok[:, 1:].flatten())
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        stream.synchronize()

    for _ in range(3):
        step()
    open(os.path.join(args.out, "ready"), "w").close()
    t_end = time.time() + args.seconds
    with open(os.path.join(args.out, "train.jsonl"), "w") as f:
        while time.time() < t_end:
            t0 = time.time()
            step()
            f.write(json.dumps({"end": time.time(), "dur": time.time() - t0}) + "\n")
            f.flush()
    dist.destroy_process_group()


def drain(args) -> None:
    import torch

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.ops import codec, native

    while not os.path.exists(os.path.join(args.out, "ready")):
        time.sleep(0.1)
    dev = torch.device("cuda", 0)
    what = args.what
    n = 0
    if what == "none":
        pass
    elif what.startswith("take"):
        ts = [(torch.randn(64 << 20, device=dev) * 0.02).to(torch.bfloat16) for _ in range(128)]
        sd = StateDict(**{f"t{i}": t for i, t in enumerate(ts)})   # 16 GiB
        comp = "hsz1" if what == "take_hsz1" else "none"
        path = os.path.join(args.dir, "iso_take")
        Snapshot.take(path, {"sd": sd}, compression=comp)  # warm (pinned pool, plan)
    elif what == "d2h":
        src = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
        pb = native.PinnedBuffer(256 << 20)
    elif what == "write":
        bufs = [native.PinnedBuffer(64 << 20) for _ in range(16)]
    elif what.startswith("encode"):
        if what == "encode_capped":  # the grid cap an async-take drain uses
            from hipsnapshot import knobs

            native.set_thread_grid_cap(knobs.get_drain_cus())
        x = (torch.randn(128 << 20, device=dev) * 0.02).to(torch.bfloat16).view(torch.uint8)
        s = torch.cuda.Stream()
        codec.encode_device(x, 2, int(s.cuda_stream))
        s.synchronize()
    torch.cuda.synchronize()
    time.sleep(args.lead)
    t0 = time.time()
    t_end = t0 + args.seconds
    moved = 0
    if what == "write":
        stop = threading.Event()
        counts = [0] * 16

        def writer(i):
            p = os.path.join(args.dir, f"iso_w{i}")
            with open(p, "wb") as fh:
                while not stop.is_set():
                    os.pwrite(fh.fileno(), bufs[i].view, 0)
                    counts[i] += 64 << 20

        ths = [threading.Thread(target=writer, args=(i,)) for i in range(16)]
        for th in ths:
            th.start()
        time.sleep(args.seconds)
        stop.set()
        for th in ths:
            th.join()
        moved = sum(counts)
    else:
        while time.time() < t_end:
            if what == "none":
                time.sleep(0.05)
            elif what.startswith("take"):
                Snapshot.take(path, {"sd": sd}, compression=comp)
                moved += 16 << 30
            elif what == "d2h":
                native.sdma_d2h(0, pb.ptr, src.data_ptr(), 256 << 20,
                                torch.cuda.current_stream(dev))
                moved += 256 << 20
            elif what.startswith("encode"):
                codec.encode_device(x, 2, int(s.cuda_stream))
                s.synchronize()
                moved += x.numel()
            n += 1
    t1 = time.time()
    with open(os.path.join(args.out, f"drain_{what}.json"), "w") as f:
        json.dump({"what": what, "start": t0, "end": t1, "GBps": moved / (t1 - t0) / 1e9}, f)


def summarize(args) -> None:
    import statistics

    steps = [json.loads(line) for line in open(os.path.join(args.out, "train.jsonl"))]
    wins = {}
    for name in sorted(os.listdir(args.out)):
        if name.startswith("drain_"):
            w = json.load(open(os.path.join(args.out, name)))
            wins[w["what"]] = w

    def inside(w):
        return [s["dur"] for s in steps
                if s["end"] - s["dur"] >= w["start"] and s["end"] <= w["end"]]

    base = statistics.median(inside(wins.pop("none")))
    for w in wins.values():
        d = inside(w)
        if d:
            m = statistics.mean(d)
            print(json.dumps({"what": w["what"], "load_GBps": round(w["GBps"], 1),
                              "steps_inside": len(d), "step_ms_mean": round(m * 1e3, 1),
                              "step_ms_quiet": round(base * 1e3, 1),
                              "slowdown": round(m / base - 1, 4)}))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", choices=["train", "drain", "summarize"], required=True)
    ap.add_argument("--what", default="take_hsz1",
                    choices=["none", "take_hsz1", "take_raw", "d2h", "write", "encode",
                             "encode_capped"])
    ap.add_argument("--out", default="gpurun_out/iso")
    ap.add_argument("--dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--lead", type=float, default=1.0)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--port", type=int, default=29611)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    {"train": train, "drain": drain, "summarize": summarize}[args.role](args)


if __name__ == "__main__":
    main()
