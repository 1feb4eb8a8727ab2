#!/usr/bin/env python3
"""Data-plane microbenchmarks on one MI355X (prints one JSON line per test).

* d2h_sdma      : hipMemcpyAsync D2H into the pinned pool, 1 and 4 streams
* d2h_kernel    : hs_copy_nd storing straight into host-mapped pinned memory
* d2h_torch     : torch ``.cpu()`` (pageable; what the reference does)
* gather_hbm    : hs_copy_nd multi-tensor gather, HBM -> HBM (GB/s of payload)
* pack_strided  : hs_copy_nd strided (transposed) -> contiguous, HBM -> HBM
* fs_write      : native engine pwrite of pinned buffers (buffered / O_DIRECT)
"""

from __future__ import annotations

import argparse
import json
import os
import threading
import time

import torch

from hipsnapshot.ops import native


def emit(**kw):
    print(json.dumps(kw), flush=True)


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts), sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1024)
    ap.add_argument("--dir", default="/tmp/hs_micro")
    ap.add_argument("--skip-fs", action="store_true")
    args = ap.parse_args()
    dev = 0
    n = args.mb << 20
    src = torch.empty(n, dtype=torch.uint8, device="cuda:0").random_(0, 255)
    pb = native.PinnedBuffer(n)

    def sdma1():
        native.memcpy(dev, 0, pb.ptr, src.data_ptr(), n, native.D2H, None, sync=True)

    best, med = timeit(sdma1)
    emit(test="d2h_sdma_1stream", GBps=n / best / 1e9, median_GBps=n / med / 1e9, bytes=n)

    def sdma4():
        q = n // 4
        th = [threading.Thread(target=native.memcpy,
                               args=(dev, i, pb.ptr + i * q, src.data_ptr() + i * q, q,
                                     native.D2H, None, True)) for i in range(4)]
        [t.start() for t in th]
        [t.join() for t in th]

    best, med = timeit(sdma4)
    emit(test="d2h_sdma_4stream", GBps=n / best / 1e9, median_GBps=n / med / 1e9)

    stream = native.copy_stream(dev, 0)

    def kern():
        b = native.CopyBatch()
        b.add(src.data_ptr(), torch.uint8, [1], pb.ptr, torch.uint8, [1], [n], 1)
        b.launch(dev, stream, sync=True)

    best, med = timeit(kern)
    emit(test="d2h_kernel_hostmapped", GBps=n / best / 1e9, median_GBps=n / med / 1e9)

    def tcpu():
        src.cpu()

    best, med = timeit(tcpu, 3)
    emit(test="d2h_torch_pageable", GBps=n / best / 1e9, median_GBps=n / med / 1e9)

    # H2D
    def h2d():
        native.memcpy(dev, 0, src.data_ptr(), pb.ptr, n, native.H2D, None, sync=True)

    best, med = timeit(h2d)
    emit(test="h2d_sdma_1stream", GBps=n / best / 1e9, median_GBps=n / med / 1e9)

    # multi-tensor gather HBM->HBM: 2000 tensors of mixed sizes
    sizes = [(4096 * 4096 * 2) if i % 10 == 0 else (4096 * 2 * (1 + i % 7)) for i in range(2000)]
    ts = [torch.empty(s // 2, dtype=torch.bfloat16, device="cuda:0").normal_() for s in sizes]
    total = sum(sizes)
    dst = torch.empty(total + 256 * len(ts), dtype=torch.uint8, device="cuda:0")
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += (s + 255) // 256 * 256

    def gather():
        b = native.CopyBatch()
        for t, off in zip(ts, offs):
            b.add(t.data_ptr(), t.dtype, [1], dst.data_ptr() + off, t.dtype, [1], [t.numel()], 2)
        b.launch(dev, int(torch.cuda.current_stream().cuda_stream), sync=True)

    best, med = timeit(gather)
    emit(test="gather_hbm_2000_tensors", GBps=total / best / 1e9, median_GBps=total / med / 1e9,
         bytes=total, note="payload bytes/s (read+write = 2x)")

    def torch_gather():
        for t, off in zip(ts, offs):
            dst[off:off + t.numel() * 2].view(torch.bfloat16).copy_(t)

    best, med = timeit(torch_gather, 3)
    emit(test="gather_hbm_torch_copy_loop", GBps=total / best / 1e9, median_GBps=total / med / 1e9)

    # GPU time of the copy kernel alone (descriptor tables pre-built): one
    # 1 GiB contiguous copy, and a Llama-3-8B-like freeze (291 tensors, 16 GB
    # -> arena) as the async_take HBM freeze issues it
    def gpu_ms(batch, dst_keep):
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(4):
            keep = batch.launch(dev, int(st.cuda_stream), sync=False)
            st.synchronize()
            del keep
        for _ in range(5):
            e0.record(st)
            keep = batch.launch(dev, int(st.cuda_stream), sync=False)
            e1.record(st)
            st.synchronize()
            del keep
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best

    big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")
    big2 = torch.empty_like(big)
    b1 = native.CopyBatch()
    b1.add_bytes(big.data_ptr(), big2.data_ptr(), big.numel())
    ms = gpu_ms(b1, big2)
    emit(test="copy_nd_contig_1GiB_gpu_time", GBps=big.numel() / ms / 1e6, ms=ms,
         note="payload bytes/s; HBM traffic 2x")
    del big, big2
    shapes = [(128256, 4096), (128256, 4096)] + [(4096, 4096), (1024, 4096), (1024, 4096),
                                                 (4096, 4096), (14336, 4096), (4096, 14336),
                                                 (14336, 4096), (4096,), (4096,)] * 32 + [(4096,)]
    ws_ = [torch.empty(sh, dtype=torch.bfloat16, device="cuda:0") for sh in shapes]
    tot = sum(w.numel() * 2 for w in ws_)
    arena = torch.empty(tot + 256 * len(ws_), dtype=torch.uint8, device="cuda:0")
    bf = native.CopyBatch()
    off = 0
    for w in ws_:
        bf.add_tensor(w, arena.data_ptr() + off)
        off += (w.numel() * 2 + 255) // 256 * 256
    ms = gpu_ms(bf, arena)
    emit(test="freeze_llama3_8b_291_tensors_gpu_time", GBps=tot / ms / 1e6, ms=ms, bytes=tot,
         note="payload bytes/s; the trainer's stream waits this long after async_take")
    tt = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tt[0].record()
    for w in ws_:
        arena[:w.numel() * 2].view(torch.bfloat16).view(w.shape).copy_(w)
    tt[1].record()
    torch.cuda.synchronize()
    emit(test="freeze_llama3_8b_torch_copy_loop_gpu_time", ms=tt[0].elapsed_time(tt[1]),
         GBps=tot / tt[0].elapsed_time(tt[1]) / 1e6)
    del ws_, arena

    # strided pack: transpose view of 8192x8192 bf16
    a = torch.empty(8192, 8192, dtype=torch.bfloat16, device="cuda:0").normal_()
    at = a.t()
    out = torch.empty(8192 * 8192, dtype=torch.bfloat16, device="cuda:0")

    def pack():
        b = native.CopyBatch()
        b.add(at.data_ptr(), at.dtype, at.stride(), out.data_ptr(), at.dtype, [8192, 1],
              [8192, 8192], 2)
        b.launch(dev, int(torch.cuda.current_stream().cuda_stream), sync=True)

    best, med = timeit(pack)
    nb = a.numel() * 2
    emit(test="pack_transpose_8192sq_bf16", GBps=nb / best / 1e9, median_GBps=nb / med / 1e9)
    assert torch.equal(out.view(8192, 8192), at.contiguous())

    def tpack():
        out.view(8192, 8192).copy_(at)

    best, med = timeit(tpack)
    emit(test="pack_transpose_torch", GBps=nb / best / 1e9, median_GBps=nb / med / 1e9)

    # column shard (narrow on dim 1) pack
    col = a[:, 1024:3072]
    out2 = torch.empty(col.numel(), dtype=torch.bfloat16, device="cuda:0")

    def colpack():
        b = native.CopyBatch()
        b.add(col.data_ptr(), col.dtype, col.stride(), out2.data_ptr(), col.dtype, [2048, 1],
              list(col.shape), 2)
        b.launch(dev, int(torch.cuda.current_stream().cuda_stream), sync=True)

    best, med = timeit(colpack)
    nb2 = col.numel() * 2
    emit(test="pack_column_shard_bf16", GBps=nb2 / best / 1e9, median_GBps=nb2 / med / 1e9)
    assert torch.equal(out2.view(col.shape), col.contiguous())

    # fp8 quantization of a 1 GiB bf16 tensor: MX (E8M0 scale per 32, the
    # default), fp32 scale per 128, and the MFMA Hadamard-32 variant
    from hipsnapshot.ops import quant

    w = torch.empty(512 << 20, dtype=torch.bfloat16, device="cuda:0").normal_()
    nw = w.numel()
    hs = int(torch.cuda.current_stream().cuda_stream)
    for mode in ("mx_e8m0", "none", "hadamard32"):
        if mode == "mx_e8m0":
            info = quant.fp8_entry_quant_info(w, rotation="none")
            assert quant.is_mx(info)
        else:
            os.environ["HIPSNAPSHOT_FP8_FORMAT"] = "block"
            info = quant.fp8_entry_quant_info(w, rotation=mode)
            del os.environ["HIPSNAPSHOT_FP8_FORMAT"]
        blob = torch.zeros(info["total_bytes"], dtype=torch.uint8, device="cuda:0")
        payload = info["payload_bytes"]
        scales = blob[payload:] if mode == "mx_e8m0" else blob[payload:].view(torch.float32)
        back = torch.empty_like(w)

        def q():
            if mode == "mx_e8m0":
                native.mx8_quantize(dev, w, blob[:payload], scales, hs)
            elif mode == "none":
                native.fp8_quantize(dev, w, blob[:payload], scales, info["vpt"], hs)
            else:
                native.fp8_hadamard_quantize(dev, w, blob[:payload], scales, hs)

        def dq():
            if mode == "mx_e8m0":
                native.mx8_dequantize(dev, blob[:nw], scales, back, hs)
            elif mode == "none":
                native.fp8_dequantize(dev, blob[:nw], scales, back, info["vpt"], hs)
            else:
                native.fp8_hadamard_dequantize(dev, blob[:payload], scales, back, hs)

        best, med = timeit(q)
        traffic = nw * 2 + info["total_bytes"]
        emit(test=f"fp8_quant_{mode}_1GiB_bf16", GBps=traffic / best / 1e9,
             median_GBps=traffic / med / 1e9, ms=best * 1e3, note="HBM bytes read+written")
        best, med = timeit(dq)
        emit(test=f"fp8_dequant_{mode}_1GiB_bf16", GBps=traffic / best / 1e9,
             median_GBps=traffic / med / 1e9, ms=best * 1e3)
        del blob, back
    del w

    # HSZ1 lossless codec: encode (4 launches) and decode of 1 GiB bf16 / fp32 in HBM
    from hipsnapshot.ops import codec

    for name, dt, w in (("bf16", torch.bfloat16, 2), ("fp32", torch.float32, 4)):
        x = (torch.randn((1 << 30) // w, device="cuda:0") / 64).to(dt).view(torch.uint8)
        st = torch.cuda.current_stream()
        out, total, meta = codec.encode_device(x, w, int(st.cuda_stream))
        st.synchronize()
        nb = int(total.item())
        nf = codec.n_frames_for(x.numel(), codec.DEFAULT_FRAME_BYTES)
        hdr = codec.parse_header(out[:codec.payload_start(nf)].cpu().numpy().tobytes())
        offs = torch.tensor(hdr.offsets, dtype=torch.int64, device="cuda:0")
        back = torch.empty_like(x)

        def enc():
            codec.launch_encode(x, w, int(st.cuda_stream), codec.DEFAULT_FRAME_BYTES, out, total,
                                meta)

        def dec():
            native.hsz_decode_gpu(dev, out.data_ptr(), offs.data_ptr(), 0, hdr.n_frames,
                                  hdr.logical_size, w, hdr.frame_bytes, back.data_ptr(),
                                  int(st.cuda_stream))

        best, med = timeit(enc)
        emit(test=f"hsz_encode_1GiB_{name}", GBps=x.numel() / best / 1e9,
             median_GBps=x.numel() / med / 1e9, ms=best * 1e3, ratio=nb / x.numel(),
             note="logical bytes/s; HBM traffic = 2 reads + ratio write")
        best, med = timeit(dec)
        emit(test=f"hsz_decode_1GiB_{name}", GBps=x.numel() / best / 1e9,
             median_GBps=x.numel() / med / 1e9, ms=best * 1e3)
        assert torch.equal(back, x)
        del x, out, back, meta, offs

    if not args.skip_fs:
        os.makedirs(args.dir, exist_ok=True)
        eng = native.IOEngine(16)
        nfiles = 16
        per = 256 << 20
        bufs = [native.PinnedBuffer(per) for _ in range(nfiles)]
        for direct in (0, 1):
            flags = native.IO_MKDIRS | (native.IO_DIRECT if direct else 0)
            t0 = time.perf_counter()
            ids = [eng.submit_write(f"{args.dir}/f{i}", b.ptr, per, 0, flags)
                   for i, b in enumerate(bufs)]
            done = 0
            while done < len(ids):
                r = eng.poll()
                for _, res in r:
                    assert res >= 0, res
                done += len(r)
                if not r:
                    time.sleep(0.0005)
            dt = time.perf_counter() - t0
            emit(test="fs_write_16x256MB", direct=direct, GBps=nfiles * per / dt / 1e9)
        import shutil

        shutil.rmtree(args.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
