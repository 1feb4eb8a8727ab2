"""HSZ1: lossless exponent-entropy compression for floating-point checkpoint blobs.

Why: a snapshot is bound by bytes moved -- PCIe D2H on one MI355X (57 GB/s
measured), host page-cache bandwidth when 8 ranks write at once.  The high
byte of a bf16/fp16/fp32 weight (sign + top exponent bits) carries ~2.6 bits
of information for trained or initialised weights (measured in
``tests/test_codec.py``), the other bytes are near-random.  HSZ1 keeps the
low bytes verbatim and codes each high byte as a 4-bit index into a per-frame
15-entry dictionary (index 15 = escape, value stored separately): bf16 blobs
shrink to ~75 %, fp32 to ~87.5 %, bit-exactly.  For 2- and 4-byte elements a
frame may instead Huffman-code those 16 indices (mode 2, ~2.7 bits per
element), so bf16 blobs shrink to ~67 % and fp32 to ~83 %.  Frames that do not compress are stored raw, so
any byte stream is accepted.

Encoding and decoding run on the GPU (``csrc/hsz.hip``) before D2H / after
H2D, and on the CPU in C++ (``csrc/hsz_cpu.cpp``).  This module holds the
format definition, a NumPy reference implementation used by the tests (the
native coders must match it byte for byte), and the helpers that parse
headers / map logical byte ranges to frames.

Blob layout (little endian)::

    header   64 B   magic "HSZ1", u32 version, u64 logical_size,
                    u32 elem_width w, u32 frame_bytes F, u32 n_frames, pad
    table    8*(n_frames+1) B   absolute offset of every frame, then the blob size
    frame i  header 32 B  u8 mode (0 raw, 1 nibble, 2 huffman), 3 pad,
                          u32 n_escapes, u8 dict[16],
                          u8 lens[8] (mode 2: code length of index 2j in the
                          low nibble of byte j, of index 2j+1 in the high one)
             mode 0: the frame's logical bytes
             mode 1: nibbles   ceil(n/2) B  (element 2k low nibble, 2k+1 high)
                     low bytes (w-1)*n B   (each element without its high byte)
                     escapes   n_escapes B (high bytes of code-15 elements, in order)
                     tail      (len - n*w) B raw
             mode 2 (w in (2, 4) and n % 8 == 0 only):
                     low bytes (w-1)*n B (each element without its high byte)
                     lane table 256 x u16: byte length of each lane's stream
                     streams   the 256 lane streams back to back; lane t codes
                               the indices of element groups t, t+256, t+512, ...
                               (group g = elements 8g..8g+7) with canonical
                               Huffman codes packed LSB-first (bit-reversed
                               codewords), each stream zero-padded to a byte
                     escapes   n_escapes B (element order), tail (len - n*w) B
             padded to 16 B
    where n = len // w elements of the frame's len logical bytes.

Dictionary: the 15 most frequent high bytes of a deterministic 2048-element
sample of the frame (64 evenly spaced runs of 32 elements, ``sample_indices``;
count descending, value ascending); a frame is coded
only if it has at most ``MAX_ESCAPES`` escapes and the coded size is smaller.
Mode 2 code lengths come from the frame's exact index histogram (Huffman with
deterministic tie-breaks, limited to ``HUFF_MAX_LEN`` bits: ``huffman_lengths``).
The lane split gives one GPU lane one stream to decode while the workgroup's
loads and stores stay coalesced.  Mode 2 is chosen when it is the smallest
encoding and its streams fit in ``HUFF_MAX_CODED`` bytes (LDS-resident on the
GPU).  Version-1 blobs (modes 0/1 only) decode unchanged.

Native decoders take ``count + 1`` frame offsets so every frame's extent is
known and corrupt frame bodies cannot make them read past it.
"""

from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

MAGIC = b"HSZ1"
VERSION = 2
HEADER_BYTES = 64
FRAME_HEADER_BYTES = 32
DEFAULT_FRAME_BYTES = 256 * 1024
SAMPLE = 2048
SAMPLE_RUN = 32  # the sample is SAMPLE // SAMPLE_RUN evenly spaced runs
MAX_ESCAPES = 1024
ESC = 15
CODEC_NAME = "hsz1"
LANES = 256
LANE_TABLE_BYTES = 2 * LANES
HUFF_MAX_LEN = 11
HUFF_MAX_CODED = 65535


def _align16(n: int) -> int:
    return (n + 15) & ~15


def table_bytes(n_frames: int) -> int:
    return 8 * (n_frames + 1)


def payload_start(n_frames: int) -> int:
    return _align16(HEADER_BYTES + table_bytes(n_frames))


def n_frames_for(logical: int, frame_bytes: int) -> int:
    return max(1, (logical + frame_bytes - 1) // frame_bytes)


def max_encoded_bytes(logical: int, frame_bytes: int = DEFAULT_FRAME_BYTES) -> int:
    """Worst case (every frame raw): capacity to allocate for an encoder."""
    nf = n_frames_for(logical, frame_bytes)
    return payload_start(nf) + nf * _align16(FRAME_HEADER_BYTES + frame_bytes)


@dataclass
class Header:
    logical_size: int
    elem_width: int
    frame_bytes: int
    n_frames: int
    offsets: List[int]  # n_frames + 1 absolute offsets

    def frame_range(self, i: int) -> Tuple[int, int]:
        lo = i * self.frame_bytes
        return lo, min(lo + self.frame_bytes, self.logical_size)

    def frames_covering(self, lo: int, hi: int) -> Tuple[int, int]:
        """[first, last) frame indices covering logical bytes [lo, hi)."""
        if hi <= lo:
            return 0, 0
        return lo // self.frame_bytes, (hi - 1) // self.frame_bytes + 1


def parse_header(buf) -> Header:
    mv = memoryview(buf).cast("B")
    if bytes(mv[:4]) != MAGIC:
        raise ValueError("not an HSZ1 blob")
    version, logical, w, fb, nf = struct.unpack_from("<IQIII", mv, 4)
    if version not in (1, VERSION):
        raise ValueError(f"unsupported HSZ1 version {version}")
    need = HEADER_BYTES + table_bytes(nf)
    if len(mv) < need:
        raise ValueError(f"HSZ1 header truncated: need {need} bytes")
    offs = list(struct.unpack_from(f"<{nf + 1}Q", mv, HEADER_BYTES))
    return Header(logical, w, fb, nf, offs)


def header_probe_bytes(max_frames: int = 4096) -> int:
    """Bytes to read to be sure to get the header of most blobs in one read."""
    return HEADER_BYTES + table_bytes(max_frames)


# ---------------------------------------------------------------------------
# Huffman code construction (mirrored exactly by csrc/hsz_cpu.cpp and hsz.hip)
# ---------------------------------------------------------------------------

def huffman_lengths(counts) -> List[int]:
    """Code lengths for the 16 dictionary indices from their counts.

    Huffman merges the two lightest live nodes, ties going to the lower node
    index (leaves are numbered by ascending index value, merged nodes after
    them in creation order).  If the longest code exceeds ``HUFF_MAX_LEN``,
    every length is clamped and, while the Kraft sum exceeds 1, the longest
    code shorter than the limit is lengthened by one (ties: the rarer index,
    then the larger index).  A single used index gets length 1.
    """
    cnt = [int(c) for c in counts]
    active = [c for c in range(16) if cnt[c] > 0]
    lens = [0] * 16
    if not active:
        return lens
    if len(active) == 1:
        lens[active[0]] = 1
        return lens
    weight = [cnt[c] for c in active]
    parent = [-1] * len(active)
    alive = list(range(len(active)))
    while len(alive) > 1:
        a = min(alive, key=lambda i: (weight[i], i))
        alive.remove(a)
        b = min(alive, key=lambda i: (weight[i], i))
        alive.remove(b)
        weight.append(weight[a] + weight[b])
        parent.append(-1)
        parent[a] = parent[b] = len(weight) - 1
        alive.append(len(weight) - 1)
    for i, c in enumerate(active):
        d, j = 0, i
        while parent[j] != -1:
            j = parent[j]
            d += 1
        lens[c] = d
    if max(lens) > HUFF_MAX_LEN:
        lens = [min(x, HUFF_MAX_LEN) for x in lens]
        while sum(1 << (HUFF_MAX_LEN - lens[c]) for c in active) > (1 << HUFF_MAX_LEN):
            s = max((c for c in active if lens[c] < HUFF_MAX_LEN),
                    key=lambda c: (lens[c], -cnt[c], c))
            lens[s] += 1
    return lens


def canonical_codes(lens) -> List[int]:
    """Bit-reversed canonical codewords (LSB-first emission) for ``lens``."""
    codes = [0] * 16
    code, prev, first = 0, 0, True
    for ln in range(1, HUFF_MAX_LEN + 1):
        for c in range(16):
            if lens[c] != ln:
                continue
            if not first:
                code = (code + 1) << (ln - prev)
            first = False
            prev = ln
            rev = 0
            for k in range(ln):
                rev |= ((code >> k) & 1) << (ln - 1 - k)
            codes[c] = rev
    return codes


def decode_table(lens) -> np.ndarray:
    """2^HUFF_MAX_LEN-entry LUT: bits 0-3 index, bits 8+ code length (0 = invalid)."""
    codes = canonical_codes(lens)
    lut = np.zeros(1 << HUFF_MAX_LEN, dtype=np.uint16)
    x = np.arange(1 << HUFF_MAX_LEN)
    for c in range(16):
        if lens[c]:
            hit = (x & ((1 << lens[c]) - 1)) == codes[c]
            lut[hit] = c | (lens[c] << 8)
    return lut


# ---------------------------------------------------------------------------
# NumPy reference (the GPU and C++ implementations must match it bit for bit)
# ---------------------------------------------------------------------------

def sample_indices(n: int) -> np.ndarray:
    """Elements of an n-element frame that choose its dictionary: all of them
    up to ``SAMPLE``, else ``SAMPLE // SAMPLE_RUN`` runs of ``SAMPLE_RUN``
    consecutive elements, run r starting at r * (n // runs).  Runs instead of
    single strided elements: the GPU's sample loads are coalesced (2 lines
    per run) instead of 2048 separate lines, which made the sample phase
    latency-bound."""
    if n <= SAMPLE:
        return np.arange(n)
    i = np.arange(SAMPLE)
    return (i // SAMPLE_RUN) * (n // (SAMPLE // SAMPLE_RUN)) + i % SAMPLE_RUN


def _frame_dict(hi: np.ndarray) -> np.ndarray:
    sample = hi[sample_indices(hi.size)]
    counts = np.bincount(sample, minlength=256)
    order = sorted(range(256), key=lambda v: (-int(counts[v]), v))
    chosen = [v for v in order[:15] if counts[v] > 0]
    d = np.zeros(16, dtype=np.uint8)
    d[: len(chosen)] = chosen
    return d, len(chosen)


def _raw_frame(data: np.ndarray) -> bytes:
    return struct.pack("<B3xI16s8x", 0, 0, bytes(16)) + data.tobytes()


def _lane_layout(codes: np.ndarray, lens: List[int]):
    """Stream order and bit offsets of a mode-2 frame's codes.

    Returns (order, bit_offset, code_length, lane_bytes): ``order`` lists the
    element indices in stream order (lane, then group, then position in the
    group) and ``bit_offset`` is each one's first bit in the concatenated,
    byte-padded lane streams."""
    g = codes.size // 8
    grp = np.arange(g)
    lane_of_group = grp % LANES
    grp_order = np.lexsort((grp, lane_of_group))
    order = (grp_order[:, None] * 8 + np.arange(8)[None, :]).reshape(-1)
    ln = np.asarray(lens, dtype=np.int64)[codes[order]]
    lane_of_el = lane_of_group[order // 8]
    lane_bits = np.bincount(lane_of_el, weights=ln, minlength=LANES).astype(np.int64)
    lane_bytes = (lane_bits + 7) // 8
    lane_start_bit = np.concatenate([[0], np.cumsum(lane_bytes)[:-1]]) * 8
    excl = np.concatenate([[0], np.cumsum(ln)])
    lane_first = np.concatenate([[0], np.cumsum(np.bincount(lane_of_el, minlength=LANES))[:-1]])
    bit_off = lane_start_bit[lane_of_el] + excl[:-1] - excl[lane_first][lane_of_el]
    return order, bit_off, ln, lane_bytes


def _huffman_streams(codes: np.ndarray, lens: List[int]) -> Tuple[bytes, np.ndarray]:
    order, bit_off, ln, lane_bytes = _lane_layout(codes, lens)
    bits = np.zeros(int(lane_bytes.sum()) * 8, dtype=np.uint8)
    rev = np.asarray(canonical_codes(lens), dtype=np.int64)[codes[order]]
    for k in range(HUFF_MAX_LEN):
        m = ln > k
        bits[bit_off[m] + k] = (rev[m] >> k) & 1
    return np.packbits(bits, bitorder="little").tobytes(), lane_bytes


def _encode_frame(data: np.ndarray, w: int) -> bytes:
    length = data.size
    n = length // w
    raw = FRAME_HEADER_BYTES + length
    if n == 0:
        return _raw_frame(data)
    el = data[: n * w].reshape(n, w)
    hi = el[:, w - 1]
    d, k = _frame_dict(hi)
    code_of = np.full(256, ESC, dtype=np.uint8)
    code_of[d[:k]] = np.arange(k, dtype=np.uint8)
    codes = code_of[hi]
    esc_mask = codes == ESC
    n_esc = int(esc_mask.sum())
    tail = length - n * w
    coded = FRAME_HEADER_BYTES + (n + 1) // 2 + (w - 1) * n + n_esc + tail
    if n_esc > MAX_ESCAPES:
        return _raw_frame(data)
    esc = hi[esc_mask]
    if w in (2, 4) and n % 8 == 0:
        lens = huffman_lengths(np.bincount(codes, minlength=16))
        c_bytes = int(_lane_layout(codes, lens)[3].sum())
        size2 = FRAME_HEADER_BYTES + (w - 1) * n + LANE_TABLE_BYTES + c_bytes + n_esc + tail
        if c_bytes <= HUFF_MAX_CODED and size2 < coded and size2 < raw:
            streams, lane_bytes = _huffman_streams(codes, lens)
            lens_b = bytes(lens[2 * j] | (lens[2 * j + 1] << 4) for j in range(8))
            lo = np.ascontiguousarray(el[:, : w - 1]).reshape(-1)
            return (struct.pack("<B3xI16s8s", 2, n_esc, d.tobytes(), lens_b)
                    + lo.tobytes() + lane_bytes.astype("<u2").tobytes() + streams
                    + esc.tobytes() + data[n * w:].tobytes())
    if coded >= raw:
        return _raw_frame(data)
    if n % 2:
        codes = np.concatenate([codes, np.zeros(1, dtype=np.uint8)])
    nib = (codes[0::2] | (codes[1::2] << 4)).astype(np.uint8)
    lo = np.ascontiguousarray(el[:, : w - 1]).reshape(-1)
    return (struct.pack("<B3xI16s8x", 1, n_esc, d.tobytes()) + nib.tobytes() + lo.tobytes()
            + esc.tobytes() + data[n * w:].tobytes())


def encode_reference(data, elem_width: int = 2,
                     frame_bytes: int = DEFAULT_FRAME_BYTES) -> bytes:
    src = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    logical = src.size
    assert frame_bytes % 16 == 0 and frame_bytes % elem_width == 0
    nf = n_frames_for(logical, frame_bytes)
    frames = []
    for i in range(nf):
        f = _encode_frame(src[i * frame_bytes: (i + 1) * frame_bytes], elem_width)
        frames.append(f + bytes(_align16(len(f)) - len(f)))
    start = payload_start(nf)
    offs = [start]
    for f in frames:
        offs.append(offs[-1] + len(f))
    head = struct.pack("<4sIQIII", MAGIC, VERSION, logical, elem_width, frame_bytes, nf)
    head += bytes(HEADER_BYTES - len(head))
    table = struct.pack(f"<{nf + 1}Q", *offs)
    pad = bytes(start - HEADER_BYTES - len(table))
    return head + table + pad + b"".join(frames)


def _decode_huffman_streams(streams: np.ndarray, lane_bytes: np.ndarray, n: int,
                            lens: List[int]) -> np.ndarray:
    """All 256 lane streams decoded in lock step (vectorised over lanes)."""
    g = n // 8
    lut = decode_table(lens)
    buf = np.concatenate([streams, np.zeros(4, dtype=np.uint8)]).astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(lane_bytes.astype(np.int64))[:-1]])
    bitpos = starts * 8
    ends = (starts + lane_bytes.astype(np.int64)) * 8
    codes = np.zeros(n, dtype=np.uint8)
    lanes = np.arange(LANES)
    for s in range((g + LANES - 1) // LANES):
        grp = s * LANES + lanes
        live = grp < g
        for e in range(8):
            p = np.minimum(bitpos, buf.size * 8 - 24)
            byte = p >> 3
            word = buf[byte] | (buf[byte + 1] << 8) | (buf[byte + 2] << 16)
            ent = lut[(word >> (p & 7)) & ((1 << HUFF_MAX_LEN) - 1)]
            ln = (ent >> 8).astype(np.int64)
            if np.any(live & ((ln == 0) | (bitpos + ln > ends))):
                raise ValueError("corrupt HSZ1 huffman stream")
            codes[grp[live] * 8 + e] = (ent[live] & 15).astype(np.uint8)
            bitpos = np.where(live, bitpos + ln, bitpos)
    return codes


def decode_frame_reference(frame, length: int, w: int) -> bytes:
    mv = memoryview(frame).cast("B")
    mode, n_esc, d, lens_b = struct.unpack_from("<B3xI16s8s", mv, 0)
    body = np.frombuffer(mv[FRAME_HEADER_BYTES:], dtype=np.uint8)
    if mode == 0:
        return body[:length].tobytes()
    n = length // w
    dic = np.frombuffer(d, dtype=np.uint8)
    if mode == 2:
        lens = [(lens_b[j // 2] >> (4 * (j % 2))) & 15 for j in range(16)]
        nlo = (w - 1) * n
        lo = body[:nlo].reshape(n, w - 1)
        lane_bytes = body[nlo: nlo + LANE_TABLE_BYTES].view("<u2")
        c_bytes = int(lane_bytes.astype(np.int64).sum())
        s0 = nlo + LANE_TABLE_BYTES
        codes = _decode_huffman_streams(body[s0: s0 + c_bytes], lane_bytes, n, lens)
        esc = body[s0 + c_bytes: s0 + c_bytes + n_esc]
        hi = dic[np.minimum(codes, 14)].copy()
        hi[codes == ESC] = esc
        out = np.empty((n, w), dtype=np.uint8)
        out[:, : w - 1] = lo
        out[:, w - 1] = hi
        tail = body[s0 + c_bytes + n_esc: s0 + c_bytes + n_esc + (length - w * n)]
        return out.tobytes() + tail.tobytes()
    nb = (n + 1) // 2
    nib = body[:nb]
    codes = np.empty(nb * 2, dtype=np.uint8)
    codes[0::2] = nib & 15
    codes[1::2] = nib >> 4
    codes = codes[:n]
    lo = body[nb: nb + (w - 1) * n].reshape(n, w - 1)
    esc = body[nb + (w - 1) * n: nb + (w - 1) * n + n_esc]
    hi = dic[np.minimum(codes, 14)].copy()
    hi[codes == ESC] = esc
    out = np.empty((n, w), dtype=np.uint8)
    out[:, : w - 1] = lo
    out[:, w - 1] = hi
    tail = body[nb + (w - 1) * n + n_esc: nb + (w - 1) * n + n_esc + (length - n * w)]
    return out.tobytes() + tail.tobytes()


def decode_reference(blob) -> bytes:
    mv = memoryview(blob).cast("B")
    h = parse_header(mv)
    out = []
    for i in range(h.n_frames):
        lo, hi = h.frame_range(i)
        out.append(decode_frame_reference(mv[h.offsets[i]: h.offsets[i + 1]], hi - lo,
                                          h.elem_width))
    return b"".join(out)


def frame_modes(blob) -> List[int]:
    """Mode byte of every frame (diagnostics / tests)."""
    mv = memoryview(blob).cast("B")
    h = parse_header(mv)
    return [mv[h.offsets[i]] for i in range(h.n_frames)]


# ---------------------------------------------------------------------------
# native implementations (C++ host, HIP device)
# ---------------------------------------------------------------------------

def encode_cpu(data, elem_width: int = 2, frame_bytes: int = DEFAULT_FRAME_BYTES,
               nthreads: int = 8) -> np.ndarray:
    """C++ encoder; returns the blob as a uint8 array."""
    from . import native

    src = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    out = np.empty(native.hsz_max_encoded_bytes(src.size, frame_bytes), dtype=np.uint8)
    n = native.hsz_encode_cpu(src.ctypes.data if src.size else out.ctypes.data, src.size,
                              elem_width, frame_bytes, out.ctypes.data, nthreads)
    return out[:n]


def decode_cpu_into(blob, out_addr: int, first: int = 0, count: int = None,
                    header: Header = None, nthreads: int = 8) -> None:
    """C++ decoder of frames [first, first+count) of a whole ``blob`` into out_addr."""
    from . import native

    mv = memoryview(blob).cast("B")
    h = header or parse_header(mv)
    count = h.n_frames - first if count is None else count
    arr = np.frombuffer(mv, dtype=np.uint8)
    offs = np.asarray(h.offsets[first: first + count + 1], dtype=np.uint64)
    validate_offsets(h, len(mv))
    native.hsz_decode_cpu(arr.ctypes.data, offs.ctypes.data, first, count, h.logical_size,
                          h.elem_width, h.frame_bytes, out_addr, nthreads)


def decode_cpu(blob) -> np.ndarray:
    h = parse_header(blob)
    out = np.empty(max(h.logical_size, 1), dtype=np.uint8)
    decode_cpu_into(blob, out.ctypes.data, header=h)
    return out[: h.logical_size]


def validate_offsets(h: Header, blob_len: int) -> None:
    """Reject corrupt frame tables before any native decoder walks them."""
    offs = h.offsets
    if len(offs) != h.n_frames + 1 or offs[-1] > blob_len:
        raise ValueError("HSZ1 frame table out of range")
    for i in range(h.n_frames):
        lo, hi = h.frame_range(i)
        if offs[i + 1] < offs[i] + FRAME_HEADER_BYTES or offs[i + 1] - offs[i] > \
                _align16(FRAME_HEADER_BYTES + (hi - lo)):
            raise ValueError(f"HSZ1 frame {i} has an invalid size")


def encode_device(src, elem_width: int, stream_handle: int,
                  frame_bytes: int = DEFAULT_FRAME_BYTES, launch: bool = True):
    """Encode a contiguous CUDA uint8 tensor on the GPU.

    Returns ``(blob_tensor, nbytes_device, meta)``: ``blob_tensor`` has the
    worst-case capacity and ``nbytes_device`` is a 1-element uint64-as-int64
    CUDA tensor with the encoded size; everything is enqueued on
    ``stream_handle`` (the caller reads the size after synchronising).
    """
    import torch

    from . import native

    logical = src.numel()
    nf = n_frames_for(logical, frame_bytes)
    out = torch.empty(max_encoded_bytes(logical, frame_bytes), dtype=torch.uint8,
                      device=src.device)
    meta = torch.empty(native.hsz_meta_bytes(nf), dtype=torch.uint8, device=src.device)
    total = torch.empty(1, dtype=torch.int64, device=src.device)
    if launch:
        launch_encode(src, elem_width, stream_handle, frame_bytes, out, total, meta)
    return out, total, meta


def launch_encode(src, elem_width: int, stream_handle: int, frame_bytes: int, out, total,
                  meta) -> None:
    import torch

    from . import native

    dev = src.device.index if src.device.index is not None else torch.cuda.current_device()
    src_addr = src.data_ptr() if src.numel() else out.data_ptr()
    native.hsz_encode_gpu(dev, src_addr, src.numel(), elem_width, frame_bytes, out.data_ptr(),
                          meta.data_ptr(), total.data_ptr(), stream_handle)


def decode_device_into(blob_dev, header: Header, out_dev, stream_handle: int,
                       first: int = 0, count: int = None, blob_base: int = 0) -> None:
    """Decode frames of a blob already in device memory into ``out_dev``.

    ``blob_dev``: CUDA uint8 tensor holding bytes [blob_base, ...) of the blob
    (the whole blob when ``blob_base`` is 0).  ``out_dev`` receives the logical
    bytes of frames [first, first+count).
    """
    import torch

    from . import native

    count = header.n_frames - first if count is None else count
    if count <= 0:
        return
    offs = [o - blob_base for o in header.offsets[first: first + count + 1]]
    if min(offs) < 0 or offs[-1] > blob_dev.numel():
        raise ValueError("HSZ1 frames outside the device buffer")
    dev = blob_dev.device.index if blob_dev.device.index is not None else \
        torch.cuda.current_device()
    offs_t = torch.tensor(offs, dtype=torch.int64).to(blob_dev.device, non_blocking=False)
    err = native.DecodeErrorWord()
    native.hsz_decode_gpu(dev, blob_dev.data_ptr(), offs_t.data_ptr(), first, count,
                          header.logical_size, header.elem_width, header.frame_bytes,
                          out_dev.data_ptr(), stream_handle, err.addr)
    # keep the offsets alive until the kernel ran
    torch.cuda.ExternalStream(stream_handle).synchronize() if stream_handle else \
        torch.cuda.synchronize(dev)
    err.check(f"frames [{first}, {first + count})")
