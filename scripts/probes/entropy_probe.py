"""Bits per bf16 element spent on the high byte (sign + top exponent bits):
entropy vs HSZ1 mode 1 (4-bit nibbles) vs mode 2 (per-frame Huffman), and
the resulting blob ratios of the NumPy reference encoder."""

import numpy as np
import torch

from hipsnapshot.ops import codec


def main():
    n = 1 << 20
    for std in (1 / 64, 0.02, 1.0, 1e-3):
        x = (torch.randn(n) * std).to(torch.bfloat16)
        raw = x.view(torch.uint8).numpy().tobytes()
        hi = np.frombuffer(raw, dtype=np.uint8)[1::2]
        c = np.bincount(hi, minlength=256).astype(float)
        p = c[c > 0] / c.sum()
        ent = -(p * np.log2(p)).sum()
        blob = codec.encode_reference(raw, 2)
        modes = set(codec.frame_modes(blob))
        print(f"std={std:.4g}: H(hi byte)={ent:.3f} bits; blob ratio {len(blob) / len(raw):.4f} "
              f"(modes {sorted(modes)}); entropy bound {(8 + ent) / 16:.4f}")


if __name__ == "__main__":
    main()
