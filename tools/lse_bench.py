"""Diagnostic: rtkv_attention_lse at the cfg3 shape (B = 1, H = 32, S = 16384, D = 128, fp16,
causal) — µs per layer and MFMA TFLOP/s of the Q·Kᵀ work (S²/2·H·D·2 flops)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "realtime-kv-cache-compression_amd"))
import rtkv  # noqa: E402

rtkv.build()
for S in (4096, 16384):
    B, H, D = 1, 32, 128
    Q = torch.randn(B, H, S, D, device="cuda").half()
    K = torch.randn(B, H, S, D, device="cuda").half()
    for _ in range(3):
        rtkv.attention_lse(Q, K)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        rtkv.attention_lse(Q, K)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    fl = S * (S + 1) / 2 * H * D * 2
    print(f"S={S}: {us:.1f} us, {fl / us / 1e6:.1f} TFLOP/s (QK only)", flush=True)
