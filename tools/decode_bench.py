"""Diagnostic (not part of the product): decode-step attention over a packed layer
(rtkv_decode_attention_packed) against torch SDPA over the dense dequantized K'/V' the reference
keeps (modified_llama.py:140-142), on a cfg3-shaped layer (B = 1, S = 16384, Hkv = 32, D = 128 f16,
ratio 0.6, bits 2/4/8) and Llama-3-8B-shaped GQA (Hkv = 8).  Prints µs per step and the algorithmic
HBM bytes / time (packed codes + per-row scale/zp + kept_index / row_offset + labels gather)."""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "realtime-kv-cache-compression_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests", "golden"))
import rtkv  # noqa: E402
import synth  # noqa: E402


TD = {"float16": torch.float16, "bfloat16": torch.bfloat16}


def dev(stored, dtype):
    return torch.from_numpy(np.ascontiguousarray(stored, np.uint16).view(np.int16)).cuda().view(TD[dtype])


def run(S, Hkv, Hq, dtype="float16", D=128, ratio=0.6, iters=200):
    F = Hkv * D
    K, V = synth.kv(11, 1, S, F, dtype)
    W = synth.attention_slice(11, 1, 8, S, rtkv.prompt_length(S), dtype)
    cfg = rtkv.CompressionConfig(num_hidden_layers=4, low_precision_bits=2, medium_precision_bits=4,
                                 high_precision_bits=8, early_layer_ratio=ratio, middle_layer_ratio=ratio,
                                 later_layer_ratio=ratio)
    comp = rtkv.RealTimePrefillCompressor(cfg)
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    k2, v2, info = comp.compress_layer_kv_cache(dev(K, dtype), dev(V, dtype), dev(W, dtype), ids, 1)
    pk = info["packed"]
    n = int(pk["rows"][0])
    q = torch.randn(1, Hq, D, device="cuda").to(TD[dtype])
    for _ in range(10):
        rtkv.decode_attention(pk, q, Hkv)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        rtkv.decode_attention(pk, q, Hkv)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    code_bytes = 2 * pk["codes_k"].numel()
    meta = n * (16 + 4 + 8 + 1)
    by = code_bytes + meta + q.numel() * 2 + Hq * D * 4
    # dense baseline: SDPA over the dequantized rows (GQA expanded as the reference's repeat_kv does)
    kd = k2[:, :n].view(1, n, Hkv, D).transpose(1, 2)
    vd = v2[:, :n].view(1, n, Hkv, D).transpose(1, 2)
    kd = kd.repeat_interleave(Hq // Hkv, 1).contiguous()
    vd = vd.repeat_interleave(Hq // Hkv, 1).contiguous()
    qq = q.view(1, Hq, 1, D)
    for _ in range(10):
        torch.nn.functional.scaled_dot_product_attention(qq, kd, vd)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        torch.nn.functional.scaled_dot_product_attention(qq, kd, vd)
    e1.record()
    torch.cuda.synchronize()
    us_d = e0.elapsed_time(e1) / iters * 1e3
    dense_by = 2 * n * Hq * D * 2
    print(f"S={S} Hkv={Hkv} Hq={Hq} {dtype}: kept {n}, packed {code_bytes/1e6:.2f} MB ({code_bytes*8/(2*n*F):.2f} bits/elem) "
          f"-> decode {us:.1f} us, {by/us/1e3:.0f} GB/s algorithmic | dense SDPA over K'/V' {us_d:.1f} us "
          f"({dense_by/1e6:.1f} MB, {dense_by/us_d/1e3:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    rtkv.build()
    cases = ((16384, 32, 32), (32768, 32, 32), (16384, 8, 32), (131072, 8, 32), (131072, 8, 8), (32768, 32, 128),
             (32768, 32, 32, "bfloat16"), (131072, 8, 32, "bfloat16"))
    only = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else range(len(cases))
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    for i in only:
        run(*cases[i], iters=iters)
