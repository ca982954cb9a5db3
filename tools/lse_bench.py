"""Time rtkv.attention_lse (row LSE of causal attention) at one shape: HIP events around N launches.
python tools/lse_bench.py [S] [H] [dtype] [head_dim] — the kernel follows RTKV_LSE_KERNEL (16: the 16x16x32
tiling; default: 32x32x16 for head_dim 128)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "realtime-kv-cache-compression_amd"))
import rtkv  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
H = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dt = getattr(torch, sys.argv[3] if len(sys.argv) > 3 else "float16")
D = int(sys.argv[4]) if len(sys.argv) > 4 else 128
n = 10
g = torch.Generator(device="cuda").manual_seed(0)
Q = torch.randn(1, H, S, D, device="cuda", generator=g).to(dt)
K = torch.randn(1, H, S, D, device="cuda", generator=g).to(dt)
for _ in range(2):
    lse = rtkv.attention_lse(Q, K)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    rtkv.attention_lse(Q, K)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / n
flops = 2.0 * H * D * S * (S + 1) / 2
print(f"lse S={S} H={H} D={D} {dt} kernel={os.environ.get('RTKV_LSE_KERNEL', 'default')}: {ms:.3f} ms, "
      f"{flops / ms / 1e9:.1f} TFLOP/s of QK^T", flush=True)
