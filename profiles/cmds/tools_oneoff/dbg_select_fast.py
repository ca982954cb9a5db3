"""Diagnostic (not a test): first mismatches between the fast and pipeline selections and the oracle."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", p) for p in ("realtime-kv-cache-compression_amd", "oracle", "tests/golden", "tests")]
import numpy as np, torch
import synth, rtkv_oracle as orc
from test_gpu_select_fast import run, dev, COV
import rtkv
from rtkv import _lib as L
S, dtype, ratio = int(sys.argv[1]), sys.argv[2], float(sys.argv[3])
H, D = 2, 64
F = H * D
P = rtkv.prompt_length(S)
K, V = synth.kv(700 + S, 1, S, F, dtype)
W = synth.attention_slice(700 + S, 1, H, S, P, dtype)
Kd, Vd, Wd = dev(K, dtype), dev(V, dtype), dev(W, dtype)
base = L.EMIT_DEQUANT | L.EMIT_PACKED
a, sa = run(Kd, Vd, Wd, dtype, S, F, COV, 1, ratio, base)
b, sb = run(Kd, Vd, Wd, dtype, S, F, COV, 1, ratio, base | L.SELECT_PIPELINE)
cfg = rtkv.CompressionConfig(num_hidden_layers=4, **COV)
dt = synth.DTYPES[dtype]
o = orc.compress_layer(K, V, dt, W, dt, P, COV["alpha"], COV["beta"], COV["gamma"], cfg.layer_weights[1],
                       COV["theta_h"], COV["theta_m"], (2, 4, 8), ratio)
for nm, x in (("fast", a), ("pipe", b)):
    sc = x["scores"][0].numpy()
    bad = np.nonzero(sc.view(np.uint32) != o["scores"][0].view(np.uint32))[0]
    print(nm, "score mismatches vs oracle:", len(bad), bad[:10], sc[bad[:5]], o["scores"][0][bad[:5]])
    print(nm, "mask mismatches:", int((x["mask"][0].numpy() != o["mask"][0]).sum()), "kept", sa.max_kept if nm == "fast" else sb.max_kept, o["max_kept"])
