"""GPU: one decode step of attention over a packed layer (rtkv_decode_attention_packed, decode.hip)
against a plain PyTorch fp32 reference over the dequantized K'/V' the same compression returned.

The reference model attends over the dequantized rows (modified_llama.py:140-142, scores scaled by
1/sqrt(head_dim), :89); the decode kernel reads the bit-packed codes instead and dequantizes them in
registers.  The dequantized values are identical (unpack_layer == k_out is asserted), so the only
differences are fp32 summation order and the hardware exp: tolerance rtol = 2e-4, atol = 2e-5 ·
max|V'| (the output is a convex combination of V' rows).  Cases cover every head-group shape the
kernel is instantiated for (Hkv·D / 512 = 1, 2, 8 → 4 × 2, 10 → 5 × 2), head_dim 64 / 128 / 256,
GQA (Hq / Hkv = 1, 4, 8), all three dtypes, batch 2 with different kept counts per row, and layers
with a single kept row."""
import numpy as np
import pytest
import torch

import synth

pytestmark = pytest.mark.gpu

TD = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import rtkv
    rtkv.build()


def dev(stored: np.ndarray, dtype: str) -> torch.Tensor:
    if dtype == "float32":
        return torch.from_numpy(np.ascontiguousarray(stored, np.float32)).cuda()
    return torch.from_numpy(np.ascontiguousarray(stored, np.uint16).view(np.int16)).cuda().view(TD[dtype])


def reference(k2, v2, rows, q, Hkv, scale):
    """softmax(q·K'ᵀ·scale)·V' in fp32 per batch row over its kept rows."""
    B, Hq, D = q.shape
    G = Hq // Hkv
    out = torch.zeros(B, Hq, D, dtype=torch.float32, device=q.device)
    for b in range(B):
        n = int(rows[b])
        if n == 0:
            continue
        Kf = k2[b, :n].float().view(n, Hkv, D)
        Vf = v2[b, :n].float().view(n, Hkv, D)
        qf = q[b].float().view(Hkv, G, D)
        s = torch.einsum("hgd,nhd->hgn", qf, Kf) * scale
        p = torch.softmax(s, dim=-1)
        out[b] = torch.einsum("hgn,nhd->hgd", p, Vf).reshape(Hq, D)
    return out


COV = dict(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25)
CASES = [
    # B, S, Hkv, D, Hq, dtype, bits, ratio
    (1, 4096, 8, 128, 32, "float16", (2, 4, 8), 0.6),     # F = 1024: 2 chunks / lane, GQA 4
    (2, 3000, 32, 128, 32, "bfloat16", (2, 4, 8), 0.5),   # F = 4096: 2 head groups × 4 chunks
    (1, 1000, 8, 64, 8, "float32", (4, 8, 16), 0.7),      # F = 512, head_dim 64
    (1, 700, 40, 128, 40, "float16", (2, 4, 8), 0.9),     # F = 5120: 2 head groups × 5 chunks
    (1, 2000, 2, 256, 16, "float16", (4, 4, 8), 0.6),     # head_dim 256, GQA 8
    (2, 5, 4, 128, 16, "bfloat16", (2, 4, 8), 0.3),       # a handful of kept rows
    (1, 8192, 8, 128, 64, "float32", (2, 4, 8), 0.4),     # fp32 codes, GQA 8, many splits
]


@pytest.mark.parametrize("B,S,Hkv,D,Hq,dtype,bits,ratio", CASES,
                         ids=lambda v: str(v) if not isinstance(v, tuple) else "-".join(map(str, v)))
def test_decode_attention_packed(B, S, Hkv, D, Hq, dtype, bits, ratio):
    import rtkv
    F = Hkv * D
    seed = S * 7 + Hkv
    K, V = synth.kv(seed, B, S, F, dtype)
    P = rtkv.prompt_length(S)
    W = synth.attention_slice(seed, B, 8, S, P, dtype)
    cfg = rtkv.CompressionConfig(num_hidden_layers=4, low_precision_bits=bits[0], medium_precision_bits=bits[1],
                                 high_precision_bits=bits[2], early_layer_ratio=ratio, middle_layer_ratio=ratio,
                                 later_layer_ratio=ratio, **COV)
    comp = rtkv.RealTimePrefillCompressor(cfg)
    ids = torch.zeros(B, S, dtype=torch.long, device="cuda")
    k2, v2, info = comp.compress_layer_kv_cache(dev(K, dtype), dev(V, dtype), dev(W, dtype), ids, 1)
    pk = info["packed"]
    dk, dv = rtkv.unpack_layer(pk)
    assert torch.equal(dk, k2) and torch.equal(dv, v2)
    q = dev(synth.cast(synth.normal(seed + 1, (B, Hq, D)), dtype), dtype)
    out = rtkv.decode_attention(pk, q, Hkv)
    ref = reference(k2, v2, pk["rows"], q, Hkv, 1.0 / D ** 0.5)
    vmax = v2.float().abs().max().item()
    torch.testing.assert_close(out, ref, rtol=2e-4, atol=2e-5 * max(vmax, 1.0))
    # the cache container routes to the same kernel
    cache = rtkv.CompressedKVCache(B, S, D)
    cache.store_packed(0, pk)
    assert torch.equal(cache.attend(0, q, Hkv), out)
    # deterministic: same inputs, same bits
    assert torch.equal(rtkv.decode_attention(pk, q, Hkv), out)


def test_decode_rejects_bad_shapes():
    import rtkv
    S, Hkv, D = 600, 4, 96  # F = 384: not a multiple of 512
    K, V = synth.kv(3, 1, S, Hkv * D, "float16")
    W = synth.attention_slice(3, 1, 4, S, rtkv.prompt_length(S), "float16")
    comp = rtkv.RealTimePrefillCompressor(rtkv.CompressionConfig(num_hidden_layers=4, low_precision_bits=2,
                                                                 medium_precision_bits=4, high_precision_bits=8, **COV))
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    _, _, info = comp.compress_layer_kv_cache(dev(K, "float16"), dev(V, "float16"), dev(W, "float16"), ids, 1)
    q = torch.zeros(1, 4, D, dtype=torch.float16, device="cuda")
    with pytest.raises(RuntimeError, match="decode"):
        rtkv.decode_attention(info["packed"], q, Hkv)
    with pytest.raises(ValueError):
        rtkv.decode_attention(info["packed"], q.float(), Hkv)


def test_packed_file_round_trip_decodes_identically(tmp_path):
    """compress → save_packed → load_packed → the same K'/V' and the same decode output."""
    import rtkv
    B, S, Hkv, D, Hq, dtype = 2, 1500, 8, 128, 32, "float16"
    K, V = synth.kv(9, B, S, Hkv * D, dtype)
    W = synth.attention_slice(9, B, 8, S, rtkv.prompt_length(S), dtype)
    comp = rtkv.RealTimePrefillCompressor(rtkv.CompressionConfig(num_hidden_layers=4, low_precision_bits=2,
                                                                 medium_precision_bits=4, high_precision_bits=8, **COV))
    ids = torch.zeros(B, S, dtype=torch.long, device="cuda")
    k2, v2, info = comp.compress_layer_kv_cache(dev(K, dtype), dev(V, dtype), dev(W, dtype), ids, 2)
    path = str(tmp_path / "layer.safetensors")
    rtkv.save_packed({2: info["packed"]}, path)
    back = rtkv.load_packed(path, device="cuda")[2]
    dk, dv = rtkv.unpack_layer(back)
    assert torch.equal(dk, k2) and torch.equal(dv, v2)
    q = dev(synth.cast(synth.normal(10, (B, Hq, D)), dtype), dtype)
    assert torch.equal(rtkv.decode_attention(back, q, Hkv), rtkv.decode_attention(info["packed"], q, Hkv))


def test_decode_inconsistent_metadata_stays_in_bounds():
    """Offsets past the code buffer read as zero codes and kept indices are clamped: the kernel
    never reads outside its buffers (the result is finite, the GPU does not fault)."""
    import rtkv
    S, Hkv, D = 800, 4, 128
    K, V = synth.kv(4, 1, S, Hkv * D, "float16")
    W = synth.attention_slice(4, 1, 4, S, rtkv.prompt_length(S), "float16")
    comp = rtkv.RealTimePrefillCompressor(rtkv.CompressionConfig(num_hidden_layers=4, low_precision_bits=2,
                                                                 medium_precision_bits=4, high_precision_bits=8, **COV))
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    _, _, info = comp.compress_layer_kv_cache(dev(K, "float16"), dev(V, "float16"), dev(W, "float16"), ids, 1)
    pk = dict(info["packed"])
    pk["row_offset"] = pk["row_offset"].clone()
    pk["row_offset"][0, :5] = 1 << 40
    pk["kept_index"] = pk["kept_index"].clone()
    pk["kept_index"][0, 5:9] = 1 << 30
    pk.pop("_rows_dev", None)
    q = torch.randn(1, 8, D, device="cuda").half()
    out = rtkv.decode_attention(pk, q, Hkv)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    bad = dict(pk, rows=[pk["kept_index"].shape[1] + 1])
    bad.pop("_rows_dev", None)
    with pytest.raises(ValueError):
        rtkv.decode_attention(bad, q, Hkv)
