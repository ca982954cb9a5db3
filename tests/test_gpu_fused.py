"""GPU: the fused selection + quantization launch (csrc/fused.h, opt-in with RTKV_FUSED_QUANT; taken
for one batch row of S <= 32768 tokens with contiguous 4096- or 5120-element rows), against the same
layer run as two launches (the default: select_fast.hip's K2, then quant_rows_kernel) and, at sizes the
oracle finishes quickly, against the C oracle.

Every output must agree byte for byte: scores, classes, mask, kept indices, row offsets, packed codes,
scale/zero-point, the dequantized rows, and the statistics.  The fused launch's quantization waves
decide keep/drop from the early mode word and the thresholds themselves (ties from phase 3's per-token
rows), so the cases cover every mode: all classes kept, partial classes with and without threshold
ties, the emergency fallback, quantization only, constant scores, and the row-count edges of the
1024-token selection workgroups."""
import numpy as np
import pytest
import torch

import rtkv_oracle as orc
import synth

pytestmark = pytest.mark.gpu

TD = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def dev(stored: np.ndarray, dtype: str) -> torch.Tensor:
    if dtype == "float32":
        return torch.from_numpy(np.ascontiguousarray(stored, np.float32)).cuda()
    return torch.from_numpy(np.ascontiguousarray(stored, np.uint16).view(np.int16)).cuda().view(TD[dtype])


def gen(seed, S, F, H, P, dtype, kind):
    """K, V, W on the device, generated there for large S (torch RNG) or by synth (the oracle's inputs)."""
    if S * F <= 4096 * 4096 and kind != "big":
        K, V = synth.kv(seed, 1, S, F, dtype)
        if kind == "tie":
            u = synth.uniform(seed, (S,))
            lvl = (np.floor(u * 3) / 2).astype(np.float32)
            W = np.zeros((1, H, S, P), np.float32)
            W[0, :, :, 0] = lvl[None, :] * 0.5
            W = synth.cast(W, dtype)
        elif kind == "const":
            W = synth.cast(np.full((1, H, S, P), 0.25, np.float32), dtype)
        else:
            W = synth.attention_slice(seed, 1, H, S, P, dtype)
        return (dev(K, dtype), dev(V, dtype), dev(W, dtype)), (K, V, W)
    g = torch.Generator(device="cuda").manual_seed(seed)
    td = TD[dtype]
    K = torch.randn(1, S, F, device="cuda", generator=g).to(td)
    V = torch.randn(1, S, F, device="cuda", generator=g).to(td)
    u = torch.rand(1, H, S, P, device="cuda", generator=g)
    W = (u * u) ** 2 + 1e-6
    W = (W / W.sum(-1, keepdim=True) * torch.rand(1, H, S, 1, device="cuda", generator=g)).to(td)
    return (K, V, W), None


def run(K, V, W, S, F, dtype, kw, layer, ratio, flags, L=4):
    import rtkv
    cfg = rtkv.CompressionConfig(num_hidden_layers=L, **kw)
    P = rtkv.prompt_length(S)
    bits = (cfg.low_precision_bits, cfg.medium_precision_bits, cfg.high_precision_bits)
    p = rtkv.params_from_config(cfg, layer, P, ratio, flags)
    from rtkv import _lib as Lb
    dq, pk = bool(flags & Lb.EMIT_DEQUANT), bool(flags & Lb.EMIT_PACKED)
    bufs = rtkv.LayerBuffers(1, S, F, TD[dtype], "cuda", bits, emit_dequant=dq, emit_packed=pk)
    bufs.arena.fill_(0xA5)  # every byte the outputs expose must be written by the launch
    res = rtkv.compress_layer(K, V, W, p, bufs, rtkv.Workspace("cuda"))
    st = res.final_stats()
    n = st.max_kept
    out = dict(scores=bufs.scores.cpu(), labels=bufs.labels.cpu(), mask=bufs.mask.cpu(),
               kept=bufs.kept_index[0, :n].cpu())
    if pk:
        pb = st.total_packed_bytes
        out.update(row_offset=bufs.row_offset[0, :n].cpu(), scale_zp=bufs.scale_zp[0, :n].cpu(),
                   pk=bufs.packed_k[:pb].cpu(), pv=bufs.packed_v[:pb].cpu())
    if dq:
        out.update(k_out=bufs.k_out[: n * F].cpu(), v_out=bufs.v_out[: n * F].cpu())
    return out, st


def same(a, b):
    for name in a:
        x, y = a[name], b[name]
        assert torch.equal(x.view(torch.uint8) if x.dtype != torch.uint8 else x,
                           y.view(torch.uint8) if y.dtype != torch.uint8 else y), name


COV = dict(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, low_precision_bits=2, medium_precision_bits=4,
           high_precision_bits=8)
CASES = [
    # S, F, dtype, ratio, cfg overrides, attention kind
    (1, 4096, "float16", 0.8, {}, "rand"),
    (2, 4096, "float32", 0.6, {}, "rand"),
    (17, 4096, "bfloat16", 0.4, {}, "rand"),
    (1023, 4096, "float32", 0.6, {}, "rand"),
    (1025, 4096, "float16", 0.4, {}, "rand"),
    (4096, 4096, "float32", 0.6, {}, "rand"),
    (4096, 4096, "float16", 1.0, {}, "rand"),          # everything fits: every class ALL
    (4097, 5120, "bfloat16", 0.8, {}, "rand"),
    (3000, 5120, "float16", 0.5, {}, "rand"),
    (3000, 5120, "bfloat16", 0.5, dict(low_precision_bits=4, medium_precision_bits=8, high_precision_bits=16),
     "rand"),                                           # bf16 16-bit codes are 17 bits wide: two launches
    (4000, 4096, "float32", 0.5, dict(low_precision_bits=4, medium_precision_bits=8, high_precision_bits=16), "rand"),
    (3000, 4096, "float16", 0.0004, {}, "rand"),       # budget below one row: the top-10% fallback
    (4096, 4096, "float16", 0.5, dict(beta=0.0), "tie"),  # threshold inside a block of equal scores
    (3000, 4096, "bfloat16", 0.3, dict(beta=0.0, gamma=0.0), "tie"),
    (2000, 4096, "float32", 0.5, dict(beta=0.0), "const"),  # every score equal: index order
    (16384, 4096, "float32", 0.6, {}, "big"),
    (16384, 4096, "float16", 0.4, {}, "big"),
    (16385, 5120, "float16", 0.8, {}, "big"),
    (32768, 4096, "bfloat16", 0.6, {}, "big"),
    (32768, 5120, "float16", 0.4, {}, "big"),
]


@pytest.mark.parametrize("S,F,dtype,ratio,over,kind", CASES, ids=lambda v: str(v))
def test_fused_matches_two_launches_and_oracle(S, F, dtype, ratio, over, kind):
    from rtkv import _lib as L
    H = F // 128
    import rtkv
    P = rtkv.prompt_length(S)
    (Kd, Vd, Wd), host = gen(900 + S, S, F, H, P, dtype, kind)
    kw = dict(COV, **over)
    base = L.EMIT_DEQUANT | L.EMIT_PACKED
    a, sa = run(Kd, Vd, Wd, S, F, dtype, kw, 1, ratio, base | L.FUSED_QUANT)
    b, sb = run(Kd, Vd, Wd, S, F, dtype, kw, 1, ratio, base)
    same(a, b)
    assert (sa.max_kept, sa.total_packed_bytes, sa.error_flags) == (sb.max_kept, sb.total_packed_bytes, sb.error_flags)
    assert sa.error_flags == 0 and sa.max_kept >= 1
    for k in ("class_count", "kept", "kept_class", "cost_units", "packed_bytes", "fallback"):
        assert sa.batch[0][k] == sb.batch[0][k], k
    if host is not None and S * F <= 3000 * 5120:
        K, V, W = host
        cfg = rtkv.CompressionConfig(num_hidden_layers=4, **kw)
        dt = synth.DTYPES[dtype]
        bits = (cfg.low_precision_bits, cfg.medium_precision_bits, cfg.high_precision_bits)
        o = orc.compress_layer(K, V, dt, W, dt, P, kw["alpha"], kw["beta"], kw["gamma"], cfg.layer_weights[1],
                               kw["theta_h"], kw["theta_m"], bits, ratio)
        assert o["max_kept"] == sa.max_kept
        assert np.array_equal(a["kept"].numpy(), o["kept_index"][0])
        assert np.array_equal(a["pk"].numpy(), o["packed_k"])
        assert np.array_equal(a["pv"].numpy(), o["packed_v"])
        assert np.array_equal(a["scale_zp"].numpy(), o["scale_zp"][0])
        stored = lambda t: t.numpy() if dtype == "float32" else t.view(torch.int16).numpy().view(np.uint16)  # noqa: E731
        assert np.array_equal(stored(a["k_out"]).reshape(-1), o["k_out"].reshape(-1))
        assert np.array_equal(stored(a["v_out"]).reshape(-1), o["v_out"].reshape(-1))


@pytest.mark.parametrize("outputs", ["packed", "dequant"])
@pytest.mark.parametrize("dtype", ["float32", "float16"])
def test_fused_single_output_modes(outputs, dtype):
    """Packed-only (the decode consumers' mode) and dequant-only outputs, and quantization only."""
    from rtkv import _lib as L
    S, F = 8192, 4096
    (Kd, Vd, Wd), _ = gen(55, S, F, 32, 128, dtype, "big")
    fl = L.EMIT_PACKED if outputs == "packed" else L.EMIT_DEQUANT
    for extra in (0, L.NO_SELECTION):
        a, sa = run(Kd, Vd, Wd, S, F, dtype, COV, 2, 0.5, fl | extra | L.FUSED_QUANT)
        b, sb = run(Kd, Vd, Wd, S, F, dtype, COV, 2, 0.5, fl | extra)
        same(a, b)
        assert sa.max_kept == sb.max_kept and (sa.max_kept == S) == bool(extra)


def test_fused_qk_mode_matches_two_launches():
    """The fused importance mode (A from Q + LSE in fp32, K/V in fp16): the fused launch scores in the
    dtype of A, quantizes in the dtype of K/V."""
    import rtkv
    from rtkv import _lib as L
    S, H, D = 4096, 32, 128
    g = torch.Generator(device="cuda").manual_seed(3)
    K = torch.randn(1, S, H * D, device="cuda", generator=g).half()
    V = torch.randn(1, S, H * D, device="cuda", generator=g).half()
    Q = torch.randn(1, H, S, D, device="cuda", generator=g).half()
    lse = rtkv.attention_lse(Q, K, k_layout="bsf")
    cfg = rtkv.CompressionConfig(num_hidden_layers=1, layer_weights=[1.0], **COV)
    outs = []
    for extra in (L.FUSED_QUANT, 0):
        p = rtkv.params_from_config(cfg, 0, rtkv.prompt_length(S), 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED | extra)
        bufs = rtkv.LayerBuffers(1, S, H * D, torch.float16, "cuda", (2, 4, 8))
        st = rtkv.compress_layer_qk(K, V, Q, lse, p, bufs, rtkv.Workspace("cuda")).final_stats()
        n, pb = st.max_kept, st.total_packed_bytes
        outs.append((bufs.kept_index[0, :n].cpu(), bufs.packed_k[:pb].cpu(), bufs.k_out[: n * H * D].cpu(),
                     bufs.scale_zp[0, :n].cpu()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
