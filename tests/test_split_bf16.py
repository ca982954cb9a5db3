"""CPU: the numerics behind the fp32 LSE on the bf16 matrix cores (csrc/attn_f32.hip,
attn_lse_f32x3_kernel).  Each fp32 operand is split into three bf16 parts by round-to-nearest-even,
x = h + l + ll, and q·k is summed over the six part products of order ≥ 2^-18 (h·h, h·l, l·h, h·ll,
ll·h, l·l).  This restates the split with numpy and checks the two claims the kernel relies on: the
split residual is below 2^-24·|x| (in practice ~2^-27), and a 128-term dot product of the six
products is as accurate as an fp32 one against float64."""
import numpy as np


def bf16_rne(x: np.ndarray) -> np.ndarray:
    """float32 → bf16 (round to nearest even) → float32, as v_cvt_pk_bf16_f32 does for finite x."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def split3(x: np.ndarray):
    h = bf16_rne(x)
    r1 = (x - h).astype(np.float32)       # exact in fp32
    lo = bf16_rne(r1)
    r2 = (r1 - lo).astype(np.float32)     # exact in fp32
    return h, lo, bf16_rne(r2)


def test_split_residual_is_below_fp32_rounding():
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(200000) * np.exp2(rng.integers(-30, 30, 200000))).astype(np.float32)
    h, lo, ll = split3(x)
    recon = h.astype(np.float64) + lo.astype(np.float64) + ll.astype(np.float64)
    rel = np.abs(recon - x.astype(np.float64)) / np.abs(x.astype(np.float64))
    assert rel.max() <= 2.0 ** -24
    assert np.median(rel) <= 2.0 ** -26


def test_six_part_products_are_fp32_accurate():
    rng = np.random.default_rng(4)
    n, D = 4000, 128
    q = (rng.standard_normal((n, D)) * 1.5).astype(np.float32)
    k = (rng.standard_normal((n, D)) * 1.5).astype(np.float32)
    exact = np.einsum("nd,nd->n", q.astype(np.float64), k.astype(np.float64))
    qh, ql, qll = split3(q)
    kh, kl, kll = split3(k)
    six = np.zeros(n, dtype=np.float32)
    for a, b in ((ql, kl), (qh, kll), (qll, kh), (qh, kl), (ql, kh), (qh, kh)):  # the kernel's order
        prod = a.astype(np.float64) * b.astype(np.float64)   # bf16 × bf16 is exact in fp32
        for d in range(D):
            six = (six + prod[:, d].astype(np.float32)).astype(np.float32)
    fp32 = np.zeros(n, dtype=np.float32)
    for d in range(D):
        fp32 = (fp32 + q[:, d] * k[:, d]).astype(np.float32)
    scale = np.einsum("nd,nd->n", np.abs(q.astype(np.float64)), np.abs(k.astype(np.float64)))
    err_six = np.abs(six - exact) / scale
    err_fp32 = np.abs(fp32 - exact) / scale
    # the split's own error (dropped l·ll, ll·l, ll·ll and the split residual) is below fp32 rounding:
    # the six-product sum is as accurate as a plain fp32 dot product of the same terms
    assert err_six.max() <= 4 * err_fp32.max()
    assert err_six.max() <= 2.0 ** -20
