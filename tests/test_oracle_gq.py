"""CPU: the definition of the rtkv-gq/1 extension (oracle/rtkv_oracle.c rtkvo_gq_*; per-channel outlier
detection + per-head group-wise pack).  The mode has no reference counterpart, so its parity is UNPINNED;
what is pinned here is (a) that with one head spanning the whole row and no outlier channels it IS the
reference's per-token quantization (rtkvo_quant_params / rtkvo_fake_quant, themselves pinned to the
reference-generated goldens by test_oracle_golden.py) bit for bit, and (b) its defining properties: votes
find injected outlier channels, the vote threshold and tie order, exact outliers, error bounds."""
import numpy as np
import pytest

import rtkv_oracle as orc
import synth


def _rows(seed, S, F, dtype):
    x = synth.cast(synth.normal(seed, (S, F)).astype(np.float32), dtype)
    return x


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
@pytest.mark.parametrize("bits", [2, 4, 8])
def test_one_group_without_outliers_is_the_reference_per_token_quantization(dtype, bits):
    dt = synth.DTYPES[dtype]
    S, D = 37, 128
    x = _rows(11 + bits, S, D, dtype)
    tok = np.arange(S, dtype=np.int32)[::2].copy()
    idx = np.full((1, 1), -1, np.int16)
    row_bits = np.full(tok.size, bits, np.int32)
    ro = np.arange(tok.size, dtype=np.int64) * (D * bits // 8)
    codes, meta, raw, deq = orc.gq_pack(x, dt, 1, D, tok, row_bits, idx, ro)
    for r, t in enumerate(tok):
        sc, zp = orc.quant_params(x[t], dt, bits)
        q, out = orc.fake_quant(x[t], dt, bits, sc, zp)
        m = synth.to_f32(meta[r, 0], dtype)
        assert m[0] == np.float32(sc) and m[1] == np.float32(zp)
        assert np.array_equal(deq[r], out)
        assert np.array_equal(orc.unpack_codes(codes[ro[r]:ro[r] + D * bits // 8], D, bits), q)


def test_votes_find_injected_outlier_channels_and_the_threshold_holds():
    S, H, D = 256, 4, 128
    x = synth.normal(3, (S, H * D)).astype(np.float32)
    hot = [5, 128 + 77, 256 + 3, 256 + 90]
    for c in hot:
        x[:, c] *= 30.0
    x[::16, 384 + 11] *= 30.0  # head 3: large in 1 row of 16 only — below a 25 % vote threshold
    tok = np.arange(S, dtype=np.int32)
    votes = orc.gq_votes(x, 0, H, D, tok, 2, 2)
    nsamp = -(-S // 2)
    for c in hot:  # (a scaled channel loses a row's vote only where its own normal draw is near zero)
        assert votes[c] >= 0.85 * nsamp
    idx = orc.gq_select(votes, H, D, 3, -(-nsamp * 250 // 1000))
    assert idx[0, 0] == 5 and idx[1, 0] == 77 and sorted(idx[2, :2]) == [3, 90]
    assert idx[3, 0] == -1 and np.all(idx[0, 1:] == -1)  # no random channel passes the threshold
    # without a threshold the slots fill by votes, ties toward the lower channel
    v = np.zeros(H * D, np.uint32)
    v[[10, 20, 30]] = 7
    v[40] = 9
    assert list(orc.gq_select(v, H, D, 3, 1)[0]) == [40, 10, 20]


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_outliers_are_exact_and_the_rest_is_within_half_a_step(dtype):
    dt = synth.DTYPES[dtype]
    S, H, D, bits = 64, 8, 128, 4
    x32 = synth.normal(21, (S, H * D)).astype(np.float32)
    x32[:, [7, 300, 700]] *= 40.0
    x = synth.cast(x32, dtype)
    tok = np.arange(S, dtype=np.int32)
    votes = orc.gq_votes(x, dt, H, D, tok, 2, 1)
    idx = orc.gq_select(votes, H, D, 2, 16)
    assert idx[0, 0] == 7 and idx[2, 0] == 300 - 256 and idx[5, 0] == 700 - 640
    ro = np.arange(S, dtype=np.int64) * (H * D * bits // 8)
    codes, meta, raw, deq = orc.gq_pack(x, dt, H, D, tok, np.full(S, bits, np.int32), idx, ro)
    xs = synth.to_f32(x, dtype)
    d = synth.to_f32(deq, dtype)
    for c in (7, 300, 700):
        assert np.array_equal(deq[:, c], x[:, c])  # bit for bit
        h = c // D
        s = list(idx[h]).index(c - h * D)
        assert np.array_equal(raw[:, h, s], x[:, c])
    m = synth.to_f32(meta, dtype)
    step = np.repeat(m[:, :, 0], D, axis=1)
    keep = np.ones(H * D, bool)
    keep[[7, 300, 700]] = False
    err = np.abs(d - xs)[:, keep]
    # half a step, plus the dtype rounding of each op (x/s, + zp, q - zp, · s: |t|, |q - zp| <= qmax + 1)
    u = {"float32": 2.0 ** -24, "float16": 2.0 ** -11, "bfloat16": 2.0 ** -8}[dtype]
    qmax = 2 ** bits - 1
    tol = step[:, keep] * (0.5 + (2 * qmax + 2) * u) + 3 * np.abs(xs[:, keep]) * u
    assert np.all(err <= tol)
    # the outlier-free groups' step is far below the per-token scheme's on the same rows
    sc_tok = np.array([orc.quant_params(x[t], dt, bits)[0] for t in range(S)], np.float32)
    assert np.median(m[:, 0, 0]) < 0.2 * np.median(sc_tok)
