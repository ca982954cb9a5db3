"""numpy front-end of the C oracle (oracle/rtkv_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg import this module,
and only as the checker / CPU baseline.  The rtkv product package never imports it.

Arrays are numpy; half types travel as uint16 bit patterns with an explicit dtype code
(0 = fp32, 1 = fp16, 2 = bf16), matching include/rtkv.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RTKV_ORACLE_LIB: an alternate build of the same source (run_sanitized.sh: the ASan/UBSan one)
_LIB_PATH = os.environ.get("RTKV_ORACLE_LIB", os.path.join(_HERE, "_build", "librtkv_oracle.so"))
_lib = None

F32, F16, BF16 = 0, 1, 2


def build() -> str:
    """Compile the oracle with its Makefile (gcc) and return the library path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        p, i64, i32, f, d = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_double
        L.rtkvo_attention_aggregation.argtypes = [p, i32, i64, i64, i64, i64, i64, i64, i64, p]
        L.rtkvo_attention_aggregation.restype = i32
        L.rtkvo_position_bias.argtypes = [i64, p]
        L.rtkvo_minmax_normalize.argtypes = [p, i32, i64, i64, p]
        L.rtkvo_importance_scores.argtypes = [p, i32, i64, i64, i64, f, f, f, f, p]
        L.rtkvo_assign_precision.argtypes = [p, i64, f, f, p, p]
        L.rtkvo_quant_params.argtypes = [p, i32, i64, i64, i32, p, p]
        L.rtkvo_fake_quant.argtypes = [p, i32, i64, i64, i32, f, f, p, p, i64]
        L.rtkvo_pack_codes.argtypes = [p, i64, i32, p]
        L.rtkvo_unpack_codes.argtypes = [p, i64, i32, p]
        L.rtkvo_mixed_precision.argtypes = [p, i32, i64, i64, i64, p, p, p]
        L.rtkvo_select.argtypes = [p, p, i64, i64, p, d, p, p, p, p]
        L.rtkvo_field_width.argtypes = [i32, i32]
        L.rtkvo_field_width.restype = i32
        L.rtkvo_torch_logf.argtypes = [ctypes.c_uint32]
        L.rtkvo_torch_logf.restype = f
        L.rtkvo_round.argtypes = [i32, f]
        L.rtkvo_round.restype = f
        L.rtkvo_compress_layer.argtypes = (
            [p, p, i32, i64, i64, i64, p, i32, i64, i64, i64, f, f, f, f, f, f, p, d, i32]
            + [p] * 13 + [p, i32])
        L.rtkvo_compress_layer.restype = i64
        L.rtkvo_gq_votes.argtypes = [p, i32, i64, i32, i32, p, i64, i32, i32, p]
        L.rtkvo_gq_select.argtypes = [p, i32, i32, i32, ctypes.c_uint32, p]
        L.rtkvo_gq_pack.argtypes = [p, i32, i64, i32, i32, p, i64, p, p, i32, p, p, p, p, p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _c(a, dtype=None):
    a = np.ascontiguousarray(a if dtype is None else a.astype(dtype, copy=False))
    return a


def f32(x):
    return np.float32(x)


# ----------------------------------------------------------------------------- stage functions
def attention_aggregation(W: np.ndarray, dt: int, P: int) -> np.ndarray:
    """W [B,H,S,cols] (float32, or uint16 bits for half types) -> A [B,S] float32."""
    W = _c(W)
    B, H, S, cols = W.shape
    A = np.zeros((B, S), np.float32)
    rc = lib().rtkvo_attention_aggregation(_ptr(W), dt, B, H, S, P, H * S * cols, S * cols, cols, _ptr(A))
    assert rc == 0
    return A


def position_bias(S: int) -> np.ndarray:
    pos = np.zeros(S, np.float32)
    lib().rtkvo_position_bias(S, _ptr(pos))
    return pos


def minmax_normalize(A: np.ndarray, dt: int) -> np.ndarray:
    A = _c(A, np.float32)
    N = np.zeros_like(A)
    lib().rtkvo_minmax_normalize(_ptr(A), dt, A.shape[0], A.shape[1], _ptr(N))
    return N


def importance_scores(A: np.ndarray, dt: int, P: int, alpha, beta, gamma, w_l) -> np.ndarray:
    A = _c(A, np.float32)
    s = np.zeros_like(A)
    lib().rtkvo_importance_scores(_ptr(A), dt, A.shape[0], A.shape[1], P, f32(alpha), f32(beta),
                                  f32(gamma), f32(w_l), _ptr(s))
    return s


def assign_precision(scores: np.ndarray, theta_h, theta_m):
    scores = _c(scores, np.float32)
    labels = np.zeros(scores.shape, np.uint8)
    counts = np.zeros(3, np.int64)
    lib().rtkvo_assign_precision(_ptr(scores), scores.size, f32(theta_h), f32(theta_m), _ptr(labels), _ptr(counts))
    return labels, counts


def quant_params(x: np.ndarray, dt: int, bits: int):
    x = _c(x)
    sc = np.zeros(1, np.float32)
    zp = np.zeros(1, np.float32)
    lib().rtkvo_quant_params(_ptr(x), dt, 0, x.size, bits, _ptr(sc), _ptr(zp))
    return float(sc[0]), float(zp[0])


def fake_quant(x: np.ndarray, dt: int, bits: int, scale: float, zp: float):
    x = _c(x)
    codes = np.zeros(x.size, np.uint32)
    out = np.zeros_like(x)
    lib().rtkvo_fake_quant(_ptr(x), dt, 0, x.size, bits, f32(scale), f32(zp), _ptr(codes), _ptr(out), 0)
    return codes.reshape(x.shape), out


def mixed_precision(x: np.ndarray, dt: int, labels: np.ndarray, bits) -> np.ndarray:
    x = _c(x)
    B, S, F = x.shape
    out = np.zeros_like(x)
    b3 = np.asarray(bits, np.int32)
    lib().rtkvo_mixed_precision(_ptr(x), dt, B, S, F, _ptr(_c(labels, np.uint8)), _ptr(b3), _ptr(out))
    return out


def pack_codes(codes: np.ndarray, w: int) -> np.ndarray:
    codes = _c(codes, np.uint32)
    dst = np.zeros((codes.size * w + 7) // 8, np.uint8)
    lib().rtkvo_pack_codes(_ptr(codes), codes.size, w, _ptr(dst))
    return dst


def unpack_codes(src: np.ndarray, n: int, w: int) -> np.ndarray:
    codes = np.zeros(n, np.uint32)
    lib().rtkvo_unpack_codes(_ptr(_c(src, np.uint8)), n, w, _ptr(codes))
    return codes


def field_width(dt: int, bits: int) -> int:
    return lib().rtkvo_field_width(dt, bits)


def select(scores: np.ndarray, labels: np.ndarray, bits, ratio: float):
    scores = _c(scores, np.float32)
    B, S = scores.shape
    mask = np.zeros((B, S), np.uint8)
    kept = np.zeros(B, np.int64)
    units = np.zeros(B, np.int64)
    fb = np.zeros(B, np.int32)
    lib().rtkvo_select(_ptr(scores), _ptr(_c(labels, np.uint8)), B, S, _ptr(np.asarray(bits, np.int32)),
                       float(ratio), _ptr(mask), _ptr(kept), _ptr(units), _ptr(fb))
    return mask, kept, units, fb


def torch_logf(n: int) -> float:
    return lib().rtkvo_torch_logf(n)


def compress_layer(K, V, kvdt, W, wdt, P, alpha, beta, gamma, w_l, theta_h, theta_m, bits, ratio,
                   no_selection=False, packed=True, threads=1):
    """Full-layer oracle.  K,V [B,S,F]; W [B,H,S,cols].  Returns a dict of numpy outputs with the
    padded dequant K'/V' trimmed to [B, S'_max, F]."""
    K, V, W = _c(K), _c(V), _c(W)
    B, S, F = K.shape
    _, H, _, cols = W.shape
    b3 = np.asarray(bits, np.int32)
    scores = np.zeros((B, S), np.float32)
    labels = np.zeros((B, S), np.uint8)
    mask = np.zeros((B, S), np.uint8)
    kept_index = np.zeros((B, S), np.int32)
    k_out = np.zeros_like(K)
    v_out = np.zeros_like(V)
    scale_zp = np.zeros((B, S, 4), np.float32)
    wmax = max(field_width(kvdt, int(b)) for b in bits)
    cap = B * S * ((F * wmax + 7) // 8) if packed else 0
    pk = np.zeros(max(cap, 1), np.uint8) if packed else None
    pv = np.zeros(max(cap, 1), np.uint8) if packed else None
    row_offset = np.zeros((B, S), np.int64)
    kept = np.zeros(B, np.int64)
    units = np.zeros(B, np.int64)
    fb = np.zeros(B, np.int32)
    cc = np.zeros(3, np.int64)
    smax = lib().rtkvo_compress_layer(
        _ptr(K), _ptr(V), kvdt, B, S, F, _ptr(W), wdt, H, cols, P, f32(alpha), f32(beta), f32(gamma),
        f32(w_l), f32(theta_h), f32(theta_m), _ptr(b3), float(ratio), int(bool(no_selection)),
        _ptr(scores), _ptr(labels), _ptr(mask), _ptr(kept_index), _ptr(k_out), _ptr(v_out),
        _ptr(scale_zp), _ptr(pk), _ptr(pv), _ptr(row_offset), _ptr(kept), _ptr(units), _ptr(fb),
        _ptr(cc), int(threads))
    assert smax >= 0, smax
    total = int(row_offset[-1, -1]) if B * S else 0
    if packed and B * S:
        # bytes used = offset after the last kept row of the last batch row
        last = B - 1
        nk = int(kept[last])
        if nk:
            lab = labels[last, kept_index[last, nk - 1]]
            total = int(row_offset[last, nk - 1]) + (F * field_width(kvdt, int(bits[lab])) + 7) // 8
        else:
            total = int(row_offset[last, 0])
    return dict(scores=scores, labels=labels, mask=mask, kept_index=kept_index[:, :smax],
                k_out=k_out[:, :smax], v_out=v_out[:, :smax], scale_zp=scale_zp[:, :smax],
                packed_k=pk[:total] if packed else None, packed_v=pv[:total] if packed else None,
                row_offset=row_offset[:, :smax], kept=kept, cost_units=units, fallback=fb,
                class_count=cc, max_kept=int(smax))


# ----------------------------------------------------------------------------- extension: rtkv-gq/1
# Per-channel outlier detection + per-head group-wise pack (no reference counterpart: parity UNPINNED;
# oracle/rtkv_oracle.c defines the mode).  x: [S, F] rows (float32, or uint16 bits for half types).
def gq_votes(x: np.ndarray, dt: int, H: int, D: int, tok: np.ndarray, n_vote: int, vote_stride: int) -> np.ndarray:
    x = _c(x)
    votes = np.zeros(H * D, np.uint32)
    tok = _c(tok, np.int32)
    lib().rtkvo_gq_votes(_ptr(x), dt, x.shape[-1], H, D, _ptr(tok), tok.size, n_vote, vote_stride, _ptr(votes))
    return votes


def gq_select(votes: np.ndarray, H: int, D: int, k: int, min_votes: int) -> np.ndarray:
    idx = np.zeros((H, k), np.int16)
    lib().rtkvo_gq_select(_ptr(_c(votes, np.uint32)), H, D, k, int(min_votes), _ptr(idx))
    return idx


def gq_pack(x: np.ndarray, dt: int, H: int, D: int, tok: np.ndarray, row_bits: np.ndarray, idx: np.ndarray,
            row_offset: np.ndarray):
    """-> (codes [bytes], meta [rows, H, 2], raw [rows, H, k], deq [rows, F]) in the storage types."""
    x = _c(x)
    tok = _c(tok, np.int32)
    rows = tok.size
    F = H * D
    k = idx.shape[1]
    store = np.float32 if dt == F32 else np.uint16
    row_bits = _c(row_bits, np.int32)
    row_offset = _c(row_offset, np.int64)
    nbytes = int(row_offset[-1]) + (F * int(row_bits[-1]) + 7) // 8 if rows else 0
    codes = np.zeros(max(nbytes, 1), np.uint8)
    meta = np.zeros((rows, H, 2), store)
    raw = np.zeros((rows, H, k), store)
    deq = np.zeros((rows, F), store)
    lib().rtkvo_gq_pack(_ptr(x), dt, x.shape[-1], H, D, _ptr(tok), rows, _ptr(row_bits), _ptr(_c(idx, np.int16)), k,
                        _ptr(row_offset), _ptr(codes), _ptr(meta), _ptr(raw), _ptr(deq))
    return codes[:nbytes], meta, raw, deq
