"""CompressedKVCache and AdaptiveQuantization — the compression_layers API surface named by the
north_star (reference src/models/compression_layers.py:7-45 and :96-175).

CompressedKVCache keeps the reference's dict-of-tensors interface and adds the packed form of a layer
(bit-packed integer codes + per-row scale/zero-point, as produced by rtkv_compress_layer) with an
on-device decoder (rtkv_unpack_dequant) that reproduces the dequantized K'/V' bit for bit.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch
import torch.nn as nn

from . import _lib as L
from .token_importance import _workspace


class CompressedKVCache:
    """Per-layer storage of compressed K/V (compression_layers.py:7-45)."""

    def __init__(self, max_batch_size: int, max_seq_len: int, head_dim: int):
        self.max_batch_size = max_batch_size
        self.max_seq_len = max_seq_len
        self.head_dim = head_dim
        self.cache_data: Dict[int, dict] = {}
        self.compression_info: Dict[int, dict] = {}

    def store_compressed_kv(self, layer_idx: int, keys: torch.Tensor, values: torch.Tensor,
                            importance_scores: torch.Tensor, precision_labels: torch.Tensor,
                            selection_mask: torch.Tensor):
        self.cache_data[layer_idx] = {
            "keys": keys.detach(),
            "values": values.detach(),
            "importance_scores": importance_scores.detach(),
            "precision_labels": precision_labels.detach(),
            "selection_mask": selection_mask.detach(),
            "compressed_seq_len": keys.shape[1],
        }

    def get_compressed_kv(self, layer_idx: int) -> Optional[Dict]:
        return self.cache_data.get(layer_idx)

    def clear_cache(self):
        self.cache_data.clear()
        self.compression_info.clear()

    # ------------------------------------------------------------------ packed form (extension)
    def store_packed(self, layer_idx: int, packed: dict):
        """Keep only the packed codes of a layer (``info['packed']`` of compress_layer_kv_cache)."""
        self.compression_info[layer_idx] = packed

    def packed_nbytes(self, layer_idx: int) -> int:
        p = self.compression_info[layer_idx]
        return (p["codes_k"].numel() + p["codes_v"].numel() + p["scale_zp"].numel() * 4
                + p["kept_index"].numel() * 4)

    def dequantize(self, layer_idx: int):
        """Decode a packed layer back to dense (K', V') [B, S'_max, F] on the device."""
        p = self.compression_info[layer_idx]
        return unpack_layer(p)

    def attend(self, layer_idx: int, q: torch.Tensor, num_kv_heads: int, scale: Optional[float] = None):
        """One decode step of attention over the packed layer (no dense K'/V'): fp32 [B, Hq, D]."""
        return decode_attention(self.compression_info[layer_idx], q, num_kv_heads, scale)

    def save(self, path: str):
        """Write every packed layer to one safetensors file (see save_packed for the format)."""
        save_packed(self.compression_info, path)

    def load(self, path: str, device="cuda"):
        """Read the packed layers of a file written by save(); replaces the packed layers held."""
        self.compression_info = load_packed(path, device)


# ---------------------------------------------------------------------- packed (de)serialization
# File format "rtkv-packed/1": a safetensors file.  Per layer i, tensors "L{i}.codes_k",
# "L{i}.codes_v" (uint8, the bit-packed rows back to back), "L{i}.row_offset" (int64 [B, S'] byte
# offset of each kept row), "L{i}.scale_zp" (fp32 [B, S', 4]: K scale, K zero-point, V scale,
# V zero-point), "L{i}.kept_index" (int32 [B, S'] source token index), "L{i}.labels" (uint8 [B, S]
# precision class per source token); the metadata entry "L{i}" holds {"rows", "bits", "dtype",
# "feature_dim"} as JSON.  Loading checks every offset and count against the tensor sizes, so a
# truncated or inconsistent file raises ValueError instead of reaching a kernel.
_FORMAT = "rtkv-packed/1"
_TENSORS = ("codes_k", "codes_v", "row_offset", "scale_zp", "kept_index", "labels")
_DTYPES = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


def save_packed(layers: Dict[int, dict], path: str):
    import json
    from safetensors.torch import save_file
    tensors, meta = {}, {"format": _FORMAT}
    for i, p in layers.items():
        for name in _TENSORS:
            tensors[f"L{i}.{name}"] = p[name].detach().contiguous().cpu()
        meta[f"L{i}"] = json.dumps({"rows": [int(r) for r in p["rows"]], "bits": [int(b) for b in p["bits"]],
                                    "dtype": str(p["dtype"]).replace("torch.", ""),
                                    "feature_dim": int(p["feature_dim"])})
    save_file(tensors, path, metadata=meta)


_TENSOR_DTYPES = {"codes_k": torch.uint8, "codes_v": torch.uint8, "row_offset": torch.int64,
                  "scale_zp": torch.float32, "kept_index": torch.int32, "labels": torch.uint8}


def _check_dtypes(where, p: dict):
    """The kernels read these buffers with fixed element types; a wrong dtype would be misread or
    read past its end."""
    for name, dt in _TENSOR_DTYPES.items():
        if p[name].dtype != dt:
            raise ValueError(f"packed layer {where}: {name} must be {dt}, got {p[name].dtype}")


def _check_packed(i: int, p: dict):
    def bad(msg):
        raise ValueError(f"packed layer {i}: {msg}")
    _check_dtypes(i, p)
    if p["kept_index"].dim() != 2:
        bad("kept_index must be [B, S']")
    B, Sp = p["kept_index"].shape
    if p["row_offset"].shape != (B, Sp) or p["scale_zp"].shape != (B, Sp, 4) or p["labels"].dim() != 2 \
            or p["labels"].shape[0] != B:
        bad("inconsistent shapes")
    if p["codes_k"].numel() != p["codes_v"].numel():
        bad("codes_k and codes_v differ in size")
    if len(p["rows"]) != B or any(r < 0 or r > Sp for r in p["rows"]):
        bad("row counts out of range")
    F, S = p["feature_dim"], p["labels"].shape[1]
    widths = [L.lib().rtkv_field_width(L.TORCH_DTYPE_CODE[p["dtype"]], b) for b in p["bits"]]
    if len(widths) != 3 or min(widths) <= 0:
        bad("unsupported bits")
    nbytes = p["codes_k"].numel()
    for b in range(B):
        n = p["rows"][b]
        if n == 0:
            continue
        ki = p["kept_index"][b, :n].to(torch.int64)
        if int(ki.min()) < 0 or int(ki.max()) >= S:
            bad("kept index out of range")
        lab = p["labels"][b].to(torch.int64)[ki]
        if int(lab.max()) > 2:
            bad("class label out of range")
        w = torch.tensor(widths, dtype=torch.int64)[lab]
        off = p["row_offset"][b, :n]
        if int(off.min()) < 0 or int((off + F * w // 8).max()) > nbytes:
            bad("row offsets past the end of the codes")


def load_packed(path: str, device="cuda") -> Dict[int, dict]:
    import json
    from safetensors import safe_open
    out: Dict[int, dict] = {}
    with safe_open(path, framework="pt", device="cpu") as f:
        meta = f.metadata() or {}
        if meta.get("format") != _FORMAT:
            raise ValueError(f"{path}: not an {_FORMAT} file")
        for key, val in meta.items():
            if not key.startswith("L"):
                continue
            i = int(key[1:])
            m = json.loads(val)
            p = {name: f.get_tensor(f"L{i}.{name}") for name in _TENSORS}
            if m["dtype"] not in _DTYPES:
                raise ValueError(f"packed layer {i}: unknown dtype {m['dtype']}")
            p.update(rows=list(m["rows"]), bits=tuple(m["bits"]), dtype=_DTYPES[m["dtype"]],
                     feature_dim=int(m["feature_dim"]))
            _check_packed(i, p)
            for name in _TENSORS:
                p[name] = p[name].to(device)
            out[i] = p
    return dict(sorted(out.items()))


def unpack_layer(p: dict):
    """Packed layer dict → dense dequantized (K', V'), bit-identical to the fused output."""
    codes_k, codes_v = p["codes_k"], p["codes_v"]
    L.require_device(codes_k, codes_v)
    dev = codes_k.device
    row_offset = p["row_offset"].contiguous()
    scale_zp = p["scale_zp"].contiguous()
    kept_index = p["kept_index"].contiguous()
    labels = p["labels"].contiguous()
    B, Sp = kept_index.shape
    S = labels.shape[1]
    F = int(p["feature_dim"])
    dtype = p["dtype"]
    rows = torch.tensor(p["rows"], dtype=torch.int64, device=dev)
    bits = (ctypes.c_int32 * 3)(*p["bits"])
    outs = []
    for which, codes in ((0, codes_k), (1, codes_v)):
        out = torch.zeros(B, Sp, F, dtype=dtype, device=dev)
        if out.numel():
            L.check(L.lib().rtkv_unpack_dequant(codes.data_ptr(), row_offset.data_ptr(), scale_zp.data_ptr(), which,
                                                kept_index.data_ptr(), labels.data_ptr(), B, S, Sp, rows.data_ptr(), 1,
                                                F, L.TORCH_DTYPE_CODE[dtype], bits, out.data_ptr(), Sp * F, F, F,
                                                L.stream_ptr(dev)), "rtkv_unpack_dequant")
        outs.append(out)
    return outs[0], outs[1]


def decode_attention(p: dict, q: torch.Tensor, num_kv_heads: int, scale: Optional[float] = None) -> torch.Tensor:
    """Attention of one new token per batch row over a packed layer, decoded on the fly
    (rtkv_decode_attention_packed).  q: [B, Hq, D] in the layer's dtype; returns fp32 [B, Hq, D] =
    softmax(q·K'ᵀ·scale)·V' over the kept rows, with K'/V' exactly the dequantized rows
    (modified_llama.py:140-142 attends over those dequantized floats).  scale defaults to 1/sqrt(D)
    (modified_llama.py:89)."""
    codes_k, codes_v = p["codes_k"], p["codes_v"]
    L.require_device(codes_k, codes_v, q)
    dev = codes_k.device
    if q.dtype != p["dtype"]:
        raise ValueError(f"q dtype {q.dtype} does not match the packed layer's {p['dtype']}")
    B, Hq, D = q.shape
    F = int(p["feature_dim"])
    if num_kv_heads * D != F:
        raise ValueError(f"num_kv_heads * head_dim = {num_kv_heads * D} != feature_dim {F}")
    row_offset = p["row_offset"].contiguous()
    scale_zp = p["scale_zp"].contiguous()
    kept_index = p["kept_index"].contiguous()
    labels = p["labels"].contiguous()
    _check_dtypes("decode", p)
    # the kernel indexes every per-batch array by q's batch row: they must all have B rows
    if kept_index.dim() != 2 or kept_index.shape[0] != B or len(p["rows"]) != B or labels.shape[0] != B \
            or row_offset.shape[0] != B or scale_zp.shape[0] != B:
        raise ValueError(f"q has {B} batch rows but the packed layer has {kept_index.shape[0]} "
                         f"(rows {len(p['rows'])}, labels {labels.shape[0]})")
    Sp = kept_index.shape[1]
    if row_offset.shape != (B, Sp) or scale_zp.shape != (B, Sp, 4):
        raise ValueError("packed layer: row_offset / scale_zp shapes disagree with kept_index")
    S = labels.shape[1]
    out = torch.zeros(B, Hq, D, dtype=torch.float32, device=dev)
    if Sp == 0:
        return out
    rows = p.get("_rows_dev")
    if rows is None or rows.device != dev:  # kept once per layer: no host→device copy per decode step
        rows = p["_rows_dev"] = torch.tensor(p["rows"], dtype=torch.int64, device=dev)
    bits = (ctypes.c_int32 * 3)(*p["bits"])
    qc = q.contiguous()
    ws = torch.empty(L.lib().rtkv_decode_workspace_size(B, Hq, num_kv_heads, D, Sp), dtype=torch.uint8, device=dev)
    sc = float(scale) if scale is not None else 1.0 / float(D) ** 0.5
    if codes_k.numel() != codes_v.numel():
        raise ValueError("codes_k and codes_v differ in size")
    if any(int(r) < 0 or int(r) > Sp for r in p["rows"]):
        raise ValueError(f"row counts {p['rows']} outside [0, {Sp}]")
    L.check(L.lib().rtkv_decode_attention_packed(codes_k.data_ptr(), codes_v.data_ptr(), codes_k.numel(),
                                                 row_offset.data_ptr(),
                                                 scale_zp.data_ptr(), kept_index.data_ptr(), labels.data_ptr(), B, S,
                                                 Sp, rows.data_ptr(), num_kv_heads, D, L.TORCH_DTYPE_CODE[q.dtype],
                                                 bits, qc.data_ptr(), Hq, sc, out.data_ptr(), ws.data_ptr(),
                                                 ws.numel(), L.stream_ptr(dev)), "rtkv_decode_attention_packed")
    return out


class AdaptiveQuantization(nn.Module):
    """One scale/zero-point per precision class over all of that class's rows; bits by class index
    (compression_layers.py:96-175)."""

    def __init__(self, feature_dim: int, num_bits_options: list = [2, 4, 8]):
        super().__init__()
        self.feature_dim = feature_dim
        self.num_bits_options = num_bits_options
        self.quantization_params = {b: {"scale": torch.ones(1), "zero_point": torch.zeros(1)}
                                    for b in num_bits_options}

    def compute_quantization_params(self, tensor: torch.Tensor, num_bits: int):
        L.require_device(tensor)
        x = tensor.contiguous()
        sz = torch.empty(2, dtype=torch.float32, device=x.device)
        ws = _workspace(x.device).get(1, 1)
        L.check(L.lib().rtkv_tensor_quant_params(x.data_ptr(), L.dtype_code(x), 1, x.numel(), None, 0, int(num_bits),
                                                 sz.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(x.device)),
                "rtkv_tensor_quant_params")
        return sz[0], sz[1]

    def quantize_tensor(self, tensor, num_bits, scale, zero_point):
        L.require_device(tensor)
        x = tensor.contiguous()
        sz = torch.stack([torch.as_tensor(scale, device=x.device).float().reshape(()),
                          torch.as_tensor(zero_point, device=x.device).float().reshape(())])
        out = torch.empty_like(x)
        L.check(L.lib().rtkv_tensor_fake_quant(x.data_ptr(), L.dtype_code(x), 1, x.numel(), None, 0, int(num_bits),
                                               sz.data_ptr(), out.data_ptr(), L.stream_ptr(x.device)),
                "rtkv_tensor_fake_quant")
        return out

    def forward(self, tensor: torch.Tensor, precision_labels: torch.Tensor) -> torch.Tensor:
        L.require_device(tensor, precision_labels)
        x = tensor.contiguous()
        labels = precision_labels.to(torch.uint8).contiguous()
        n_rows = labels.numel()
        row_len = x.numel() // max(n_rows, 1)
        out = torch.zeros_like(x)
        dev = x.device
        st = L.stream_ptr(dev)
        present = torch.bincount(precision_labels.reshape(-1).long().clamp(0, 255), minlength=256).tolist()
        for level, bits in enumerate(self.num_bits_options):
            if level > 255 or present[level] == 0:
                continue
            sz = torch.empty(2, dtype=torch.float32, device=dev)
            ws = _workspace(dev).get(1, 1)
            L.check(L.lib().rtkv_tensor_quant_params(x.data_ptr(), L.dtype_code(x), n_rows, row_len, labels.data_ptr(),
                                                     level, int(bits), sz.data_ptr(), ws.data_ptr(), ws.numel(), st),
                    "rtkv_tensor_quant_params")
            L.check(L.lib().rtkv_tensor_fake_quant(x.data_ptr(), L.dtype_code(x), n_rows, row_len, labels.data_ptr(),
                                                   level, int(bits), sz.data_ptr(), out.data_ptr(), st),
                    "rtkv_tensor_fake_quant")
        return out
