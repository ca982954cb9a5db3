"""Dynamic precision assignment + per-token asymmetric quantization on the GPU.

Mirrors src/compression/dynamic_quantization.py of the reference (class DynamicPrecisionQuantizer,
same method names, arguments, return types):

    assign_precision_levels              :21-60   → rtkv_assign_precision
    get_quantization_params              :62-95   → rtkv_tensor_quant_params
    quantize_tensor                      :97-126  → rtkv_tensor_fake_quant
    apply_mixed_precision_quantization   :128-196 → rtkv_quantize_rows (every token, dequantized)
    estimate_memory_savings              :198-241 (host arithmetic on class counts)

Results are bit-identical to the reference's PyTorch CPU path (see tests/test_gpu_parity.py).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L
from .engine import decode_stats, kv_desc, params_from_config
from .token_importance import _workspace

F16_OVERFLOW_MSG = "value cannot be converted to type c10::Half without overflow"


class DynamicPrecisionQuantizer:
    """HIGH / MEDIUM / LOW classes by importance, quantized at high/medium/low_precision_bits."""

    def __init__(self, config):
        self.config = config
        self.theta_h = config.theta_h
        self.theta_m = config.theta_m
        self.high_bits = config.high_precision_bits
        self.medium_bits = config.medium_precision_bits
        self.low_bits = config.low_precision_bits

    def _bits(self):
        return (int(self.low_bits), int(self.medium_bits), int(self.high_bits))

    def assign_precision_levels(self, importance_scores: torch.Tensor):
        """[B,S] scores → (int64 labels 0=LOW/1=MID/2=HIGH, count statistics)."""
        L.require_device(importance_scores)
        s = importance_scores.to(torch.float32).contiguous()
        B, S = s.shape
        labels = torch.empty(B, S, dtype=torch.uint8, device=s.device)
        stats = torch.empty(L.stats_bytes(B), dtype=torch.uint8, device=s.device)
        p = params_from_config(self.config, 0, 1, 1.0, 0)
        p.theta_h, p.theta_m = float(self.theta_h), float(self.theta_m)
        if B * S:
            ws = _workspace(s.device).get(B, S)
            L.check(L.lib().rtkv_assign_precision(s.data_ptr(), B, S, ctypes.byref(p), labels.data_ptr(),
                                                  stats.data_ptr(), ws.data_ptr(), ws.numel(),
                                                  L.stream_ptr(s.device)), "rtkv_assign_precision")
            st = decode_stats(stats.cpu().numpy().tobytes(), B)
            high = sum(r["class_count"][2] for r in st.batch)
            medium = sum(r["class_count"][1] for r in st.batch)
        else:
            high = medium = 0
        total = B * S
        low = total - high - medium
        stats_d = {
            "high_count": high,
            "medium_count": medium,
            "low_count": low,
            "high_ratio": high / total,
            "medium_ratio": medium / total,
            "low_ratio": low / total,
        }
        return labels.long(), stats_d

    def get_quantization_params(self, tensor: torch.Tensor, num_bits: int):
        """(scale, zero_point) 0-dim tensors in the tensor's dtype over ALL elements."""
        L.require_device(tensor)
        x = tensor.contiguous()
        sz = torch.empty(2, dtype=torch.float32, device=x.device)
        ws = _workspace(x.device).get(1, 1)
        L.check(L.lib().rtkv_tensor_quant_params(x.data_ptr(), L.dtype_code(x), 1, x.numel(), None, 0, int(num_bits),
                                                 sz.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(x.device)),
                "rtkv_tensor_quant_params")
        sz = sz.to(x.dtype)
        return sz[0], sz[1]

    def quantize_tensor(self, tensor: torch.Tensor, num_bits: int, scale: torch.Tensor,
                        zero_point: torch.Tensor) -> torch.Tensor:
        """round/clamp to [0, 2^b-1] then dequantize, in the tensor's dtype."""
        L.require_device(tensor)
        x = tensor.contiguous()
        if x.dtype == torch.float16 and (1 << int(num_bits)) - 1 > 65504:
            raise RuntimeError(F16_OVERFLOW_MSG)
        sz = torch.stack([torch.as_tensor(scale, device=x.device).to(x.dtype).reshape(()),
                          torch.as_tensor(zero_point, device=x.device).to(x.dtype).reshape(())]).to(torch.float32)
        out = torch.empty_like(x)
        L.check(L.lib().rtkv_tensor_fake_quant(x.data_ptr(), L.dtype_code(x), 1, x.numel(), None, 0, int(num_bits),
                                               sz.data_ptr(), out.data_ptr(), L.stream_ptr(x.device)),
                "rtkv_tensor_fake_quant")
        return out

    def apply_mixed_precision_quantization(self, key_states: torch.Tensor, value_states: torch.Tensor,
                                           precision_labels: torch.Tensor):
        """Per-token fake quantization of K and V [B,S,F] at the bits of each token's class."""
        L.require_device(key_states, value_states, precision_labels)
        K, V = key_states.contiguous(), value_states.contiguous()
        B, S, F = K.shape
        labels = precision_labels.to(torch.uint8).contiguous()
        bits = self._bits()
        if K.dtype == torch.float16:
            present = [bool((precision_labels == g).any()) for g in range(3)]
            if any(present[g] and (1 << bits[g]) - 1 > 65504 for g in range(3)):
                raise RuntimeError(F16_OVERFLOW_MSG)
        qk = torch.zeros_like(K)
        qv = torch.zeros_like(V)
        quant_info = {"scales": {}, "zero_points": {}, "bit_assignments": precision_labels.detach().cpu().numpy()}
        if K.numel():
            p = params_from_config(self.config, 0, 1, 1.0, L.EMIT_DEQUANT | L.NO_SELECTION)
            p.bits[0], p.bits[1], p.bits[2] = bits
            kd = kv_desc(K, V, "bsf")
            out = L.LayerOut()
            out.k_out_dev, out.v_out_dev = qk.data_ptr(), qv.data_ptr()
            out.o_stride_b, out.o_stride_s, out.o_stride_h = S * F, F, F
            out.row_capacity = S
            L.check(L.lib().rtkv_quantize_rows(ctypes.byref(kd), labels.data_ptr(), None, ctypes.byref(p),
                                               ctypes.byref(out), L.stream_ptr(K.device)), "rtkv_quantize_rows")
        return qk, qv, quant_info

    def estimate_memory_savings(self, original_tensor: torch.Tensor, precision_labels: torch.Tensor):
        """Element counts by class × bits against a 16-bit original (dynamic_quantization.py:198-241)."""
        total_elements = original_tensor.numel()
        per_token = original_tensor.shape[-1]
        counts = torch.bincount(precision_labels.reshape(-1).long().clamp(0, 3), minlength=4).tolist()
        high_elements = counts[2] * per_token
        medium_elements = counts[1] * per_token
        low_elements = counts[0] * per_token
        original_memory = total_elements * 2
        compressed_memory = (high_elements * (self.high_bits / 8) + medium_elements * (self.medium_bits / 8)
                             + low_elements * (self.low_bits / 8))
        compression_ratio = compressed_memory / original_memory
        return {
            "original_memory_mb": original_memory / (1024 * 1024),
            "compressed_memory_mb": compressed_memory / (1024 * 1024),
            "compression_ratio": compression_ratio,
            "memory_savings": 1.0 - compression_ratio,
            "high_elements_ratio": high_elements / total_elements,
            "medium_elements_ratio": medium_elements / total_elements,
            "low_elements_ratio": low_elements / total_elements,
        }
