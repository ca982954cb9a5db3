"""Budgeted selective token propagation on the GPU.

Mirrors src/compression/selective_propagation.py of the reference (class SelectiveTokenPropagator):

    get_layer_propagation_ratio   :23-38   host (layer-group boundaries int(0.3L), int(0.7L))
    compute_token_costs           :40-66   cost = bits(class)/8
    select_tokens_with_budget     :68-161  → rtkv_select_tokens (closed-form greedy, no sort)
    apply_token_selection         :163-244 → rtkv_select_tokens (+ fallback) + rtkv_gather_rows
    estimate_compression_ratio    :246-259 host

Ties among equal scores are broken by ascending token index (the reference's CPU argsort is not
stable; see tests/golden/gen_golden.py for how fixtures flag tie-dependent cases).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib as L
from .engine import decode_stats, params_from_config
from .token_importance import _workspace


class SelectiveTokenPropagator:
    """Keep, per layer, the most important tokens whose summed cost fits S·ratio."""

    def __init__(self, config):
        self.config = config
        self.early_layer_ratio = config.early_layer_ratio
        self.middle_layer_ratio = config.middle_layer_ratio
        self.later_layer_ratio = config.later_layer_ratio
        n_layers = config.num_hidden_layers
        self.early_boundary = int(0.3 * n_layers)
        self.middle_boundary = int(0.7 * n_layers)

    def get_layer_propagation_ratio(self, layer_idx: int) -> float:
        if layer_idx < self.early_boundary:
            return self.early_layer_ratio
        if layer_idx < self.middle_boundary:
            return self.middle_layer_ratio
        return self.later_layer_ratio

    def _bits(self):
        c = self.config
        return (int(c.low_precision_bits), int(c.medium_precision_bits), int(c.high_precision_bits))

    def compute_token_costs(self, precision_labels: torch.Tensor) -> torch.Tensor:
        """[B,S] classes → fp32 costs bits/8 (0 for labels outside {0,1,2})."""
        table = torch.tensor([b / 8 for b in self._bits()] + [0.0], dtype=torch.float32,
                             device=precision_labels.device)
        idx = precision_labels.long()
        idx = torch.where((idx >= 0) & (idx <= 2), idx, torch.full_like(idx, 3))
        return table[idx]

    # ------------------------------------------------------------------ device selection
    def _run_select(self, scores, labels, ratio, fallback: bool, F: int = 0, kv_dtype: int = -1):
        L.require_device(scores, labels)
        s = scores.to(torch.float32).contiguous()
        B, S = s.shape
        lab = labels.to(torch.uint8).contiguous()
        dev = s.device
        mask = torch.empty(B, S, dtype=torch.uint8, device=dev)
        kept_index = torch.empty(B, S, dtype=torch.int32, device=dev)
        stats = torch.empty(L.stats_bytes(B), dtype=torch.uint8, device=dev)
        p = params_from_config(self.config, 0, 1, float(ratio), 0 if fallback else L.NO_FALLBACK)
        ws = _workspace(dev).get(B, S)
        L.check(L.lib().rtkv_select_tokens(s.data_ptr(), lab.data_ptr(), B, S, ctypes.byref(p), mask.data_ptr(),
                                           kept_index.data_ptr(), S, None, F, kv_dtype, stats.data_ptr(),
                                           ws.data_ptr(), ws.numel(), L.stream_ptr(dev)), "rtkv_select_tokens")
        return s, mask, kept_index, stats

    def _selection_info(self, s, st, ratio, S):
        """selection_info dict of select_tokens_with_budget (selective_propagation.py:80-158)."""
        total_budget = S * ratio
        info = {"selected_counts": [], "budget_utilization": [], "avg_importance": [],
                "cost_distribution": {"high": 0, "medium": 0, "low": 0}}
        for row in st.batch:
            n = row["kept"]
            if n == 0 or row["fallback"]:  # the greedy itself selected nothing in a fallback layer
                continue
            info["selected_counts"].append(n)
            info["budget_utilization"].append((row["cost_units"] / 8.0) / total_budget)
            info["avg_importance"].append(row["kept_score_sum"] / n)
            info["cost_distribution"]["low"] += row["kept_class"][0]
            info["cost_distribution"]["medium"] += row["kept_class"][1]
            info["cost_distribution"]["high"] += row["kept_class"][2]
        if info["selected_counts"]:
            k = len(info["selected_counts"])
            info["avg_selected"] = sum(info["selected_counts"]) / k
            info["avg_budget_util"] = sum(info["budget_utilization"]) / k
            info["overall_avg_importance"] = sum(info["avg_importance"]) / k
        return info

    def select_tokens_with_budget(self, importance_scores: torch.Tensor, precision_labels: torch.Tensor,
                                  budget_ratio: float, layer_idx: int):
        """→ (bool selection mask [B,S], selection statistics)."""
        s, mask, _, stats = self._run_select(importance_scores, precision_labels, budget_ratio, fallback=False)
        st = decode_stats(stats.cpu().numpy().tobytes(), s.shape[0])
        return mask.bool(), self._selection_info(s, st, budget_ratio, s.shape[1])

    def apply_token_selection(self, key_states: torch.Tensor, value_states: torch.Tensor,
                              importance_scores: torch.Tensor, precision_labels: torch.Tensor, layer_idx: int,
                              input_ids: Optional[torch.Tensor] = None):
        """Select (with the top-10% fallback) and gather K, V, scores and labels of the kept tokens
        in ascending index order, zero-padded across the batch."""
        L.require_device(key_states, value_states)
        ratio = self.get_layer_propagation_ratio(layer_idx)
        s, mask, kept_index, stats = self._run_select(importance_scores, precision_labels, ratio, fallback=True)
        B, S = s.shape
        st = decode_stats(stats.cpu().numpy().tobytes(), B)
        Sp = st.max_kept
        info = self._selection_info(s, st, ratio, S)
        dev = s.device
        st_ptr = stats.data_ptr()
        stream = L.stream_ptr(dev)

        def gather(x: torch.Tensor, shape_tail):
            x = x.contiguous()
            row_bytes = x.element_size() * (x[0, 0].numel() if x.dim() > 2 else 1)
            out = torch.empty((B, Sp) + shape_tail, dtype=x.dtype, device=dev)
            if out.numel():
                L.check(L.lib().rtkv_gather_rows(x.data_ptr(), B, S, row_bytes, kept_index.data_ptr(), S,
                                                 x.stride(0) * x.element_size(), out.data_ptr(), -1,
                                                 x.stride(1) * x.element_size(), st_ptr, stream), "rtkv_gather_rows")
            return out

        sel_k = gather(key_states, tuple(key_states.shape[2:]))
        sel_v = gather(value_states, tuple(value_states.shape[2:]))
        sel_s = gather(importance_scores.to(dev), ())
        sel_l = gather(precision_labels.to(dev), ())
        propagation_info = {
            "layer_idx": layer_idx,
            "propagation_ratio": ratio,
            "original_length": S,
            "max_selected_length": Sp,
            "selection_mask": mask.bool(),
            "selection_stats": info,
        }
        return sel_k, sel_v, sel_s, sel_l, propagation_info

    def estimate_compression_ratio(self, layer_idx: int, original_length: int):
        cumulative = 1.0
        for l in range(layer_idx + 1):
            cumulative *= self.get_layer_propagation_ratio(l)
        return {
            "layer_ratio": self.get_layer_propagation_ratio(layer_idx),
            "cumulative_ratio": cumulative,
            "estimated_length": int(original_length * cumulative),
            "compression_factor": 1.0 / cumulative,
        }
