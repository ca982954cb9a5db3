"""CompressionConfig — field-for-field mirror of the reference's configs/base_config.py:4-56.

The compressor classes accept this dataclass or the reference's own CompressionConfig object (they
only read attributes).  Behaviour is kept identical, including the reference's ZeroDivisionError
for num_hidden_layers = 1 with default layer_weights (base_config.py:47-51).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional


@dataclass
class CompressionConfig:
    # Model configuration
    model_name: str = "meta-llama/Llama-2-7b-hf"
    max_position_embeddings: int = 4096
    num_hidden_layers: int = 32
    hidden_size: int = 4096
    num_attention_heads: int = 32

    # Compression hyperparameters (token_importance.py:163-171)
    alpha: float = 0.4
    beta: float = 0.3
    gamma: float = 0.3

    # Importance thresholds (dynamic_quantization.py:41-42)
    theta_h: float = 0.7
    theta_m: float = 0.3

    # Layer-specific weights (decreasing for later layers)
    layer_weights: Optional[List[float]] = None

    # Propagation ratios for the three layer groups (selective_propagation.py:23-38)
    early_layer_ratio: float = 0.8
    middle_layer_ratio: float = 0.6
    later_layer_ratio: float = 0.4

    # Quantization bits by precision class
    high_precision_bits: int = 16
    medium_precision_bits: int = 8
    low_precision_bits: int = 4

    # Memory and performance (unused by the reference path)
    memory_budget_ratio: float = 0.5
    quality_loss_tolerance: float = 0.05

    # Evaluation settings
    context_lengths: List[int] = None
    batch_sizes: List[int] = None

    def __post_init__(self):
        if self.layer_weights is None:
            self.layer_weights = [
                1.0 - 0.5 * (i / (self.num_hidden_layers - 1))
                for i in range(self.num_hidden_layers)
            ]
        if self.context_lengths is None:
            self.context_lengths = [4096, 8192, 16384, 32768]
        if self.batch_sizes is None:
            self.batch_sizes = [1, 4, 8]
