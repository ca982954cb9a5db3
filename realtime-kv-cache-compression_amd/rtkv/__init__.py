"""rtkv — MI355X-native (gfx950, HIP) streaming prefill KV-cache compression.

Drop-in for the hot path of EvelynHung-79/RealTime-KV-cache-Compression:
token importance → dynamic precision quantization → selective propagation, with the reference's
class and method names.  All compute runs in librtkv.so (include/rtkv.h); there is no CPU path.
"""
from . import _lib
from .base_config import CompressionConfig
from .compression_layers import (AdaptiveQuantization, CompressedKVCache, decode_attention, load_packed, save_packed,
                                 unpack_layer)
from .dynamic_quantization import DynamicPrecisionQuantizer
from .group_quant import GroupQuantConfig, GroupQuantKVCache, gq_compress
from .engine import (LayerBuffers, LayerResult, Workspace, attention_lse, compress_layer, compress_layer_qk,
                     importance_qk_lse, params_from_config, prompt_length)
from .model_side import CompressedPrefillAttention
from .selective_propagation import SelectiveTokenPropagator
from .token_importance import LayerWiseImportanceTracker, PromptGuidedImportanceScorer
from .unified_compressor import CompressionHook, RealTimePrefillCompressor, UnifiedCompressor

__all__ = [
    "CompressionConfig", "RealTimePrefillCompressor", "UnifiedCompressor", "CompressionHook",
    "PromptGuidedImportanceScorer", "LayerWiseImportanceTracker", "DynamicPrecisionQuantizer",
    "SelectiveTokenPropagator", "CompressedKVCache", "AdaptiveQuantization", "unpack_layer", "decode_attention",
    "save_packed", "load_packed", "CompressedPrefillAttention",
    "LayerBuffers", "LayerResult", "Workspace", "compress_layer", "compress_layer_qk", "importance_qk_lse", "attention_lse",
    "params_from_config", "prompt_length", "GroupQuantConfig", "GroupQuantKVCache", "gq_compress",
]

__version__ = "0.1.0"


def build(force: bool = False) -> str:
    """Compile librtkv.so for gfx950 in-tree."""
    return _lib.build(force)
