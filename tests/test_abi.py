"""CPU: librtkv.so builds for gfx950, loads, and exports every entry point include/rtkv.h declares.
Only pure host functions are called here (no GPU in this container)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "rtkv.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rtkv_\w+)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if n != "rtkv_stats_bytes"))  # static inline helper


@pytest.fixture(scope="module")
def lib():
    import rtkv._lib as L
    L.build()
    return L.lib()


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["rtkv_compress_layer", "rtkv_attention_aggregation", "rtkv_importance_scores",
                 "rtkv_assign_precision", "rtkv_select_tokens", "rtkv_quantize_rows", "rtkv_unpack_dequant",
                 "rtkv_gather_rows", "rtkv_position_bias", "rtkv_minmax_normalize", "rtkv_tensor_quant_params",
                 "rtkv_tensor_fake_quant", "rtkv_last_error", "rtkv_version", "rtkv_workspace_size"]:
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    for name in declared_functions():
        assert hasattr(lib, name), f"{name} declared in rtkv.h but not exported by librtkv.so"


def test_python_binding_covers_every_export():
    import rtkv._lib as L
    assert sorted(L.EXPORTS) == declared_functions()


def test_library_is_gfx950_code(lib):
    so = open(os.path.join(PKG, "librtkv.so"), "rb").read()
    assert b".hip_fatbin" in so or b"__CLANG_OFFLOAD_BUNDLE__" in so
    assert b"amdgcn-amd-amdhsa--gfx950" in so


def test_host_helpers(lib):
    assert lib.rtkv_version().decode().startswith("rtkv")
    # field widths: exact integer codes fit in `bits`; the clamp bound rounds up in half types
    assert lib.rtkv_field_width(0, 16) == 16
    assert lib.rtkv_field_width(0, 2) == 2
    assert lib.rtkv_field_width(1, 8) == 8
    assert lib.rtkv_field_width(1, 12) == 13
    assert lib.rtkv_field_width(1, 16) == 0   # the reference raises for fp16 at 16 bits
    assert lib.rtkv_field_width(2, 8) == 8
    assert lib.rtkv_field_width(2, 9) == 10
    assert lib.rtkv_field_width(0, 0) == 0 and lib.rtkv_field_width(0, 17) == 0
    assert lib.rtkv_workspace_size(1, 16384) >= 16384 * 5
    bits = (ctypes.c_int32 * 3)(2, 4, 8)
    assert lib.rtkv_packed_capacity(1, 16384, 4096, 1, bits) == 16384 * 4096


def test_struct_layouts_match_header():
    import rtkv._lib as L
    assert ctypes.sizeof(L.LayerParams) == 56
    assert ctypes.sizeof(L.AttnDesc) == 72
    assert ctypes.sizeof(L.KVDesc) == 80
    assert ctypes.sizeof(L.BatchStats) == 88
    assert ctypes.sizeof(L.LayerStatsHeader) == 48
    assert ctypes.sizeof(L.LayerOut) == 128
    assert ctypes.alignment(L.LayerParams) == 8


def test_no_gpu_means_loud_failure():
    import torch
    import rtkv
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    cfg = rtkv.CompressionConfig(num_hidden_layers=2)
    comp = rtkv.RealTimePrefillCompressor(cfg)
    K = torch.zeros(1, 8, 16)
    with pytest.raises(RuntimeError, match="ROCm"):
        comp.compress_layer_kv_cache(K, K, torch.zeros(1, 2, 8, 8), torch.zeros(1, 8, dtype=torch.long), 0)


def test_early_line_must_be_128_byte_aligned(lib):
    """The early statistics line is one 128-byte store checked by its first and last words: a buffer that
    straddles two lines is refused by every entry point that takes it (host-only calls here)."""
    buf = ctypes.create_string_buffer(1024)
    base = (ctypes.addressof(buf) + 127) // 128 * 128
    lib.rtkv_wait_early.restype = ctypes.c_int
    assert lib.rtkv_wait_early(ctypes.c_void_p(base + 8), ctypes.c_uint64(1), ctypes.c_int64(0)) == -1
    assert "128-byte aligned" in lib.rtkv_last_error().decode()
    assert lib.rtkv_wait_final(ctypes.c_void_p(base + 64), ctypes.c_uint64(1), ctypes.c_int64(0)) == -1
    # aligned: a plain timeout (nothing published)
    assert lib.rtkv_wait_early(ctypes.c_void_p(base), ctypes.c_uint64(1), ctypes.c_int64(0)) == -5
