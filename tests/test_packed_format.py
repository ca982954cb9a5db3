"""CPU: the packed-layer file format ("rtkv-packed/1", compression_layers.save_packed / load_packed).

A packed layer is built on the host with the same layout rtkv_compress_layer emits (rows back to back,
F·w/8 bytes each, offsets per kept row); it must survive a save → load round trip bit for bit, and
every inconsistent file (truncated codes, an offset past the end, a kept index outside the row, a
foreign file) must raise ValueError at load time, before any kernel could read it."""
import numpy as np
import pytest
import torch


@pytest.fixture(scope="module")
def rtkv():
    import rtkv
    return rtkv


def packed_layer(seed=0, B=2, S=40, F=512, bits=(2, 4, 8), dtype=torch.float16):
    rng = np.random.default_rng(seed)
    labels = torch.from_numpy(rng.integers(0, 3, (B, S)).astype(np.uint8))
    rows, kept, offs = [], [], []
    off = 0
    Sp = 0
    for b in range(B):
        idx = np.sort(rng.choice(S, size=rng.integers(1, S), replace=False)).astype(np.int32)
        kept.append(idx)
        Sp = max(Sp, len(idx))
    kept_index = torch.zeros(B, Sp, dtype=torch.int32)
    row_offset = torch.zeros(B, Sp, dtype=torch.int64)
    for b in range(B):
        idx = kept[b]
        rows.append(len(idx))
        kept_index[b, :len(idx)] = torch.from_numpy(idx)
        for j, i in enumerate(idx):
            row_offset[b, j] = off
            off += F * bits[int(labels[b, i])] // 8
    codes_k = torch.from_numpy(rng.integers(0, 256, off).astype(np.uint8))
    codes_v = torch.from_numpy(rng.integers(0, 256, off).astype(np.uint8))
    scale_zp = torch.from_numpy(rng.standard_normal((B, Sp, 4)).astype(np.float32))
    return dict(codes_k=codes_k, codes_v=codes_v, row_offset=row_offset, scale_zp=scale_zp,
                kept_index=kept_index, labels=labels, rows=rows, bits=bits, dtype=dtype, feature_dim=F)


def same(p, q):
    for k in ("codes_k", "codes_v", "row_offset", "scale_zp", "kept_index", "labels"):
        assert p[k].dtype == q[k].dtype and torch.equal(p[k].cpu(), q[k].cpu()), k
    assert list(p["rows"]) == list(q["rows"]) and tuple(p["bits"]) == tuple(q["bits"])
    assert p["dtype"] == q["dtype"] and p["feature_dim"] == q["feature_dim"]


def test_round_trip(rtkv, tmp_path):
    layers = {0: packed_layer(0), 3: packed_layer(1, dtype=torch.bfloat16), 7: packed_layer(2, B=1, F=1024,
                                                                                              bits=(4, 8, 16),
                                                                                              dtype=torch.float32)}
    path = str(tmp_path / "cache.safetensors")
    rtkv.save_packed(layers, path)
    back = rtkv.load_packed(path, device="cpu")
    assert list(back) == [0, 3, 7]
    for i in layers:
        same(layers[i], back[i])


def test_cache_container_round_trip(rtkv, tmp_path):
    cache = rtkv.CompressedKVCache(2, 40, 128)
    cache.store_packed(2, packed_layer(5))
    path = str(tmp_path / "c.safetensors")
    cache.save(path)
    other = rtkv.CompressedKVCache(2, 40, 128)
    other.load(path, device="cpu")
    same(cache.compression_info[2], other.compression_info[2])
    assert other.packed_nbytes(2) == cache.packed_nbytes(2)


@pytest.mark.parametrize("breakage", ["truncated", "offset", "kept_index", "rows", "label"])
def test_inconsistent_files_raise(rtkv, tmp_path, breakage):
    p = packed_layer(3)
    if breakage == "truncated":
        p["codes_k"] = p["codes_k"][:-1]
        p["codes_v"] = p["codes_v"][:-1]
    elif breakage == "offset":
        p["row_offset"][0, 0] = p["codes_k"].numel()
    elif breakage == "kept_index":
        p["kept_index"][1, 0] = 40
    elif breakage == "rows":
        p["rows"] = [p["rows"][0], p["kept_index"].shape[1] + 1]
    else:
        p["labels"][0, int(p["kept_index"][0, 0])] = 3
    path = str(tmp_path / "bad.safetensors")
    rtkv.save_packed({0: p}, path)
    with pytest.raises(ValueError):
        rtkv.load_packed(path, device="cpu")


def test_foreign_file_raises(rtkv, tmp_path):
    from safetensors.torch import save_file
    path = str(tmp_path / "foreign.safetensors")
    save_file({"x": torch.zeros(3)}, path)
    with pytest.raises(ValueError):
        rtkv.load_packed(path, device="cpu")
