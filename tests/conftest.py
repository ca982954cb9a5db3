"""Test configuration: `gpu` marker, import paths, shared fixture loading.

CPU tests (`-m "not gpu"`): oracle vs the reference's golden fixtures, ABI/export checks, host logic,
multi-process (gloo) sharding logic.  GPU tests (`-m gpu`): the HIP path through the C ABI against
the fixtures and the oracle.
"""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "realtime-kv-cache-compression_amd")
for p in (PKG, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests", "golden"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

FIXTURES = os.path.join(REPO, "tests", "golden", "fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and librtkv.so")


def load_manifest():
    with open(os.path.join(FIXTURES, "manifest.json")) as f:
        return json.load(f)


def load_case(case):
    """(arrays dict, case) — arrays holds the stored (small) expected outputs."""
    with np.load(os.path.join(FIXTURES, case["name"] + ".npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    return arrays


def sha256(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def assert_matches(case, key, actual, arrays):
    """Bitwise check of `actual` against the fixture's stored array or its sha256."""
    actual = np.ascontiguousarray(actual)
    if key in arrays:
        exp = arrays[key]
        assert actual.shape == exp.shape, f"{case['name']}:{key} shape {actual.shape} != {exp.shape}"
        if not np.array_equal(actual.view(np.uint8), exp.view(np.uint8)):
            bad = np.nonzero(actual.reshape(-1) != exp.reshape(-1))[0]
            raise AssertionError(f"{case['name']}:{key}: {bad.size} mismatches, first at {bad[:5]}")
    else:
        assert list(actual.shape) == case["shapes"][key], f"{case['name']}:{key} shape"
        assert sha256(actual) == case["sha256"][key], f"{case['name']}:{key} sha256 mismatch"


@pytest.fixture(scope="session")
def manifest():
    return load_manifest()
