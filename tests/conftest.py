import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "learnable-triangulation-pytorch_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box: pytest -m gpu)")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(autouse=True)
def _device_asserts(request):
    """With the debug library loaded (MVN_HIP_LIB=.../libmvn_hip_debug.so, `make debug`), fail
    a GPU test whose kernels tripped a device-side assertion (csrc/common.hpp MVN_DASSERT:
    index / layout invariants, counted instead of trapping)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    from mvn_rocm import _lib
    if _lib._lib is None:
        return
    import torch
    if not torch.cuda.is_available():
        return
    enabled, count, line = _lib.device_asserts()
    if enabled:
        assert count == 0, f"{count} device-side assertion failure(s), the first at source line {line}"


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch.device("cuda:0")


def assert_bits_equal(a, b):
    """float32 arrays equal bit for bit: unlike assert_array_equal, +0 vs -0 (and NaN
    payloads) count as differences — grid_sample's zero padding yields +0, and a kernel that
    multiplies a clamped negative pixel by a zero weight yields -0."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    assert a.shape == b.shape, (a.shape, b.shape)
    bad = a.view(np.uint32) != b.view(np.uint32)
    assert not bad.any(), f"{int(bad.sum())} of {bad.size} elements differ in their bits (first: {a[bad][:4]} vs {b[bad][:4]})"


def assert_parity_with_nans(out, ref, method, tol=1e-5):
    """NaN at the same elements; elsewhere bit-equal (softmax: max_rel <= tol)."""
    out, ref = np.asarray(out, np.float32), np.asarray(ref, np.float32)
    nan_o, nan_r = np.isnan(out), np.isnan(ref)
    assert (nan_o == nan_r).all(), f"NaN at {int((nan_o != nan_r).sum())} differing elements"
    fin = ~nan_r
    if method == "softmax":
        assert max_rel(out[fin], ref[fin]) <= tol
    else:
        assert_bits_equal(out[fin], ref[fin])


def max_rel(a, b):
    """max |a - b| / max |b| (SURVEY.md §8d parity metric)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.abs(b).max()
    return float(np.abs(a - b).max() / (den if den > 0 else 1.0))
