"""C ABI of libmvn_hip.so and the host-side checks of mvn_rocm — no GPU needed
(only argument-validation paths are called; they return before any HIP call)."""
import os
import re
import subprocess

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mvn_hip.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(mvn_\w+)\s*\(", text, re.M)))


@pytest.fixture(scope="module")
def lib():
    from mvn_rocm import _lib
    return _lib.load()


def test_header_declares_the_three_entry_points():
    fns = header_functions()
    for name in ("mvn_unproject", "mvn_softargmax3d", "mvn_dlt", "mvn_softargmax2d", "mvn_coord_volumes",
                 "mvn_nearest_voxel", "mvn_unproject_ex", "mvn_v2v_front",
                 "mvn_softargmax3d_workspace_bytes",
                 "mvn_strerror", "mvn_version"):
        assert name in fns


def test_every_declared_symbol_is_exported(lib):
    from mvn_rocm import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT\s+(mvn_\w+)", out))
    for name in header_functions():
        assert name in exported, name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
        getattr(lib, name)


def test_debug_build_exports_the_same_symbols_and_reports_itself(lib):
    """The debug build (device-side assertions, `make debug`) is a drop-in for the release
    library: the same C ABI; mvn_debug_device_asserts says which build it is."""
    import ctypes
    from mvn_rocm import _lib
    dbg = os.path.join(os.path.dirname(_lib.__file__), "libmvn_hip_debug.so")
    if not os.path.exists(dbg):
        pytest.skip("debug library not built (make -C learnable-triangulation-pytorch_amd debug)")
    out = subprocess.run(["nm", "-D", "--defined-only", dbg], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT\s+(mvn_\w+)", out))
    assert set(header_functions()) <= exported
    en, cnt, line = ctypes.c_int(7), ctypes.c_uint(7), ctypes.c_uint(7)
    assert lib.mvn_debug_device_asserts(ctypes.byref(en), ctypes.byref(cnt), ctypes.byref(line)) == 0
    assert (en.value, cnt.value, line.value) == (0, 0, 0)          # release build: no checks compiled in
    assert lib.mvn_debug_device_asserts(None, ctypes.byref(cnt), ctypes.byref(line)) == -1


def test_version_and_errors(lib):
    assert lib.mvn_version() == (0 << 16) | (1 << 8)
    for code in (0, -1, -2, -3, -4, -5):
        assert lib.mvn_strerror(code)
    assert lib.mvn_strerror(-99) == b"unknown error"


def _unproject(lib, **kw):
    a = dict(feat=1, fdt=0, proj=1, coords=1, conf=None, out=1, odt=0, B=1, N=4, C=32, H=96, W=96,
             Vx=64, Vy=64, Vz=64, agg=2, ac=0)
    a.update(kw)
    return lib.mvn_unproject(a["feat"], a["fdt"], a["proj"], a["coords"], a["conf"], a["out"], a["odt"],
                             a["B"], a["N"], a["C"], a["H"], a["W"], a["Vx"], a["Vy"], a["Vz"], a["agg"], a["ac"],
                             None)


def test_unproject_argument_validation(lib):
    assert _unproject(lib, feat=None) == -1
    assert _unproject(lib, agg=7) == -1
    assert _unproject(lib, agg=3, conf=None) == -1          # 'conf' aggregation needs confidences
    assert _unproject(lib, ac=2) == -1
    assert _unproject(lib, B=0) == -2
    assert _unproject(lib, W=-1) == -2
    assert _unproject(lib, Vx=2048, Vy=2048, Vz=2048) == -2
    assert _unproject(lib, fdt=0, odt=1) == -3               # f32 features -> bf16 volume unsupported


def test_unproject_precision_argument_validation(lib):
    """mvn_unproject_precision: exactly one coordinate source, a known precision, cuboids only
    for cubic volumes of <= 8 views — all checked before any HIP call."""
    def call(**kw):
        a = dict(coords=1, cub=None, N=4, Vz=64, prec=1)
        a.update(kw)
        return lib.mvn_unproject_precision(1, 0, 1, a["coords"], a["cub"], 0, None, 1, 0, 0, 1, a["N"], 32, 96, 96,
                                           64, 64, a["Vz"], 2, 0, a["prec"], None)
    assert call(coords=None) == -1
    assert call(coords=1, cub=1) == -1
    assert call(prec=2) == -1
    assert call(prec=-1) == -1
    assert call(coords=None, cub=1, Vz=32) == -2
    assert call(coords=None, cub=1, N=9) == -2
    from mvn_rocm import op
    with pytest.raises(ValueError, match="Unknown unprojection precision"):
        op.precision_code("fp8")
    with pytest.raises(ValueError):
        op.set_unproject_precision("approximate")
    assert op.precision_code(None) == op.precision_code("exact") == 0 and op.precision_code("fast") == 1
    prev = op.set_unproject_precision("fast")
    try:
        assert op.precision_code(None) == 1
    finally:
        op.set_unproject_precision(prev)


def test_channels_last_paths_refuse_autograd():
    """the channels-last unprojection and the one-call V2V pipeline have no backward;
    with grad mode on and a feature or confidence tensor that requires grad they raise instead
    of returning a volume whose confidence gradient is silently lost."""
    from mvn_rocm import v2v
    feat = torch.zeros(1, 4, 32, 8, 8)
    conf = torch.ones(1, 4, 32, requires_grad=True)
    P, coords = torch.zeros(1, 4, 3, 4), torch.zeros(1, 4, 4, 4, 3)
    with pytest.raises(RuntimeError, match="inference-only"):
        v2v.unproject_channels_last(feat, P, coords, "conf", vol_confidences=conf)
    with pytest.raises(RuntimeError, match="inference-only"):
        v2v.unproject_v2v_front(feat.requires_grad_(), P, coords, None, None, None, "softmax")
    with torch.no_grad(), pytest.raises(RuntimeError, match="no CPU fallback"):
        v2v.unproject_channels_last(feat, P, coords, "conf", vol_confidences=conf)


def test_softargmax_argument_validation(lib):
    ws = lib.mvn_softargmax3d_workspace_bytes(32, 17, 64, 64, 64)
    assert ws == 32 * 17 * (256 * 5 + 2) * 4          # 1024-voxel partial chunks
    assert lib.mvn_softargmax3d_workspace_bytes(0, 17, 64, 64, 64) == 0
    call = lambda **k: lib.mvn_softargmax3d(
        k.get("vol", 1), 0, 17 * 64 ** 3, 64 ** 3, 1, 1.0, k.get("sm", 1), 1, None, 0, k.get("ws", 1),
        k.get("wsb", ws), 32, 17, 64, 64, 64, None)
    assert call(vol=None) == -1
    assert call(sm=3) == -1
    assert call(ws=None) == -5
    assert call(wsb=ws - 4) == -5


def test_dlt_argument_validation(lib):
    assert lib.mvn_dlt(None, 1, None, 1, 1, 4, 17, None) == -1
    assert lib.mvn_dlt(1, 1, None, 1, 1, 0, 17, None) == -2


def test_python_api_has_no_cpu_fallback():
    from mvn_rocm import op, multiview
    feat = torch.zeros(1, 2, 3, 8, 8)
    P = torch.zeros(1, 2, 3, 4)
    coords = torch.zeros(1, 4, 4, 4, 3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        op.unproject_heatmaps(feat, P, coords, "softmax")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        op.integrate_tensor_3d_with_coordinates(torch.zeros(1, 2, 4, 4, 4), coords)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        multiview.triangulate_batch_of_points(P, torch.zeros(1, 2, 5, 2))


def test_python_api_error_types_match_reference():
    from mvn_rocm import op, multiview
    feat = torch.zeros(1, 2, 3, 8, 8)
    P = torch.zeros(1, 2, 3, 4)
    coords = torch.zeros(1, 4, 4, 4, 3)
    with pytest.raises(ValueError, match="Unknown volume_aggregation_method: mean"):   # op.py:161
        op.unproject_heatmaps(feat, P, coords, "mean")
    with pytest.raises(AssertionError):                                                # multiview.py:143
        multiview.triangulate_batch_of_points(torch.zeros(1, 3, 3, 4), torch.zeros(1, 2, 5, 2))
    assert op.aggregation_code("conf_norm") == op.aggregation_code("conf")             # op.py:147


def test_unproject_v2v_front_argument_validation(lib):
    """The one-call config-5 pipeline: exactly one coordinate source, 32 channels, V % 16,
    'conf' aggregation only through the _ex form, a workspace of one group (no HIP call on
    these paths)."""
    assert lib.mvn_unproject_v2v_front_workspace_bytes(8, 64) == 8 * 64 ** 3 * 32 * 2
    assert lib.mvn_unproject_v2v_front_workspace_bytes(0, 64) == 8 * 64 ** 3 * 32 * 2     # default: 8 frames
    ws = lib.mvn_unproject_v2v_front_workspace_bytes(2, 64)

    def call(**k):
        return lib.mvn_unproject_v2v_front(k.get("feat", 1), 0, 1, k.get("coords", 1), k.get("cub", None), 0,
                                           k.get("agg", 2), 0, 1, 1, 1, 1, 0, k.get("ws", 1), k.get("wsb", ws),
                                           2, 3, 4, k.get("C", 32), 96, 96, k.get("V", 64), None)
    assert call(feat=None) == -1
    assert call(coords=None) == -1                      # neither coordinate source
    assert call(cub=1) == -1                            # both
    assert call(agg=3) == -1                            # conf*
    assert call(C=16) == -2
    assert call(V=40) == -2
    assert call(ws=None) == -5
    assert call(wsb=ws - 1) == -5

    # the _ex form takes 'conf*' with the (B, N, C) confidences (triangulation.py:349)
    def call_ex(**k):
        return lib.mvn_unproject_v2v_front_ex(1, 0, 1, 1, None, 0, k.get("agg", 3), k.get("conf", None), 0, 1, 1, 1,
                                              1, 0, k.get("ws", 1), ws, 2, 3, 4, 32, 96, 96, 64, None)
    assert call_ex(agg=3, conf=None) == -1               # conf* without confidences
    assert call_ex(agg=3, conf=1, ws=None) == -5         # (validated up to the workspace: no HIP call)


def test_channels_last_conf_needs_confidences():
    """'conf*' on the channels-last and one-call config-5 paths needs vol_confidences, as
    unproject_heatmaps does (TypeError before any device work)."""
    from mvn_rocm import v2v
    feat, P, coords = torch.zeros(1, 4, 32, 8, 8), torch.zeros(1, 4, 3, 4), torch.zeros(1, 16, 16, 16, 3)
    with pytest.raises(TypeError, match="vol_confidences"):
        v2v.unproject_channels_last(feat, P, coords, "conf_norm")
    with pytest.raises(TypeError, match="vol_confidences"):
        v2v.unproject_v2v_front(feat, P, coords, None, None, None, "conf")


def test_deterministic_backward_argument_checks(lib):
    """mvn_unproject_backward_deterministic validates before any HIP call: the workspace
    (a header for the per-call scale and its partial maxima, then 64-bit fixed-point sums: one per feature
    element and per confidence) must be present and large enough (MVN_ERR_WORKSPACE), shapes
    and enums as mvn_unproject_backward."""
    B, N, C, H, W = 2, 4, 8, 24, 24
    need = lib.mvn_unproject_backward_workspace_bytes(B, N, C, H, W)
    # header, per-(frame, channel) scales (padded to 256 B), a 64-bit sum and a flag word per element
    assert need == 256 + (B * C * 8 + 255) // 256 * 256 + (B * N * C * H * W + B * N * C) * (8 + 4)
    assert lib.mvn_unproject_backward_workspace_bytes(0, N, C, H, W) == 0

    def call(ws=1, ws_bytes=need, agg=0, B_=B, N_=N):
        return lib.mvn_unproject_backward_deterministic(1, 0, 1, 1, None, 1, 0, 1, None, ws, ws_bytes, B_, N_, C, H,
                                                        W, 16, 16, 16, agg, 0, None)
    assert call(ws=None) == -5
    assert call(ws_bytes=need - 1) == -5
    assert call(agg=7) == -1
    assert call(B_=0) == -2
    assert call(N_=9) == -2
