"""MVN_PRECISION_FAST unprojection against the pinned C oracle (MI355X only).

The fast mode computes op.py:99-163 within the north_star tolerance instead of the
reference's rounding: reciprocal projection (one v_rcp per view), the view softmax without
its max pass, and — for bf16 maps — bf16 bilinear weights on bf16 pixel pairs (v_dot2).

Bars (written here):
  f32 maps            volume max-rel <= 1e-4 (north_star's fp32 bound; measured 2-4e-5: one ulp of
                      a reciprocal-based pixel coordinate moves a bilinear sample by ~1e-5 px x the
                      neighbouring pixels' difference)
  bf16 maps, f32 out  volume max-rel <= 2^-8; softmax 2^-7 (the bf16 weights enter the exponent: a
                      sample's error 2^-9 * M (M = the largest tap magnitude) moves each view's
                      softmax weight by up to the same relative amount, times the spread of the
                      samples over the views; measured 3.1-3.9e-3 over seeds and shapes,
                      tools/fast_bf16_error_probe.py, profiles/r21_fast_bf16_error_probe.txt)
  bf16 maps, bf16 out every value within one bf16 ulp of the f32 oracle + the f32-out bar x max|ref|
  joints              soft-argmax of the fast volume vs of the oracle volume <= 1e-4 (north_star)
  validity            voxels behind every camera (op.py:121) are exactly 0, as in the reference
"""
import numpy as np
import pytest
import torch

from conftest import max_rel
from oracle import capi

pytestmark = pytest.mark.gpu

METHODS = ("sum", "max", "softmax", "conf")
F32_TOL = 1e-4
BF16_REL = 2.0 ** -8
BF16_SOFTMAX_REL = 2.0 ** -7


def bf16_bar(method):
    """The bf16-maps bar of one aggregation (module docstring)."""
    return BF16_SOFTMAX_REL if method == "softmax" else BF16_REL


def _t(a, device, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(device)
    return t if dtype is None else t.to(dtype)


def bf16_bits(t):
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


def bf16_ulp(ref):
    _, e = np.frexp(np.asarray(ref, np.float64))
    return np.where(ref == 0, 0.0, np.ldexp(1.0, e - 8))


def assert_bf16_fast(out16, ref, method):
    got = out16.float().cpu().numpy().astype(np.float64)
    bound = bf16_ulp(ref) + bf16_bar(method) * np.abs(ref).max()
    err = np.abs(got - ref)
    assert (err <= bound).all(), float((err / np.maximum(bound, 1e-45)).max())


def _unproject(vb_feat, proj, coords, method, conf=None, **kw):
    from mvn_rocm import op
    return op.unproject_heatmaps(vb_feat, proj, coords, method, conf, precision="fast", **kw)


# ----------------------------------------------------------------------------- f32 maps
@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_fast_config_slice_golden(golden, device, method):
    """The reference's own config-shaped golden (4 views x 8 ch x 96^2 -> 16^3, f32)."""
    d = golden("unproject_cfg.npz")
    out = _unproject(_t(d["feat"], device), _t(d["proj"], device), _t(d["coords"], device), method)
    assert max_rel(out.cpu().numpy(), d[f"{method}_ac0"]) <= F32_TOL


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("ac", (False, True))
def test_fast_cfg2_f32_full_size(device, method, ac):
    """BASELINE config 2's frame (4 views x 32 ch x 96^2 -> 64^3, f32), every aggregation,
    both align_corners conventions."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, seed=5)
    conf = np.random.default_rng(5).uniform(0.05, 1.0, (1, 4, 32)).astype(np.float32)
    ref = capi.unproject(vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy(), method, conf, align_corners=int(ac))
    out = _unproject(vb.features.to(device), vb.proj.to(device), vb.coords.to(device), method, _t(conf, device),
                     align_corners=ac)
    assert max_rel(out.cpu().numpy(), ref) <= F32_TOL
    assert 0.2 < (ref != 0).mean()


@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_fast_cfg4_eight_views(device, method):
    """BASELINE config 4's frame: 8 views (2-channel slots), f32."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, n_views=8, seed=45)
    ref = capi.unproject(vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy(), method)
    out = _unproject(vb.features.to(device), vb.proj.to(device), vb.coords.to(device), method)
    assert max_rel(out.cpu().numpy(), ref) <= F32_TOL


@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_fast_eight_views_bf16(device, method):
    """8 views of bf16 maps (2-channel f32 slots: the fast projection and softmax, no pixel
    pairs) against the oracle on the same bf16 bits, at the bf16 bar."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, n_views=8, channels=8, volume=32, seed=46, dtype=torch.bfloat16)
    ref = capi.unproject(bf16_bits(vb.features), vb.proj.numpy(), vb.coords.numpy(), method, feat_bf16_bits=True)
    out = _unproject(vb.features.to(device), vb.proj.to(device), vb.coords.to(device), method,
                     out_dtype=torch.float32)
    assert max_rel(out.cpu().numpy(), ref) <= bf16_bar(method)
    assert 0.2 < (ref != 0).mean()


@pytest.mark.parametrize("n_views", (1, 3, 5))
def test_fast_falls_back_to_exact_where_it_does_not_apply(device, n_views):
    """View counts other than 4 and 8 run the exact kernels in either mode:
    precision='fast' returns the exact volume bit for bit."""
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(1, n_views=n_views, channels=8, volume=16, seed=47)
    f, P, c = vb.features.to(device), vb.proj.to(device), vb.coords.to(device)
    fast = op.unproject_heatmaps(f, P, c, "softmax", precision="fast")
    exact = op.unproject_heatmaps(f, P, c, "softmax", precision="exact")
    assert torch.equal(fast.view(torch.int32), exact.view(torch.int32))


# ----------------------------------------------------------------------------- bf16 maps (pixel pairs, v_dot2)
@pytest.mark.parametrize("method", METHODS)
def test_fast_cfg3_bf16_full_size(device, method):
    """BASELINE config 3: two of the bench's frames, bf16 maps, against the C oracle on the
    same bf16 bits (f32 arithmetic): bf16 volume and f32 volume."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(2, dtype=torch.bfloat16, device=device, seed=0)
    conf = np.random.default_rng(9).uniform(0.05, 1.0, (2, 4, 32)).astype(np.float32)
    ref = capi.unproject(bf16_bits(vb.features), vb.proj.cpu().numpy(), vb.coords.cpu().numpy(), method, conf,
                         feat_bf16_bits=True)
    out16 = _unproject(vb.features, vb.proj, vb.coords, method, _t(conf, device))
    assert out16.dtype == torch.bfloat16
    assert_bf16_fast(out16, ref, method)
    out32 = _unproject(vb.features, vb.proj, vb.coords, method, _t(conf, device), out_dtype=torch.float32)
    assert max_rel(out32.cpu().numpy(), ref) <= bf16_bar(method)
    assert 0.2 < (ref != 0).mean()


def test_fast_cfg3_joints_within_north_star(device):
    """The bench's config-3 step in fast mode: the joints of the fast volume's channels [0:17]
    against the joints of the oracle's volume (the chain end to end): <= 1e-4 (north_star)."""
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(2, dtype=torch.bfloat16, device=device, seed=3)
    vol = _unproject(vb.features, vb.proj, vb.coords, "softmax")
    xyz, _ = op.integrate_tensor_3d_with_coordinates(vol[:, :17], vb.coords)
    co = vb.coords.cpu().numpy()
    ref_vol = capi.unproject(bf16_bits(vb.features), vb.proj.cpu().numpy(), co, "softmax", feat_bf16_bits=True)
    ref_xyz, _ = capi.softargmax3d(np.ascontiguousarray(ref_vol[:, :17]), co, True, 1.0)
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-4


def test_fast_cfg2_joints_within_north_star(device):
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(2, seed=4)
    f, P, c = vb.features.to(device), vb.proj.to(device), vb.coords.to(device)
    xyz, _ = op.integrate_tensor_3d_with_coordinates(_unproject(f, P, c, "softmax")[:, :17], c)
    ref_vol = capi.unproject(vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy(), "softmax")
    ref_xyz, _ = capi.softargmax3d(np.ascontiguousarray(ref_vol[:, :17]), vb.coords.numpy(), True, 1.0)
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-4


@pytest.mark.parametrize("dtype", (torch.float32, torch.bfloat16))
@pytest.mark.parametrize("path", ("lds_1pass", "lds_multipass", "global_fallback"))
@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_fast_every_staging_path(device, dtype, path, method):
    """One LDS pass, several passes of whole views (the pixel-pair slots' overlapping chunk
    deal in its second loop) and the global-gather fallback, forced by the LDS slot budget."""
    from mvn_rocm import _lib, synth
    from test_gpu_parity import tile_footprints
    vb = synth.volumetric_batch(2, channels=12, heatmap=64, volume=32, seed=33, dtype=dtype)
    feat = bf16_bits(vb.features) if dtype == torch.bfloat16 else vb.features.numpy()
    proj, coords = vb.proj.numpy(), vb.coords.numpy()
    # the fast bf16 kernel runs an 8x8x8 tile (X4Shape<4>), the f32 one 4x8x16
    areas = tile_footprints(proj, coords, 64, 64, (8, 8, 8) if dtype == torch.bfloat16 else (4, 8, 16))
    budget = 0
    if path == "lds_multipass":
        budget = int(areas.max()) + 64
        assert (areas.sum(1) + 1 > budget).any()
    elif path == "global_fallback":
        budget = int(np.median(areas[areas > 0]))
        assert (areas.max(1) > budget - 1).any() and (areas.max(1) <= budget - 1).any()
    ref = capi.unproject(feat, proj, coords, method, feat_bf16_bits=dtype == torch.bfloat16)
    with _lib.unproject_knobs(budget):
        out = _unproject(vb.features.to(device), vb.proj.to(device), vb.coords.to(device), method,
                         out_dtype=torch.float32)
    assert max_rel(out.cpu().numpy(), ref) <= (F32_TOL if dtype == torch.float32 else bf16_bar(method))


@pytest.mark.parametrize("dtype", (torch.float32, torch.bfloat16))
@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_fast_ragged_non_cubic_volume(device, dtype, method):
    """A (13, 21, 10) coordinate volume: every axis leaves a partial tile of the fast kernels'
    8x8x8 (bf16) and 4x8x16 (f32) tiles; inactive voxels neither write nor stage."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(2, channels=8, heatmap=64, volume=24, seed=41, dtype=dtype)
    coords = vb.coords[:, :13, :21, :10].contiguous()
    feat = bf16_bits(vb.features) if dtype == torch.bfloat16 else vb.features.numpy()
    ref = capi.unproject(feat, vb.proj.numpy(), coords.numpy(), method, feat_bf16_bits=dtype == torch.bfloat16)
    out = _unproject(vb.features.to(device), vb.proj.to(device), coords.to(device), method, out_dtype=torch.float32)
    assert out.shape == (2, 8, 13, 21, 10)
    assert max_rel(out.cpu().numpy(), ref) <= (F32_TOL if dtype == torch.float32 else bf16_bar(method))
    assert 0.2 < (ref != 0).mean()


# ----------------------------------------------------------------------------- range guard, NaN, validity
@pytest.mark.parametrize("dtype", (torch.float32, torch.bfloat16))
@pytest.mark.parametrize("scale", (80.0, -80.0))
def test_fast_softmax_range_guard(device, dtype, scale):
    """Samples beyond the max-free softmax's range (|s| ~ 300: 2^(s log2 e) overflows, or
    underflows in every view) take the max-first fallback: still the reference's values."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, channels=8, volume=32, seed=12)
    feat = (vb.features * scale).to(dtype)
    bits = bf16_bits(feat) if dtype == torch.bfloat16 else feat.numpy()
    ref = capi.unproject(bits, vb.proj.numpy(), vb.coords.numpy(), "softmax", feat_bf16_bits=dtype == torch.bfloat16)
    out = _unproject(feat.to(device), vb.proj.to(device), vb.coords.to(device), "softmax", out_dtype=torch.float32)
    got = out.cpu().numpy()
    assert np.isfinite(got).all()
    assert max_rel(got, ref) <= (F32_TOL if dtype == torch.float32 else bf16_bar("softmax"))


@pytest.mark.parametrize("dtype", (torch.float32, torch.bfloat16))
def test_fast_nan_features_propagate(device, dtype):
    """NaN pixels give NaN voxels as in the reference (the zero-weight tap included): the NaN
    sets agree except where the fast projection's floor lands on the other side of a pixel
    edge (a few voxels), and the finite values meet the fast bar."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, channels=8, volume=32, seed=13)
    feat = vb.features.clone()
    feat[0, 1, 2, 40:44, 50:53] = float("nan")
    feat[0, 3, :, 10, 10] = float("nan")
    feat = feat.to(dtype)
    bits = bf16_bits(feat) if dtype == torch.bfloat16 else feat.numpy()
    ref = capi.unproject(bits, vb.proj.numpy(), vb.coords.numpy(), "softmax", feat_bf16_bits=dtype == torch.bfloat16)
    got = _unproject(feat.to(device), vb.proj.to(device), vb.coords.to(device), "softmax",
                     out_dtype=torch.float32).cpu().numpy()
    nr, ng = np.isnan(ref), np.isnan(got)
    assert nr.sum() > 50
    assert (nr != ng).sum() <= max(4, nr.sum() // 50)
    fin = ~(nr | ng)
    assert max_rel(got[fin], ref[fin]) <= (F32_TOL if dtype == torch.float32 else bf16_bar("softmax"))


@pytest.mark.parametrize("dtype", (torch.float32, torch.bfloat16))
def test_fast_validity_mask_is_the_references(device, dtype):
    """Voxels behind every camera (w <= 0, op.py:121) are exactly 0 in every channel; the
    depth test is the reference's own f32 chain in both modes."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, channels=8, volume=32, seed=14)
    coords = vb.coords
    P = vb.proj.clone()
    P[0, :, 2, :] = -P[0, :, 2, :]                    # every camera looking away: all w < 0
    feat = vb.features.to(dtype)
    bits = bf16_bits(feat) if dtype == torch.bfloat16 else feat.numpy()
    ref = capi.unproject(bits, P.numpy(), coords.numpy(), "sum", feat_bf16_bits=dtype == torch.bfloat16)
    got = _unproject(feat.to(device), P.to(device), coords.to(device), "sum", out_dtype=torch.float32).cpu().numpy()
    assert (ref == 0).all()
    assert (got == 0).all()


def test_fast_is_deterministic_and_exact_mode_unchanged(device):
    """Fast mode twice: bit-identical; the default mode is still the exact kernel."""
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(2, dtype=torch.bfloat16, device=device, seed=6)
    a = _unproject(vb.features, vb.proj, vb.coords, "softmax")
    b = _unproject(vb.features, vb.proj, vb.coords, "softmax")
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    e1 = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    e2 = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax", precision="exact")
    assert torch.equal(e1.view(torch.int16), e2.view(torch.int16))
    assert not torch.equal(a.view(torch.int16), e1.view(torch.int16))
    prev = op.set_unproject_precision("fast")
    try:
        c = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    finally:
        op.set_unproject_precision(prev)
    assert torch.equal(a.view(torch.int16), c.view(torch.int16))


def test_fast_in_kernel_coordinates(device):
    """The cuboid entry (coordinates formed in-kernel) in fast mode: the fast bar against the
    oracle on the materialised coordinate volume."""
    from mvn_rocm import synth, volumetric
    from oracle import restate_np
    vb = synth.volumetric_batch(2, dtype=torch.bfloat16, device=device, seed=7)
    base, theta = np.array([[120.0, -80.0, 900.0], [-300.0, 200.0, 950.0]]), np.array([0.7, 2.1])
    cub = volumetric.build_cuboids(base, 2500.0, 64, theta, device=device)
    co = restate_np.coord_volumes(base, 2500.0, 64, theta, "coco", False)
    ref = capi.unproject(bf16_bits(vb.features), vb.proj.cpu().numpy(), co, "softmax", feat_bf16_bits=True)
    out = _unproject(vb.features, vb.proj, cub, "softmax")
    assert_bf16_fast(out, ref, "softmax")


def test_fast_volumetric_chain_matches_reference_model(golden, device):
    """VolumetricTriangulationNet.forward as recorded from the reference (tests/golden/chains.npz:
    4 views x 32 ch x 32^2 -> 32^3, softmax, V2V stand-in = channels [0:17]) with the fast
    unprojection: volume <= 1e-4 (f32 bar), joints <= 1e-4 (north_star), both coordinate forms."""
    from mvn_rocm import op, volumetric
    d = golden("chains.npz")
    side, V = float(d["vol_side"]), d["vol_coords"].shape[1]
    cv = volumetric.build_coord_volumes(d["vol_base"], side, V, d["vol_thetas"], "mpii", False, device=device)
    cub = volumetric.build_cuboids(d["vol_base"], side, V, d["vol_thetas"], "mpii", False, device=device)
    f, P = _t(d["vol_features"], device), _t(d["vol_proj"], device)
    sub = (slice(None), slice(None), slice(None, None, 4), slice(None, None, 4), slice(None, None, 4))
    for coords in (cv, cub):
        vol = _unproject(f, P, coords, "softmax")
        assert max_rel(vol.cpu().numpy()[sub], d["vol_unprojected_sub"]) <= F32_TOL
        xyz, _ = op.integrate_tensor_3d_with_coordinates(vol[:, :17], coords, True)
        assert max_rel(xyz.cpu().numpy(), d["vol_kp3d"]) <= 1e-4


def test_fast_cfg5_channels_last_full_size(device):
    """BASELINE config 5's unprojection (bf16, channels-last, 64^3) in the fast arithmetic: the
    transpose of the fast NCDHW volume bit for bit, within the fast bar of the C oracle; the
    one-call pipeline in fast mode equals the two steps."""
    from mvn_rocm import synth, v2v
    vb = synth.volumetric_batch(1, dtype=torch.bfloat16, device=device, seed=57)
    cl = v2v.unproject_channels_last(vb.features, vb.proj, vb.coords, "softmax", precision="fast")
    nc = _unproject(vb.features, vb.proj, vb.coords, "softmax")
    assert torch.equal(cl.view(torch.int16), nc.permute(0, 2, 3, 4, 1).contiguous().view(torch.int16))
    ref = capi.unproject(bf16_bits(vb.features), vb.proj.cpu().numpy(), vb.coords.cpu().numpy(), "softmax",
                         feat_bf16_bits=True)
    assert_bf16_fast(nc, ref, "softmax")
    g = torch.Generator().manual_seed(57)
    w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
    packed, scale, shift = v2v.fold_basic3d_block(w, torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
                                                  torch.randn(16, generator=g) * 0.1, torch.zeros(16), torch.ones(16),
                                                  device=device)
    y1 = v2v.unproject_v2v_front(vb.features, vb.proj, vb.coords, packed, scale, shift, "softmax", precision="fast")
    y2 = v2v.v2v_front(cl, packed, scale, shift, torch.float32)
    assert torch.equal(y1, y2)
