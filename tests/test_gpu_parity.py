"""HIP kernels vs the oracle and the reference's golden vectors (MI355X only).

Bars (BASELINE.json north_star):
  unproject 'sum' / 'max' / 'conf' : bit-exact (same f32 op order as ATen CPU)
  unproject 'softmax'              : max-rel <= 1e-5 (exp rounding only; target 1e-4)
  soft-argmax                      : max-rel <= 1e-5 on coordinates and volumes
  DLT                              : max-rel <= 1e-6 vs the float64 restatement
  bf16                             : f32 reference on bf16-rounded features, output
                                     rounded to bf16 -> <= 1 bf16 ulp (2^-8 rel)
"""
import numpy as np
import pytest
import torch

from conftest import assert_bits_equal, max_rel
from oracle import capi, restate_np

pytestmark = pytest.mark.gpu

METHODS = ("sum", "max", "softmax", "conf")


def _op():
    from mvn_rocm import op
    return op


def _t(a, device, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(device)
    return t if dtype is None else t.to(dtype)


def bf16_to_f32(bits):
    return (np.asarray(bits, np.uint32) << 16).view(np.float32)


def assert_unproject_parity(out, ref, method, tol=1e-5):
    if method == "softmax":
        assert max_rel(out, ref) <= tol
    else:                       # bit for bit, signed zeros included
        assert_bits_equal(out, ref)


# ----------------------------------------------------------------------------- unproject
@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("ac", (0, 1))
def test_unproject_matches_reference_golden(golden, device, method, ac):
    d = golden("unproject_small.npz")
    out = _op().unproject_heatmaps(_t(d["feat"], device), _t(d["proj"], device), _t(d["coords"], device), method,
                                   _t(d["conf"], device), align_corners=bool(ac))
    assert out.dtype == torch.float32 and out.shape == (2, 5, 8, 9, 10)
    assert_unproject_parity(out.cpu().numpy(), d[f"{method}_ac{ac}"], method)


def tile_footprints(proj, coords, H, W, tile):
    """Per (frame, tile, view) LDS slots the tiled kernel stages (its bbox rule, in numpy):
    lets a test pick a budget that forces several passes / the global fallback."""
    TX, TY, TZ = tile
    B, Vx, Vy, Vz = coords.shape[:4]
    P = proj.astype(np.float64)
    X = np.concatenate([coords, np.ones(coords.shape[:4] + (1,))], -1).astype(np.float64)
    uvw = np.einsum("bvrk,bxyzk->bvxyzr", P, X)
    w = np.where(uvw[..., 2] == 0, 1.0, uvw[..., 2])
    fx = np.floor((2 * (uvw[..., 0] / w / H - 0.5) + 1) * W / 2 - 0.5)
    fy = np.floor((2 * (uvw[..., 1] / w / W - 0.5) + 1) * H / 2 - 0.5)
    ok = (fx >= -1) & (fx < W) & (fy >= -1) & (fy < H) & (uvw[..., 2] > 0)
    out = []
    for b in range(B):
        for x in range(0, Vx, TX):
            for y in range(0, Vy, TY):
                for z in range(0, Vz, TZ):
                    areas = []
                    for v in range(P.shape[1]):
                        m = ok[b, v, x:x + TX, y:y + TY, z:z + TZ]
                        a = fx[b, v, x:x + TX, y:y + TY, z:z + TZ][m]
                        c = fy[b, v, x:x + TX, y:y + TY, z:z + TZ][m]
                        areas.append(0 if a.size == 0 else int((int(a.max() - a.min() + 2) | 1) * (c.max() - c.min() + 2)))
                    out.append(areas)
    return np.array(out)


@pytest.mark.parametrize("n_views", (4, 8))
@pytest.mark.parametrize("path", ("lds_1pass", "lds_multipass", "global_fallback", "simple"))
@pytest.mark.parametrize("method", METHODS)
def test_unproject_every_kernel_path(device, path, method, n_views):
    """Each code path of the unprojection — one LDS pass, several LDS passes, the
    global-gather fallback and the simple kernel — against the oracle, for the 4- and
    8-view instantiations."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(2, n_views=n_views, channels=10, heatmap=64, volume=32, seed=31)
    feat, proj, coords = vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy()
    areas = tile_footprints(proj, coords, 64, 64, (4, 8, 16))     # TileShape<4>, <8> in unproject_tiled.hip
    budget, simple = 0, path == "simple"
    if path == "lds_multipass":        # every footprint fits alone, no tile's views fit together
        budget = int(areas.max()) + 64        # margin: the kernel rounds in f32
        assert (areas.sum(1) + 1 > budget).any()
    elif path == "global_fallback":    # some single footprints exceed the budget
        budget = int(np.median(areas[areas > 0]))
        assert (areas.max(1) > budget - 1).any() and (areas.max(1) <= budget - 1).any()
    conf = np.random.default_rng(2).uniform(0, 1, (2, n_views, 10)).astype(np.float32)
    ref = capi.unproject(feat, proj, coords, method, conf)
    from mvn_rocm import _lib
    with _lib.unproject_knobs(budget, simple):
        out = _op().unproject_heatmaps(vb.features.to(device), vb.proj.to(device), vb.coords.to(device), method,
                                       _t(conf, device))
    assert_unproject_parity(out.cpu().numpy(), ref, method)


@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_unproject_bf16_matches_reference_golden(golden, device, method):
    d = golden("unproject_small.npz")
    feat = _t(d["feat"], device).to(torch.bfloat16)
    ref = d[f"bf16in_{method}_ac0"]
    out32 = _op().unproject_heatmaps(feat, _t(d["proj"], device), _t(d["coords"], device), method,
                                     out_dtype=torch.float32)
    assert_unproject_parity(out32.cpu().numpy(), ref, method)
    out16 = _op().unproject_heatmaps(feat, _t(d["proj"], device), _t(d["coords"], device), method)
    assert out16.dtype == torch.bfloat16
    np.testing.assert_allclose(out16.float().cpu().numpy(), ref, rtol=2 ** -8, atol=2 ** -8 * np.abs(ref).max())


@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_unproject_config_slice_golden(golden, device, method):
    d = golden("unproject_cfg.npz")
    out = _op().unproject_heatmaps(_t(d["feat"], device), _t(d["proj"], device), _t(d["coords"], device), method)
    assert_unproject_parity(out.cpu().numpy(), d[f"{method}_ac0"], method)


@pytest.mark.parametrize("n_views", (1, 2, 3, 5, 8, 9, 12))
@pytest.mark.parametrize("method", METHODS)
def test_unproject_random_shapes_vs_oracle(device, n_views, method):
    from mvn_rocm import synth
    rng = np.random.default_rng(100 + n_views)
    B, C, H, W = 2, 3, 13, 19
    vb = synth.volumetric_batch(B, n_views=n_views, channels=C, heatmap=max(H, W), volume=12, seed=n_views)
    feat = rng.standard_normal((B, n_views, C, H, W)).astype(np.float32)
    proj = vb.proj.numpy()
    proj[:, :, 0] *= W / max(H, W)
    proj[:, :, 1] *= H / max(H, W)
    coords = vb.coords.numpy()[:, :12, :11, :10]          # non-cubic volume
    conf = rng.uniform(0.0, 1.0, (B, n_views, C)).astype(np.float32)
    for ac in (False, True):
        ref = capi.unproject(feat, proj, coords, method, conf, ac)
        out = _op().unproject_heatmaps(_t(feat, device), _t(proj, device), _t(coords, device), method,
                                       _t(conf, device), align_corners=ac)
        assert_unproject_parity(out.cpu().numpy(), ref, method)


@pytest.mark.parametrize("method", ("softmax", "sum"))
def test_unproject_full_config_frame_vs_oracle(device, method):
    """One frame of BASELINE config 2 (4 views x 32 ch x 96^2 -> 64^3)."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, seed=21)
    ref = capi.unproject(vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy(), method)
    out = _op().unproject_heatmaps(vb.features.to(device), vb.proj.to(device), vb.coords.to(device), method)
    assert_unproject_parity(out.cpu().numpy(), ref, method)
    assert 0.2 < (ref != 0).mean()          # the cuboid really projects into the maps


def test_unproject_full_size_properties(device):
    """Batch-32 properties the oracle cannot afford at full size: linearity of 'sum'
    in the features, view-permutation invariance, frame independence."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(32, dtype=torch.float32, device=device, seed=4)
    op = _op()
    f, P, X = vb.features, vb.proj, vb.coords
    a = op.unproject_heatmaps(f, P, X, "sum")
    b = op.unproject_heatmaps(2.0 * f, P, X, "sum")
    torch.testing.assert_close(b, 2.0 * a, rtol=0, atol=0)         # scaling by 2 is exact
    perm = torch.tensor([2, 0, 3, 1], device=device)
    s1 = op.unproject_heatmaps(f, P, X, "softmax")
    s2 = op.unproject_heatmaps(f[:, perm], P[:, perm], X, "softmax")
    assert max_rel(s2.cpu().numpy(), s1.cpu().numpy()) <= 1e-6
    one = op.unproject_heatmaps(f[7:8], P[7:8], X[7:8], "softmax")
    torch.testing.assert_close(one[0], s1[7], rtol=0, atol=0)      # frames are independent
    assert torch.isfinite(s1).all()


# ----------------------------------------------------------------------------- soft-argmax
@pytest.mark.parametrize("softmax", (True, False))
@pytest.mark.parametrize("mult", (1.0, 1.7))
def test_softargmax_matches_reference_golden(golden, device, softmax, mult):
    d = golden("softargmax_small.npz")
    key = f"sm{int(softmax)}_m{mult}"
    xyz, vol = _op().integrate_tensor_3d_with_coordinates(_t(d["vol"], device), _t(d["coords"], device),
                                                          softmax, multiplier=mult)
    assert max_rel(xyz.cpu().numpy(), d[f"xyz_{key}"]) <= 1e-5
    assert max_rel(vol.cpu().numpy(), d[f"vol_{key}"]) <= 1e-5


def test_softargmax_blob_golden(golden, device):
    d = golden("softargmax_blob.npz")
    xyz, vol = _op().integrate_tensor_3d_with_coordinates(_t(d["vol"], device), _t(d["coords"], device))
    assert max_rel(xyz.cpu().numpy(), d["xyz"]) <= 1e-5
    assert max_rel(vol.cpu().numpy(), d["vol_out"]) <= 1e-5


@pytest.mark.parametrize("softmax", (True, False))
def test_softargmax_full_size_vs_oracle(device, softmax):
    from mvn_rocm import synth
    vb = synth.volumetric_batch(2, channels=1, seed=8)
    vol = synth.blob_volumes(vb.coords, 17, seed=8)
    ref_xyz, ref_vol = capi.softargmax3d(vol.numpy(), vb.coords.numpy(), softmax, 1.0)
    xyz, out = _op().integrate_tensor_3d_with_coordinates(vol.to(device), vb.coords.to(device), softmax)
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-5
    assert max_rel(out.cpu().numpy(), ref_vol) <= 1e-5


def test_softargmax_channel_slice_and_bf16(device):
    """The bench feeds channels [0:17] of a (B, 32, V^3) unprojection without a copy."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(2, channels=1, volume=32, seed=9)
    big = torch.randn((2, 32, 32, 32, 32), generator=torch.Generator().manual_seed(3)) * 4
    sl = big.to(device)[:, :17]
    assert not sl.is_contiguous()
    ref_xyz, ref_vol = capi.softargmax3d(big[:, :17].numpy(), vb.coords.numpy(), True, 1.3)
    xyz, out = _op().integrate_tensor_3d_with_coordinates(sl, vb.coords.to(device), multiplier=1.3)
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-5
    assert max_rel(out.cpu().numpy(), ref_vol) <= 1e-5
    # bf16 volume: oracle on the bf16-rounded logits, bf16 output within 1 ulp
    sl16 = sl.to(torch.bfloat16)
    ref_xyz, ref_vol = capi.softargmax3d(sl16.float().cpu().numpy(), vb.coords.numpy(), True, 1.3)
    xyz, out = _op().integrate_tensor_3d_with_coordinates(sl16, vb.coords.to(device), multiplier=1.3)
    assert out.dtype == torch.bfloat16
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-5
    np.testing.assert_allclose(out.float().cpu().numpy(), ref_vol, rtol=2 ** -8, atol=1e-30)
    xyz2, none = _op().integrate_tensor_3d_with_coordinates(sl16, vb.coords.to(device), multiplier=1.3,
                                                            return_volumes=False)
    assert none is None
    torch.testing.assert_close(xyz2, xyz, rtol=0, atol=0)


def test_softargmax_translation_equivariance(device):
    from mvn_rocm import synth
    vb = synth.volumetric_batch(4, channels=1, device=device, seed=10)
    vol = synth.blob_volumes(vb.coords, 17, seed=10)
    shift = torch.tensor([123.5, -77.25, 10.0], device=device)
    a, _ = _op().integrate_tensor_3d_with_coordinates(vol, vb.coords)
    b, _ = _op().integrate_tensor_3d_with_coordinates(vol, vb.coords + shift)
    torch.testing.assert_close(b, a + shift, rtol=0, atol=2e-3)


@pytest.mark.parametrize("dtype", (torch.float32, torch.bfloat16))
def test_softargmax_nan_volume_follows_torch(device, dtype):
    """a joint whose volume holds NaNs — one whole 1,024-voxel pass-1 chunk (its
    max is NaN) or a single voxel (the chunk's max drops it) — comes out NaN in coordinates
    and normalised volume, as torch's softmax over the flattened volume (op.py:89) does;
    the other joints of the frame are untouched."""
    from mvn_rocm import synth
    vb = synth.volumetric_batch(1, channels=1, volume=16, seed=21)
    vol = synth.blob_volumes(vb.coords, 3, seed=21).to(dtype)
    flat = vol.view(1, 3, -1)
    flat[0, 1, 1024:2048] = float("nan")          # pass-1 chunk 1 of joint 1, all NaN
    flat[0, 2, 3000] = float("nan")               # one voxel of joint 2
    sm = torch.softmax(vol.float().view(1, 3, -1), dim=2).view_as(vol)          # op.py:89
    ref_xyz = torch.einsum("bnxyz,bxyzc->bnc", sm, vb.coords)                  # op.py:94
    xyz, out = _op().integrate_tensor_3d_with_coordinates(vol.to(device), vb.coords.to(device))
    xyz, out = xyz.cpu(), out.float().cpu()
    assert torch.isnan(ref_xyz[0, 1:]).all() and torch.isnan(sm[0, 1:]).all()
    assert torch.isnan(xyz[0, 1:]).all() and torch.isnan(out[0, 1:]).all()
    assert torch.isfinite(xyz[0, 0]).all() and torch.isfinite(out[0, 0]).all()
    assert max_rel(xyz[0, 0].numpy(), ref_xyz[0, 0].numpy()) <= 1e-5


# ----------------------------------------------------------------------------- DLT
@pytest.mark.parametrize("case", ("cfg1", "b3n3", "n8"))
@pytest.mark.parametrize("use_conf", (True, False))
def test_dlt_matches_float64_restatement(golden, device, case, use_conf):
    from mvn_rocm import multiview
    d = golden("dlt.npz")
    key = f"{case}_c{int(use_conf)}"
    conf = d[f"conf_{case}"] if use_conf else None
    out = multiview.triangulate_batch_of_points(_t(d[f"proj_{case}"], device), _t(d[f"points_{case}"], device),
                                                None if conf is None else _t(conf, device)).cpu().numpy()
    x64 = restate_np.triangulate_batch_of_points(d[f"proj_{case}"], d[f"points_{case}"], conf)
    assert max_rel(out, x64) <= 1e-6
    assert max_rel(out, d[f"out64_{key}"]) <= 2e-6
    assert max_rel(out, d[f"out_{key}"]) <= 1e-3      # the float32 reference's own SVD error


def test_dlt_many_views_and_degenerate_confidences(device):
    from mvn_rocm import multiview, synth
    ab = synth.algebraic_batch(4, n_views=31, n_joints=17, seed=5)
    conf = ab.confidences.clone()
    conf[:, 5:20] = 0.0                  # zero-confidence views contribute nothing
    out = multiview.triangulate_batch_of_points(ab.proj.to(device), ab.points.to(device), conf.to(device))
    x64 = restate_np.triangulate_batch_of_points(ab.proj.numpy(), ab.points.numpy(), conf.numpy())
    assert max_rel(out.cpu().numpy(), x64) <= 1e-6
    # noise-free points reproduce the ground truth
    ab0 = synth.algebraic_batch(2, n_views=4, n_joints=17, seed=6, noise_px=0.0)
    out = multiview.triangulate_batch_of_points(ab0.proj.to(device), ab0.points.to(device))
    assert np.abs(out.cpu().numpy() - ab0.points_3d.numpy()).max() < 0.5     # mm; f32 pixel rounding


def test_dlt_degenerate_inputs_follow_the_reference(golden, device):
    """SURVEY §5 'failure' row: degenerate DLT inputs give the reference's zeros / inf / nan
    (multiview.py:147-157) without disturbing the other joints of the batch.  Fixture: the
    reference itself on this build container's torch (tests/golden/make_golden.py
    dlt_degenerate).
      * a joint whose confidences are all zero: A = 0, the reference's SVD returns V = I,
        X = -e4 and the point is (0, 0, 0) — so must ours (bit for bit, +0);
      * cameras that do not see z (third column of every P zero): column 2 of A is exactly 0
        and e3 is an exact null vector, so X[3] = 0 and X[:3] / X[3] = (nan, nan, +-inf).  Ours
        detects the zero column and returns exactly that.  The reference's LAPACK returns the
        exact e3 for 4 of the 6 joints (their NaN / inf positions must match ours; the sign of
        the infinity is the arbitrary sign of the singular vector) and a rounding-perturbed
        vector for the other 2 (X[3] ~ 1e-7: coordinates of ~1e7 — the degenerate limit, which
        no other LAPACK need reproduce; on the GPU box's host the pattern differs again)."""
    from mvn_rocm import multiview
    d = golden("dlt_degenerate.npz")
    P, pts, conf = (torch.from_numpy(d[k]) for k in ("proj", "points", "conf"))
    ref = d["out_zero_conf"]
    out = multiview.triangulate_batch_of_points(P.to(device), pts.to(device), conf.to(device)).cpu().numpy()
    assert np.isfinite(out).all()
    assert_bits_equal(out[0, 1], ref[0, 1])
    assert_bits_equal(out[1, 2], ref[1, 2])
    keep = np.ones((2, 3), bool)
    keep[0, 1] = keep[1, 2] = False
    x64 = restate_np.triangulate_batch_of_points(P.numpy(), pts.numpy(), conf.numpy())
    assert max_rel(out[keep], x64[keep]) <= 1e-6          # the other joints are unaffected
    assert max_rel(out[keep], ref[keep]) <= 1e-3          # (the f32 reference's own SVD error)
    ref = d["out_zero_col"]
    out = multiview.triangulate_batch_of_points(torch.from_numpy(d["proj_zero_col"]).to(device),
                                                pts.to(device)).cpu().numpy()
    assert np.isnan(out[..., :2]).all() and np.isinf(out[..., 2]).all()
    exact = ~np.isfinite(ref).all(-1)                      # joints where LAPACK found e3 exactly
    assert exact.sum() == 4
    np.testing.assert_array_equal(np.isnan(out[exact]), np.isnan(ref[exact]))
    np.testing.assert_array_equal(np.isinf(out[exact]), np.isinf(ref[exact]))
    assert (np.abs(ref[~exact][:, 2]) > 1e6).all()         # the others: the degenerate limit


def test_dlt_single_point_api(device):
    from mvn_rocm import multiview, synth
    ab = synth.algebraic_batch(1, 4, 3, seed=7)
    one = multiview.triangulate_point_from_multiple_views_linear_torch(
        ab.proj[0].to(device), ab.points[0, :, 1].to(device), ab.confidences[0, :, 1].to(device))
    batch = multiview.triangulate_batch_of_points(ab.proj.to(device), ab.points.to(device), ab.confidences.to(device))
    torch.testing.assert_close(one, batch[0, 1], rtol=0, atol=0)


# ----------------------------------------------------------------------------- plumbing
def test_ops_follow_the_current_stream(device):
    from mvn_rocm import synth
    vb = synth.volumetric_batch(2, volume=16, device=device, seed=12)
    ref = _op().unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        out = _op().unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    torch.cuda.current_stream(device).wait_stream(s)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)


def test_hip_library_is_the_one_loaded():
    """The product path must run libmvn_hip.so from this tree, not a fallback."""
    from mvn_rocm import _lib
    _lib.load()
    maps = open("/proc/self/maps").read()
    assert _lib.LIB_PATH in maps


# ----------------------------------------------------------------------------- 2D soft-argmax
@pytest.mark.parametrize("softmax", (True, False))
@pytest.mark.parametrize("mult", (1.0, 1.7))
def test_softargmax2d_matches_reference_golden(golden, device, softmax, mult):
    d = golden("softargmax2d.npz")
    key = f"sm{int(softmax)}_m{mult}"
    xy, maps = _op().integrate_tensor_2d(_t(d["hm"], device), softmax, multiplier=mult)
    assert xy.shape == (2, 5, 2) and maps.shape == (2, 5, 17, 23)
    assert max_rel(xy.cpu().numpy(), d[f"xy_{key}"]) <= 1e-5
    assert max_rel(maps.cpu().numpy(), d[f"maps_{key}"]) <= 1e-5


def test_softargmax2d_cfg_slice_and_bf16(golden, device):
    d = golden("softargmax2d.npz")
    xy, _ = _op().integrate_tensor_2d(_t(d["cfg"], device), return_heatmaps=False)
    ref64, _ = restate_np.integrate_tensor_2d(d["cfg"], True)
    assert max_rel(xy.cpu().numpy(), ref64) <= 1e-5
    assert max_rel(xy.cpu().numpy(), d["cfg_xy"]) <= 5e-5     # the f32 reference is 1.2e-5 off f64
    h16 = _t(d["hm"], device).to(torch.bfloat16)
    ref_xy, ref_maps = restate_np.integrate_tensor_2d(h16.float().cpu().numpy() * 1.7, True)
    xy, maps = _op().integrate_tensor_2d(h16, multiplier=1.7)
    assert maps.dtype == torch.bfloat16
    assert max_rel(xy.cpu().numpy(), ref_xy) <= 1e-5
    np.testing.assert_allclose(maps.float().cpu().numpy(), ref_maps, rtol=2 ** -8, atol=1e-30)


# ----------------------------------------------------------------------------- coordinate volumes
@pytest.mark.parametrize("case", ("coco_eval", "coco_train", "mpii_cmu"))
def test_coord_volumes_match_reference_golden(golden, device, case):
    from mvn_rocm import volumetric
    d = golden("coord_volumes.npz")
    kind = "coco" if case.startswith("coco") else "mpii"
    cv = volumetric.build_coord_volumes(d["base"], 2500.0, 16, d[f"theta_{case}"], kind, case == "mpii_cmu",
                                        device=device)
    np.testing.assert_array_equal(cv.cpu().numpy(), d[f"cv_{case}"])


def test_coord_volumes_full_size_vs_restatement(device):
    from mvn_rocm import volumetric
    rng = np.random.default_rng(5)
    base = rng.uniform(-500, 500, (2, 3)) + np.array([0, 0, 900.0])
    thetas = rng.uniform(0, 2 * np.pi, 2)
    ref = restate_np.coord_volumes(base, 2500.0, 64, thetas, "coco", False)   # pinned by the goldens
    cv = volumetric.build_coord_volumes(base, 2500.0, 64, thetas, "coco", False, device=device)
    np.testing.assert_array_equal(cv.cpu().numpy(), ref)


# ----------------------------------------------------------------------------- VolumetricCELoss
def test_nearest_voxel_and_ce_loss_match_reference(golden, device):
    from mvn_rocm import loss as mloss
    d = golden("ce_loss.npz")
    idx = mloss.nearest_voxel(_t(d["coords"], device), _t(d["kps"], device))
    np.testing.assert_array_equal(idx.cpu().numpy(), restate_np.nearest_voxel(d["coords"], d["kps"]))
    vol = _t(d["vol"], device).requires_grad_(True)
    loss = mloss.VolumetricCELoss()(_t(d["coords"], device), vol, _t(d["kps"], device), _t(d["validity"], device))
    loss.backward()
    assert abs(float(loss) - float(d["loss"])) <= 1e-6 * abs(float(d["loss"]))
    assert max_rel(vol.grad.cpu().numpy(), d["grad_vol"]) <= 1e-6


def test_nearest_voxel_full_size(device):
    from mvn_rocm import loss as mloss, synth
    vb = synth.volumetric_batch(2, channels=1, seed=4)
    rng = np.random.default_rng(4)
    kps = (rng.uniform(-1200, 1200, (2, 17, 3)) + np.array([0, 0, 900.0])).astype(np.float32)
    idx = mloss.nearest_voxel(vb.coords.to(device), _t(kps, device))
    np.testing.assert_array_equal(idx.cpu().numpy(), restate_np.nearest_voxel(vb.coords.numpy(), kps))


# ----------------------------------------------------------------------------- V2V front block (config 5)
def test_v2v_front_matches_reference_golden(golden, device):
    from mvn_rocm import v2v
    d = golden("v2v_front.npz")
    t = {k: torch.from_numpy(np.asarray(d[k])) for k in ("weight", "bias", "bn_weight", "bn_bias", "bn_mean", "bn_var")}
    blk = v2v.Basic3DBlockFront(*v2v.fold_basic3d_block(t["weight"], t["bias"], t["bn_weight"], t["bn_bias"],
                                                         t["bn_mean"], t["bn_var"], float(d["eps"]), device=device))
    x_cl = _t(d["x"], device).permute(0, 2, 3, 4, 1).contiguous().to(torch.bfloat16)
    y = blk(x_cl)
    assert y.shape == (2, 16, 16, 16, 16)
    assert max_rel(y.cpu().numpy(), d["y"]) <= 1e-4          # bf16 operands, f32 accumulation order only
    y16 = blk(x_cl, out_dtype=torch.bfloat16)
    np.testing.assert_allclose(y16.float().cpu().numpy(), d["y"], rtol=2 ** -7, atol=2 ** -7 * np.abs(d["y"]).max())


def test_unproject_channels_last_is_a_transpose(device):
    from mvn_rocm import synth, v2v
    vb = synth.volumetric_batch(2, channels=32, volume=32, dtype=torch.bfloat16, device=device, seed=12)
    ref = _op().unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    cl = v2v.unproject_channels_last(vb.features, vb.proj, vb.coords, "softmax")
    torch.testing.assert_close(cl, ref.permute(0, 2, 3, 4, 1), rtol=0, atol=0)
    ref32 = _op().unproject_heatmaps(vb.features, vb.proj, vb.coords, "sum", out_dtype=torch.float32)
    cl32 = v2v.unproject_channels_last(vb.features, vb.proj, vb.coords, "sum", out_dtype=torch.float32)
    torch.testing.assert_close(cl32, ref32.permute(0, 2, 3, 4, 1), rtol=0, atol=0)


def test_v2v_front_full_size_vs_torch_cpu(device):
    import torch.nn.functional as F
    from mvn_rocm import v2v
    g = torch.Generator().manual_seed(5)
    w = (torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02).bfloat16().float()
    b, gam, bet = torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5, torch.randn(16, generator=g)
    mean, var = torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5
    x = torch.randn((1, 32, 32, 32, 32), generator=g).bfloat16().float()
    packed, scale, shift = v2v.fold_basic3d_block(w, b, gam, bet, mean, var, 1e-5, device=device)
    y = v2v.v2v_front(x.permute(0, 2, 3, 4, 1).contiguous().to(device).to(torch.bfloat16), packed, scale, shift)
    ref = torch.relu(F.conv3d(x, w, None, padding=3) * scale.cpu().view(1, -1, 1, 1, 1)
                     + shift.cpu().view(1, -1, 1, 1, 1))
    assert max_rel(y.cpu().numpy(), ref.numpy()) <= 1e-4


@pytest.mark.parametrize("softmax", (True, False))
@pytest.mark.parametrize("hw", ((96, 96), (20, 24), (37, 12), (112, 108)))
def test_softargmax2d_register_path_vs_restatement(device, softmax, hw):
    """The register-resident 2D soft-argmax (maps <= 12,288 pixels with W % 4 == 0, csrc/
    softargmax2d.hip softargmax2d_reg): coordinates and returned maps against the float64
    restatement of op.py:11-47, f32 and bf16, a last run of 4 pixels partly past the map
    (37 x 12 = 444 pixels) and the largest map it takes (112 x 108 = 12,096)."""
    H, W = hw
    hm = torch.randn((3, 17, H, W), generator=torch.Generator().manual_seed(H * W)) * 3
    for dt in (torch.float32, torch.bfloat16):
        x = hm.to(dt)
        ref_xy, ref_maps = restate_np.integrate_tensor_2d(x.float().numpy() * 1.3, softmax)
        xy, maps = _op().integrate_tensor_2d(x.to(device), softmax, multiplier=1.3)
        assert max_rel(xy.cpu().numpy(), ref_xy) <= 1e-5
        if dt == torch.float32:
            assert max_rel(maps.cpu().numpy(), ref_maps) <= 1e-5
        else:
            np.testing.assert_allclose(maps.float().cpu().numpy(), ref_maps, rtol=2 ** -8, atol=1e-30)
