"""Parity at the BASELINE.json configs' own sizes (MI355X only), the caller chains of the two
models, the nearest-voxel tie rule and C-ABI reentrancy.

Bars as in test_gpu_parity.py: 'sum' / 'max' / 'conf' bit-exact, 'softmax' <= 1e-5, bf16
output within one bf16 ulp of the f32 oracle on the same bf16 inputs, soft-argmax <= 1e-5,
V2V front <= 1e-4 (bf16 operands, f32 accumulation order).
"""
import threading

import numpy as np
import pytest
import torch

from conftest import assert_bits_equal, max_rel
from oracle import capi, restate_np

pytestmark = pytest.mark.gpu

METHODS = ("sum", "max", "softmax", "conf")


def _t(a, device, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(device)
    return t if dtype is None else t.to(dtype)


def bf16_ulp(ref):
    """Spacing of bf16 numbers at |ref| (8 significant bits): 2^(e - 8) for ref = m 2^e,
    m in [0.5, 1); 0 for ref == 0."""
    _, e = np.frexp(np.asarray(ref, np.float64))
    return np.where(ref == 0, 0.0, np.ldexp(1.0, e - 8))


def assert_within_one_bf16_ulp(out_bf16, ref, atol=0.0):
    """|out - ref| <= one bf16 ulp of ref (+ atol: the f32 tolerance of an aggregation that
    is not bit-exact, e.g. softmax's max-rel 1e-5, where a sum can cancel to ~0)."""
    got = out_bf16.float().cpu().numpy().astype(np.float64)
    err = np.abs(got - ref)
    bound = bf16_ulp(ref) + atol
    assert (err <= bound).all(), float((err / np.maximum(bound, 1e-45)).max())


def bf16_bits(t):
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


# ----------------------------------------------------------------------------- config 3 (bf16, 64^3)
@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_cfg3_bf16_unproject_full_size_vs_oracle(device, method):
    """BASELINE config 3: 4 views x 32 ch x 96^2 bf16 maps -> 64^3, two frames of the bench's
    inputs, against the C oracle on the same bf16 bits (f32 arithmetic)."""
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(2, dtype=torch.bfloat16, device=device, seed=0)
    ref = capi.unproject(bf16_bits(vb.features), vb.proj.cpu().numpy(), vb.coords.cpu().numpy(), method,
                         feat_bf16_bits=True)
    out32 = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, method, out_dtype=torch.float32)
    if method == "softmax":
        assert max_rel(out32.cpu().numpy(), ref) <= 1e-5
    else:
        assert_bits_equal(out32.cpu().numpy(), ref)
    out16 = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, method)
    assert out16.dtype == torch.bfloat16
    assert_within_one_bf16_ulp(out16, ref, 1e-5 * np.abs(ref).max() if method == "softmax" else 0.0)
    assert 0.2 < (ref != 0).mean()


def test_cfg3_bf16_path_unproject_then_softargmax(device):
    """The bench's config-3 step: bf16 unprojection (softmax), soft-argmax over its channels
    [0:17] (strided slice, no copy) with bf16 volumes out, against the oracle on the bf16
    volume the kernel wrote."""
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(2, dtype=torch.bfloat16, device=device, seed=3)
    vol = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    sl = vol[:, :17]
    ref_xyz, ref_vol = capi.softargmax3d(sl.float().cpu().numpy(), vb.coords.cpu().numpy(), True, 1.0)
    xyz, out = op.integrate_tensor_3d_with_coordinates(sl, vb.coords)
    assert out.dtype == torch.bfloat16
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-5
    assert_within_one_bf16_ulp(out, ref_vol, 1e-30)


@pytest.mark.parametrize("softmax", (True, False))
def test_cfg3_bf16_softargmax_full_size(device, softmax):
    """Soft-argmax of bf16 64^3 blob volumes (17 joints, two frames), multiplier fused."""
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(2, channels=1, seed=8)
    vol16 = synth.blob_volumes(vb.coords, 17, seed=8).to(torch.bfloat16)
    ref_xyz, ref_vol = capi.softargmax3d(vol16.float().numpy(), vb.coords.numpy(), softmax, 1.3)
    xyz, out = op.integrate_tensor_3d_with_coordinates(vol16.to(device), vb.coords.to(device), softmax,
                                                       multiplier=1.3)
    assert out.dtype == torch.bfloat16
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-5
    assert_within_one_bf16_ulp(out, ref_vol, 1e-30)


# ----------------------------------------------------------------------------- config 4 (8 views, 64^3)
@pytest.mark.parametrize("method", METHODS)
def test_cfg4_eight_views_full_size_vs_oracle(device, method):
    """BASELINE config 4's frame: 8 views x 32 ch x 96^2 -> 64^3 (f32), every aggregation,
    against the C oracle; plus the in-kernel-coordinate path (bit-identical)."""
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(1, n_views=8, seed=44)
    conf = np.random.default_rng(44).uniform(0.05, 1.0, (1, 8, 32)).astype(np.float32)
    ref = capi.unproject(vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy(), method, conf)
    f, P = vb.features.to(device), vb.proj.to(device)
    out = op.unproject_heatmaps(f, P, vb.coords.to(device), method, _t(conf, device))
    if method == "softmax":
        assert max_rel(out.cpu().numpy(), ref) <= 1e-5
    else:
        assert_bits_equal(out.cpu().numpy(), ref)
    assert 0.2 < (ref != 0).mean()


# ----------------------------------------------------------------------------- config 5 (V2V front, 64^3)
def test_cfg5_pipeline_full_size(device):
    """BASELINE config 5 at V = 64: the channels-last bf16 unprojection (softmax) is the
    transpose of the NCDHW one, and the V2V front block on it matches torch's CPU conv3d
    (same bf16 operands, f32 math) + folded BatchNorm + ReLU to 1e-4."""
    import torch.nn.functional as F
    from mvn_rocm import op, synth, v2v
    vb = synth.volumetric_batch(1, dtype=torch.bfloat16, device=device, seed=55)
    cl = v2v.unproject_channels_last(vb.features, vb.proj, vb.coords, "softmax")
    ref_cl = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    assert torch.equal(cl, ref_cl.permute(0, 2, 3, 4, 1).contiguous())
    g = torch.Generator().manual_seed(55)
    w = (torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02).bfloat16().float()
    b, gam, bet = torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5, torch.randn(16, generator=g)
    mean, var = torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5
    packed, scale, shift = v2v.fold_basic3d_block(w, b, gam, bet, mean, var, 1e-5, device=device)
    y = v2v.v2v_front(cl, packed, scale, shift)
    x = ref_cl.float().cpu()
    ref = torch.relu(F.conv3d(x, w, None, padding=3) * scale.cpu().view(1, -1, 1, 1, 1)
                     + shift.cpu().view(1, -1, 1, 1, 1))
    assert y.shape == (1, 16, 64, 64, 64)
    assert max_rel(y.cpu().numpy(), ref.numpy()) <= 1e-4
    y16 = v2v.v2v_front(cl, packed, scale, shift, torch.bfloat16)
    assert_within_one_bf16_ulp(y16, y.cpu().numpy().astype(np.float64), 1e-30)


@pytest.mark.parametrize("coords_kind", ("volume", "cuboids"))
def test_cfg5_one_call_pipeline_equals_two_steps(device, coords_kind):
    """mvn_unproject_v2v_front (frame groups through a one-group workspace) at V = 64 with a
    ragged last group (3 frames in groups of 2) and the default grouping: bit-identical to
    unproject_channels_last + v2v_front on the whole batch, f32 and bf16 outputs."""
    from mvn_rocm import synth, v2v, volumetric
    vb = synth.volumetric_batch(3, dtype=torch.bfloat16, device=device, seed=56)
    coords = vb.coords
    if coords_kind == "cuboids":
        rng = np.random.default_rng(56)
        base = rng.uniform(-500, 500, (3, 3)) + np.array([0, 0, 900.0])
        coords = volumetric.build_cuboids(base, 2500.0, 64, rng.uniform(0, 2 * np.pi, 3), "coco", False, device=device)
    g = torch.Generator().manual_seed(56)
    w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
    packed, scale, shift = v2v.fold_basic3d_block(w, torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
                                                  torch.randn(16, generator=g) * 0.1, torch.zeros(16), torch.ones(16),
                                                  device=device)
    cl = v2v.unproject_channels_last(vb.features, vb.proj, coords, "softmax")
    for od in (torch.float32, torch.bfloat16):
        ref = v2v.v2v_front(cl, packed, scale, shift, od)
        for gf in (2, 0):
            got = v2v.unproject_v2v_front(vb.features, vb.proj, coords, packed, scale, shift, "softmax", od, gf)
            assert torch.equal(got, ref), (od, gf)


@pytest.mark.parametrize("coords_kind", ("volume", "cuboids"))
def test_cfg5_conf_aggregation_channels_last_and_one_call(device, coords_kind):
    """'conf*' aggregation (op.py:147-148; the volumetric model with a conf-prefixed
    volume_aggregation_method, triangulation.py:268-269, 349) on the config-5 paths at V = 64:
    the channels-last bf16 volume is the bf16 rounding of the C oracle's bit-exact f32 volume,
    bit for bit, and the one-call pipeline (ragged groups, default groups) equals the two
    calls bit for bit."""
    from mvn_rocm import synth, v2v, volumetric
    vb = synth.volumetric_batch(3, dtype=torch.bfloat16, device=device, seed=57)
    conf = np.random.default_rng(57).uniform(0.05, 1.0, (3, 4, 32)).astype(np.float32)
    conf_d = _t(conf, device)
    coords, coords_np = vb.coords, vb.coords.cpu().numpy()
    if coords_kind == "cuboids":
        rng = np.random.default_rng(57)
        base = rng.uniform(-500, 500, (3, 3)) + np.array([0, 0, 900.0])
        coords = volumetric.build_cuboids(base, 2500.0, 64, rng.uniform(0, 2 * np.pi, 3), "coco", False, device=device)
        coords_np = coords.coord_volumes().cpu().numpy()
    cl = v2v.unproject_channels_last(vb.features, vb.proj, coords, "conf_norm", vol_confidences=conf_d)
    feat32 = vb.features.float().cpu().numpy()
    for f in range(3):
        ref = capi.unproject(feat32[f:f + 1], vb.proj[f:f + 1].cpu().numpy(), coords_np[f:f + 1], "conf",
                             conf[f:f + 1])
        ref_cl = torch.from_numpy(ref).permute(0, 2, 3, 4, 1).contiguous().bfloat16()
        assert np.array_equal(bf16_bits(cl[f:f + 1]), bf16_bits(ref_cl)), f
    g = torch.Generator().manual_seed(57)
    w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
    packed, scale, shift = v2v.fold_basic3d_block(w, torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
                                                  torch.randn(16, generator=g) * 0.1, torch.zeros(16), torch.ones(16),
                                                  device=device)
    ref = v2v.v2v_front(cl, packed, scale, shift, torch.float32)
    for gf in (2, 0):
        got = v2v.unproject_v2v_front(vb.features, vb.proj, coords, packed, scale, shift, "conf", torch.float32, gf,
                                      vol_confidences=conf_d)
        assert torch.equal(got, ref), gf


def test_v2v_front_two_frames_64(device):
    """Two frames at V = 64 (the x-column walk over 16 tiles, both frames' halos)."""
    import torch.nn.functional as F
    from mvn_rocm import v2v
    g = torch.Generator().manual_seed(56)
    w = (torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02).bfloat16().float()
    packed, scale, shift = v2v.fold_basic3d_block(w, None, torch.ones(16), torch.zeros(16), torch.zeros(16),
                                                  torch.ones(16), 0.0, device=device)
    x = torch.randn((2, 32, 64, 64, 64), generator=g).bfloat16().float()
    y = v2v.v2v_front(x.permute(0, 2, 3, 4, 1).contiguous().to(device).to(torch.bfloat16), packed, scale, shift)
    ref = torch.relu(F.conv3d(x, w, None, padding=3))
    assert max_rel(y.cpu().numpy(), ref.numpy()) <= 1e-4


@pytest.mark.parametrize("cfg", ("cfg2", "cfg4"))
def test_frames_are_independent_of_the_batch(device, cfg):
    """What the multi-GPU bench's gather check (bench.verify_gather) relies on: a frame's
    unprojection and soft-argmax do not depend on the batch it is launched in.  The first and
    the last frame of a config-2 (8 frames, 4 views, f32) / config-4-shaped (4 frames, 8
    views) batch equal, bit for bit, the same frames launched alone (batch 1)."""
    from mvn_rocm import op, synth
    B, NV = (8, 4) if cfg == "cfg2" else (4, 8)
    vb = synth.volumetric_batch(B, n_views=NV, device=device, seed=58)
    vol = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
    xyz, sm = op.integrate_tensor_3d_with_coordinates(vol[:, :17], vb.coords, True)
    for f in (0, B - 1):
        v1 = op.unproject_heatmaps(vb.features[f:f + 1], vb.proj[f:f + 1], vb.coords[f:f + 1], "softmax")
        x1, s1 = op.integrate_tensor_3d_with_coordinates(v1[:, :17], vb.coords[f:f + 1], True)
        assert torch.equal(v1, vol[f:f + 1]), f
        assert torch.equal(x1, xyz[f:f + 1]), f
        assert torch.equal(s1, sm[f:f + 1]), f


# ----------------------------------------------------------------------------- caller chains
def test_volumetric_chain_matches_reference_model(golden, device):
    """VolumetricTriangulationNet.forward (triangulation.py:245-355) as recorded from the
    reference (tests/golden/chains.npz): coordinate volumes from the base points and seeded
    rotations ('mpii'), unprojection (softmax), V2V stand-in = channels [0:17], soft-argmax
    with volume_multiplier — run as the mvn_rocm ops in the same sequence, with the
    coordinate volume materialised and formed in-kernel."""
    from mvn_rocm import op, volumetric
    d = golden("chains.npz")
    side, V = float(d["vol_side"]), d["vol_coords"].shape[1]
    cv = volumetric.build_coord_volumes(d["vol_base"], side, V, d["vol_thetas"], "mpii", False, device=device)
    np.testing.assert_array_equal(cv.cpu().numpy(), d["vol_coords"])
    f, P = _t(d["vol_features"], device), _t(d["vol_proj"], device)
    sub = (slice(None), slice(None), slice(None, None, 4), slice(None, None, 4), slice(None, None, 4))
    cub = volumetric.build_cuboids(d["vol_base"], side, V, d["vol_thetas"], "mpii", False, device=device)
    results = []
    for coords in (cv, cub):
        vol = op.unproject_heatmaps(f, P, coords, "softmax")
        assert max_rel(vol.cpu().numpy()[sub], d["vol_unprojected_sub"]) <= 1e-5
        xyz, sm = op.integrate_tensor_3d_with_coordinates(vol[:, :17] * 1.0, coords, True)
        assert max_rel(xyz.cpu().numpy(), d["vol_kp3d"]) <= 1e-4
        assert max_rel(sm.cpu().numpy()[sub], d["vol_volumes_sub"]) <= 1e-5
        results.append(xyz)
    torch.testing.assert_close(results[0], results[1], rtol=0, atol=0)


def test_algebraic_chain_matches_reference_model(golden, device):
    """AlgebraicTriangulationNet.forward (triangulation.py:149-200) as recorded from the
    reference: 2D soft-argmax of heatmaps * 100, confidence normalisation (+1e-5), upscale
    to image pixels, DLT.  Joints vs the reference chain re-run in float64 <= 1e-4 (the
    float32 reference's own SVD error is up to ~2e-4)."""
    from mvn_rocm import multiview, op
    d = golden("chains.npz")
    B, N, J, H, W = d["alg_heatmaps"].shape
    hm = _t(d["alg_heatmaps"].astype(np.float32), device).reshape(B * N, J, H, W)
    xy, _ = op.integrate_tensor_2d(hm, True, multiplier=float(d["alg_multiplier"]), return_heatmaps=False)
    xy = xy.reshape(B, N, J, 2)
    assert max_rel(xy.cpu().numpy() * 4.0, d["alg_kp2d64"]) <= 1e-5
    conf = _t(d["alg_conf"], device)
    conf = conf / conf.sum(dim=1, keepdim=True) + 1e-5
    kp2 = torch.stack([xy[..., 0] * (384 / W), xy[..., 1] * (384 / H)], dim=-1)
    X = multiview.triangulate_batch_of_points(_t(d["alg_proj"], device), kp2, conf)
    assert max_rel(X.cpu().numpy(), d["alg_kp3d64"]) <= 1e-4
    assert max_rel(X.cpu().numpy(), d["alg_kp3d"]) <= 1e-3


# ----------------------------------------------------------------------------- VolumetricCELoss tie rule
def _sqrt_tie_pair():
    """Two voxel offsets (1000, 0, za) and (1000, 0, zb) from the keypoint whose f32 squared
    distances ((x^2 + y^2) + z^2, loss.py:63) differ, da > db, but whose f32 roots are equal."""
    f = np.float32

    def d2(z):
        return f(f(f(1000.0) * f(1000.0) + f(0.0)) + f(f(z) * f(z)))

    zs = [f(0.05 * i) for i in range(1, 200)]
    for za in zs:
        for zb in zs:
            da, db = d2(za), d2(zb)
            if da > db and np.sqrt(da) == np.sqrt(db):
                return za, zb
    raise AssertionError("no tie found")


def test_nearest_voxel_sqrt_tie_takes_first_index(device):
    """loss.py:63-66 takes argmin of sqrt(sum d^2): two squared distances that round to one
    root tie, and torch.argmin returns the FIRST index.  Voxel 0 is farther (larger d^2) but
    ties at the root with voxel 5, which a squared-distance argmin would pick instead."""
    from mvn_rocm import loss as mloss
    za, zb = _sqrt_tie_pair()
    coords = np.full((1, 2, 2, 2, 3), 1e5, np.float32)
    coords.reshape(-1, 3)[0] = (1000.0, 0, za)
    coords.reshape(-1, 3)[5] = (1000.0, 0, zb)
    kps = np.zeros((1, 1, 3), np.float32)
    ref = restate_np.nearest_voxel(coords, kps)
    assert ref[0, 0] == 0
    idx = mloss.nearest_voxel(_t(coords, device), _t(kps, device))
    assert int(idx[0, 0]) == 0


def test_nearest_voxel_nan_distance_wins_like_argmin(device):
    """torch.argmin (loss.py:66) treats NaN as the minimum and returns the FIRST NaN's index:
    a NaN voxel coordinate (or keypoint) beats every finite distance."""
    from mvn_rocm import loss as mloss
    rng = np.random.default_rng(80)
    coords = rng.uniform(-100, 100, (2, 4, 4, 4, 3)).astype(np.float32)
    coords.reshape(2, -1, 3)[0, 37, 1] = np.nan
    coords.reshape(2, -1, 3)[0, 50, 0] = np.nan
    kps = rng.uniform(-100, 100, (2, 3, 3)).astype(np.float32)
    kps[1, 2, 2] = np.nan                                    # every distance of this joint NaN
    ref = restate_np.nearest_voxel(coords, kps)
    assert (ref[0] == 37).all() and ref[1, 2] == 0
    idx = mloss.nearest_voxel(_t(coords, device), _t(kps, device))
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)


# ----------------------------------------------------------------------------- C ABI reentrancy
def test_c_abi_two_threads_two_streams(device):
    """§8b Threading: the C entry points are reentrant — two host threads launching on two
    streams at once give the same bits as serial calls."""
    from mvn_rocm import op, synth
    vb = [synth.volumetric_batch(2, volume=32, device=device, seed=s) for s in (60, 61)]
    serial = [op.unproject_heatmaps(v.features, v.proj, v.coords, "softmax") for v in vb]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device) for _ in vb]
    results, errors = [None, None], []

    def worker(i):
        try:
            with torch.cuda.stream(streams[i]):
                outs = [op.unproject_heatmaps(vb[i].features, vb[i].proj, vb[i].coords, "softmax") for _ in range(8)]
                xyz = [op.integrate_tensor_3d_with_coordinates(o[:, :17], vb[i].coords)[0] for o in outs]
            streams[i].synchronize()
            results[i] = (outs, xyz)
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    for i in range(2):
        ref_xyz, _ = op.integrate_tensor_3d_with_coordinates(serial[i][:, :17], vb[i].coords)
        for o, x in zip(*results[i]):
            assert torch.equal(o, serial[i])
            assert torch.equal(x, ref_xyz)


# ----------------------------------------------------------------------------- empty batches
def test_empty_batch_matches_reference_behaviour(device):
    """B = 0 as the reference handles it: unproject_heatmaps returns the empty (0, C, V^3)
    volume (op.py:104-107, the batch loop never runs) and triangulate_batch_of_points the
    empty (0, J, 3) points (multiview.py:164-174); the soft-argmaxes raise RuntimeError like the
    reference's reshape(..., -1) of an empty tensor (op.py:16, :87)."""
    from mvn_rocm import multiview, op, synth
    vb = synth.volumetric_batch(1, channels=8, volume=16, seed=3)
    feat = vb.features[:0].to(device)
    P = vb.proj[:0].to(device)
    coords = vb.coords[:0].to(device)
    for method in ("sum", "softmax"):
        out = op.unproject_heatmaps(feat, P, coords, method)
        assert out.shape == (0, 8, 16, 16, 16) and out.dtype == torch.float32
    # backward through the empty batch: the reference's autograd returns zero-sized gradients
    feat_g = feat.clone().requires_grad_(True)
    op.unproject_heatmaps(feat_g, P, coords, "softmax").sum().backward()
    assert feat_g.grad is not None and feat_g.grad.shape == feat.shape
    from mvn_rocm import volumetric
    cub = volumetric.build_cuboids(np.zeros((0, 3)), 2500.0, 16, device=device)
    feat_c = feat.clone().requires_grad_(True)
    out = op.unproject_heatmaps(feat_c, P, cub, "sum")
    assert out.shape == (0, 8, 16, 16, 16)
    out.sum().backward()
    assert feat_c.grad.shape == feat.shape
    ab = synth.algebraic_batch(1, 4, 17, seed=0)
    X = multiview.triangulate_batch_of_points(ab.proj[:0].to(device), ab.points[:0].to(device),
                                              ab.confidences[:0].to(device))
    assert X.shape == (0, 17, 3)
    pts_g = ab.points[:0].to(device).requires_grad_(True)
    conf_g = ab.confidences[:0].to(device).requires_grad_(True)
    X = multiview.triangulate_batch_of_points(ab.proj[:0].to(device), pts_g, conf_g)
    X.sum().backward()
    assert pts_g.grad.shape == pts_g.shape and conf_g.grad.shape == conf_g.shape
    with pytest.raises(RuntimeError):
        op.integrate_tensor_3d_with_coordinates(torch.zeros((0, 17, 16, 16, 16), device=device), coords)
    with pytest.raises(RuntimeError):
        op.integrate_tensor_2d(torch.zeros((0, 17, 8, 8), device=device))


@pytest.mark.gpu
def test_channels_last_entry_points_empty_batch_and_many_views(device):
    """The channels-last entry points handle what unproject_heatmaps handles: an empty batch
    returns the empty volume without a launch, and more than 8 views (beyond the channels-last
    kernels, mvn_hip.h) go through the NCDHW unprojection and a device permute — bit-identical
    to it (sum) — and, for the one-call pipeline, through the two steps."""
    from mvn_rocm import op, synth, v2v
    vb = synth.volumetric_batch(1, n_views=10, channels=32, heatmap=24, volume=16, seed=5)
    feat, P, coords = (t.to(device) for t in (vb.features, vb.proj, vb.coords))
    cl = v2v.unproject_channels_last(feat, P, coords, "sum", out_dtype=torch.float32)
    ref = op.unproject_heatmaps(feat, P, coords, "sum")
    assert torch.equal(cl, ref.permute(0, 2, 3, 4, 1))
    # bf16 maps into an f32 channels-last volume at 10 views: written in f32 by the kernel
    # (no bf16 round trip), bit-identical to the NCDHW f32 volume of the same bf16 maps
    fb = feat.to(torch.bfloat16)
    cl32 = v2v.unproject_channels_last(fb, P, coords, "softmax", out_dtype=torch.float32)
    ref32 = op.unproject_heatmaps(fb, P, coords, "softmax", out_dtype=torch.float32)
    assert cl32.dtype == torch.float32 and torch.equal(cl32, ref32.permute(0, 2, 3, 4, 1))
    empty = v2v.unproject_channels_last(feat[:0], P[:0], coords[:0], "softmax")
    assert empty.shape == (0, 16, 16, 16, 32) and empty.dtype == torch.bfloat16
    g = torch.Generator().manual_seed(0)
    packed, scale, shift = v2v.fold_basic3d_block(torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02,
                                                  torch.zeros(16), torch.ones(16), torch.zeros(16), torch.zeros(16),
                                                  torch.ones(16), device=device)
    y0 = v2v.unproject_v2v_front(feat[:0], P[:0], coords[:0], packed, scale, shift)
    assert y0.shape == (0, 16, 16, 16, 16)
    y = v2v.unproject_v2v_front(feat, P, coords, packed, scale, shift)
    two = v2v.v2v_front(v2v.unproject_channels_last(feat, P, coords, "softmax"), packed, scale, shift)
    assert torch.equal(y, two)


def test_device_assertions_count_and_clear(device):
    """The debug build's device-side assertions (csrc/common.hpp MVN_DASSERT) count failures
    without trapping and report the failing line; the release build compiles them away.
    Run with MVN_HIP_LIB=.../libmvn_hip_debug.so for the debug half."""
    from mvn_rocm import _lib
    lib = _lib.load()
    enabled, count, _ = _lib.device_asserts()          # clear anything earlier
    assert count == 0
    _lib.check(lib.mvn_debug_dassert_selftest(40, torch.cuda.current_stream().cuda_stream), "selftest")
    enabled, count, line = _lib.device_asserts()
    if enabled:
        assert count == 24 and line > 0
        assert _lib.device_asserts()[1] == 0            # read-and-clear
    else:
        assert (count, line) == (0, 0)
