"""The oracle itself, pinned against vectors captured from the reference (CPU only)."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, assert_bits_equal, assert_parity_with_nans, max_rel
from oracle import capi, restate_np, restate_torch

METHODS = ("sum", "max", "softmax", "conf")


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("ac", (0, 1))
def test_c_oracle_unproject_small(golden, method, ac):
    d = golden("unproject_small.npz")
    ref = d[f"{method}_ac{ac}"]
    out = capi.unproject(d["feat"], d["proj"], d["coords"], method, d["conf"], bool(ac))
    if method == "softmax":     # expf rounding differs from ATen's vectorised exp
        assert max_rel(out, ref) <= 1e-6
    else:                       # bit-exact recipe, signed zeros included
        assert_bits_equal(out, ref)


@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_c_oracle_unproject_bf16_input(golden, method):
    d = golden("unproject_small.npz")
    out = capi.unproject(d["feat_bf16_bits"], d["proj"], d["coords"], method, None, False, feat_bf16_bits=True)
    ref = d[f"bf16in_{method}_ac0"]
    if method == "sum":
        assert_bits_equal(out, ref)
    else:
        assert max_rel(out, ref) <= 1e-6


@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_c_oracle_unproject_cfg_slice(golden, method):
    d = golden("unproject_cfg.npz")
    out = capi.unproject(d["feat"], d["proj"], d["coords"], method)
    ref = d[f"{method}_ac0"]
    if method == "sum":
        assert_bits_equal(out, ref)
    else:
        assert max_rel(out, ref) <= 1e-6


def test_golden_exercises_edge_cases(golden):
    """The small fixture must contain behind-camera voxels, exact-zero depth and
    out-of-bounds taps, or the bit-exact claims above prove little."""
    d = golden("unproject_small.npz")
    P, X = d["proj"].astype(np.float64), d["coords"].reshape(2, -1, 3).astype(np.float64)
    Xh = np.concatenate([X, np.ones(X.shape[:2] + (1,))], -1)
    w = np.einsum("bvk,bnk->bvn", P[:, :, 2, :], Xh)
    assert (w < 0).any() and (w == 0).any() and (w > 0).any()
    # some (frame, view) pairs leave voxels with nothing sampled (behind / out of bounds)
    zero_frac = [(capi.unproject(d["feat"][:, v:v + 1], d["proj"][:, v:v + 1], d["coords"], "sum")[b] == 0).mean()
                 for v in range(d["feat"].shape[1]) for b in range(2)]
    assert max(zero_frac) > 0.5 and min(zero_frac) < 0.5


@pytest.mark.parametrize("method", METHODS)
def test_torch_restatement_is_bit_exact(golden, method):
    d = golden("unproject_small.npz")
    for ac in (0, 1):
        out = restate_torch.unproject_heatmaps(
            torch.from_numpy(d["feat"]), torch.from_numpy(d["proj"]), torch.from_numpy(d["coords"]), method,
            torch.from_numpy(d["conf"]), align_corners=bool(ac)).numpy()
        assert_bits_equal(out, d[f"{method}_ac{ac}"])


def test_torch_restatement_rejects_unknown_aggregation(golden):
    d = golden("unproject_small.npz")
    with pytest.raises(ValueError, match="Unknown volume_aggregation_method"):
        restate_torch.unproject_heatmaps(torch.from_numpy(d["feat"]), torch.from_numpy(d["proj"]),
                                         torch.from_numpy(d["coords"]), "mean")


@pytest.mark.parametrize("softmax", (True, False))
@pytest.mark.parametrize("mult", (1.0, 1.7))
def test_softargmax_oracles(golden, softmax, mult):
    d = golden("softargmax_small.npz")
    key = f"sm{int(softmax)}_m{mult}"
    xyz, vol = capi.softargmax3d(d["vol"], d["coords"], softmax, mult)
    assert max_rel(xyz, d[f"xyz_{key}"]) <= 5e-6   # f32 reference vs f64 oracle (1.3e-6)
    assert max_rel(vol, d[f"vol_{key}"]) <= 1e-6
    v = torch.from_numpy(d["vol"]) * mult
    txyz, tvol = restate_torch.integrate_tensor_3d_with_coordinates(v, torch.from_numpy(d["coords"]), softmax)
    np.testing.assert_array_equal(txyz.numpy(), d[f"xyz_{key}"])
    np.testing.assert_array_equal(tvol.numpy(), d[f"vol_{key}"])


def test_softargmax_oracle_blob(golden):
    d = golden("softargmax_blob.npz")
    xyz, vol = capi.softargmax3d(d["vol"], d["coords"], True, 1.0)
    assert max_rel(xyz, d["xyz"]) <= 1e-6
    assert max_rel(vol, d["vol_out"]) <= 1e-6


@pytest.mark.parametrize("case", ("cfg1", "b3n3", "n8"))
@pytest.mark.parametrize("use_conf", (True, False))
def test_dlt_oracles(golden, case, use_conf):
    d = golden("dlt.npz")
    key = f"{case}_c{int(use_conf)}"
    conf = d[f"conf_{case}"] if use_conf else None
    # torch restatement reproduces the float32 reference bit-for-bit
    t = restate_torch.triangulate_batch_of_points(torch.from_numpy(d[f"proj_{case}"]),
                                                  torch.from_numpy(d[f"points_{case}"]),
                                                  None if conf is None else torch.from_numpy(conf)).numpy()
    np.testing.assert_array_equal(t, d[f"out_{key}"])
    # float64 restatement: agrees with the reference's own float64 re-run
    x64 = restate_np.triangulate_batch_of_points(d[f"proj_{case}"], d[f"points_{case}"], conf)
    assert max_rel(x64, d[f"out64_{key}"]) <= 2e-6
    # ... and the float32 reference is within its known conditioning error of it
    assert max_rel(d[f"out_{key}"], x64) <= 1e-3
    # design matrix: C restatement == numpy restatement, bit for bit
    for b in range(d[f"points_{case}"].shape[0]):
        for j in range(0, d[f"points_{case}"].shape[2], 4):
            a_c = capi.dlt_design(d[f"proj_{case}"], d[f"points_{case}"], conf, b, j)
            a_n = restate_np.design_matrix(d[f"proj_{case}"][b], d[f"points_{case}"][b, :, j],
                                           None if conf is None else conf[b, :, j])
            np.testing.assert_array_equal(a_c, a_n)


@pytest.mark.parametrize("softmax", (True, False))
@pytest.mark.parametrize("mult", (1.0, 1.7))
def test_softargmax2d_oracles(golden, softmax, mult):
    """integrate_tensor_2d (op.py:11-47): the torch restatement reproduces the reference's
    bits; the float64 restatement is within f32 rounding."""
    d = golden("softargmax2d.npz")
    key = f"sm{int(softmax)}_m{mult}"
    h = torch.from_numpy(d["hm"]) * mult
    xy, maps = restate_torch.integrate_tensor_2d(h, softmax)
    np.testing.assert_array_equal(xy.numpy(), d[f"xy_{key}"])
    np.testing.assert_array_equal(maps.numpy(), d[f"maps_{key}"])
    xy64, maps64 = restate_np.integrate_tensor_2d(h.numpy(), softmax)
    assert max_rel(xy64, d[f"xy_{key}"]) <= 1e-6
    assert max_rel(maps64, d[f"maps_{key}"]) <= 1e-6


def test_softargmax2d_oracle_cfg_slice(golden):
    """96^2 peaked maps: the f32 reference's own summation error (9216-term mass sums times
    the pixel index) is 1.2e-5 relative to the float64 restatement — inside the 1e-4 bar."""
    d = golden("softargmax2d.npz")
    xy64, _ = restate_np.integrate_tensor_2d(d["cfg"], True)
    assert max_rel(xy64, d["cfg_xy"]) <= 5e-5
    xy, _ = restate_torch.integrate_tensor_2d(torch.from_numpy(d["cfg"]), True)
    np.testing.assert_array_equal(xy.numpy(), d["cfg_xy"])


@pytest.mark.parametrize("case", ("coco_eval", "coco_train", "mpii_cmu"))
def test_coord_volume_restatement(golden, case):
    """triangulation.py:280-341 restated op for op, with its own rotation restatement, equals
    the loop run through the reference's volumetric.rotate_coord_volume bit for bit."""
    d = golden("coord_volumes.npz")
    kind = "coco" if case.startswith("coco") else "mpii"
    cv = restate_torch.build_coord_volumes(d["base"], 2500.0, 16, d[f"theta_{case}"], kind, case == "mpii_cmu")
    np.testing.assert_array_equal(cv.numpy(), d[f"cv_{case}"])


def test_coord_volume_numpy_recipe(golden):
    """The kernel's f32 op order (csrc/coord_volumes.hip), restated in numpy
    (oracle/restate_np.coord_volumes), reproduces the reference's bits."""
    d = golden("coord_volumes.npz")
    for case, kind, cmu in (("coco_eval", "coco", False), ("coco_train", "coco", False), ("mpii_cmu", "mpii", True)):
        cv = restate_np.coord_volumes(d["base"], 2500.0, 16, d[f"theta_{case}"], kind, cmu)
        np.testing.assert_array_equal(cv, d[f"cv_{case}"])


def test_ce_loss_oracles(golden):
    """VolumetricCELoss (loss.py:52-80): the torch restatement reproduces the reference's
    loss and gradient; the squared-distance argmin (the kernel's rule) selects exactly the
    voxels where the reference's gradient is non-zero."""
    d = golden("ce_loss.npz")
    vol = torch.from_numpy(d["vol"]).requires_grad_(True)
    loss = restate_torch.volumetric_ce_loss(torch.from_numpy(d["coords"]), vol, torch.from_numpy(d["kps"]),
                                            torch.from_numpy(d["validity"]))
    loss.backward()
    np.testing.assert_array_equal(loss.detach().numpy(), d["loss"])
    np.testing.assert_array_equal(vol.grad.numpy(), d["grad_vol"])
    idx = restate_np.nearest_voxel(d["coords"], d["kps"])
    g = d["grad_vol"].reshape(2, 17, -1)
    valid = d["validity"][..., 0] > 0
    for b in range(2):
        for j in range(17):
            if valid[b, j]:
                assert np.flatnonzero(g[b, j]).tolist() == [idx[b, j]]


def test_v2v_front_folding_and_packing(golden):
    """Eval-mode Basic3DBlock(32, 16, 7) = relu(conv * s + shift) with the BN folded in
    float64 (mvn_rocm.v2v.fold_basic3d_block); the packed MFMA B operands hold
    W[lane & 15][8 * (lane >> 4) + j][tap]."""
    import torch.nn.functional as F
    from mvn_rocm import v2v
    d = golden("v2v_front.npz")
    t = {k: torch.from_numpy(np.asarray(d[k])) for k in ("weight", "bias", "bn_weight", "bn_bias", "bn_mean", "bn_var")}
    packed, scale, shift = v2v.fold_basic3d_block(t["weight"], t["bias"], t["bn_weight"], t["bn_bias"], t["bn_mean"],
                                                  t["bn_var"], float(d["eps"]), device="cpu")
    conv = F.conv3d(torch.from_numpy(d["x"]), t["weight"], None, padding=3)
    y = torch.relu(conv * scale.view(1, -1, 1, 1, 1) + shift.view(1, -1, 1, 1, 1))
    assert max_rel(y.numpy(), d["y"]) <= 1e-5
    w = t["weight"].reshape(16, 32, 343)
    for tap, lane, j in ((0, 0, 0), (123, 37, 5), (342, 63, 7), (200, 16, 0)):
        assert float(packed[tap, lane, j]) == float(w[lane % 16, 8 * (lane // 16) + j, tap].bfloat16())


# ----------------------------------------------------------------------------- caller chains
def test_chain_golden_pins_the_oracles(golden):
    """tests/golden/chains.npz ran the reference models' own forward() (triangulation.py:149-200,
    :245-355) with fixed backbone outputs.  The oracles reproduce every stage of it: the
    coordinate volumes (numpy recipe, bit-exact), the unprojection (C restatement,
    bit-exact for the f32 path up to the softmax exp), the soft-argmax and the DLT."""
    d = golden("chains.npz")
    # volumetric: coordinate volumes, unprojection, soft-argmax (multiplier 1.0, softmax)
    cv = restate_np.coord_volumes(d["vol_base"], float(d["vol_side"]), 32, d["vol_thetas"], "mpii", False)
    np.testing.assert_array_equal(cv, d["vol_coords"])
    np.testing.assert_array_equal(d["vol_base_points"], d["vol_base"].astype(np.float32))
    vol = capi.unproject(d["vol_features"], d["vol_proj"], cv, "softmax")
    sub = (slice(None), slice(None), slice(None, None, 4), slice(None, None, 4), slice(None, None, 4))
    assert max_rel(vol[sub], d["vol_unprojected_sub"]) <= 1e-6
    xyz, sm = capi.softargmax3d(vol[:, :17], cv, True, 1.0)
    assert max_rel(xyz, d["vol_kp3d"]) <= 1e-5
    assert max_rel(sm[sub], d["vol_volumes_sub"]) <= 1e-5
    # algebraic: 2D soft-argmax of heatmaps * 100, confidence normalisation, upscale, DLT
    B, N, J, H, W = d["alg_heatmaps"].shape
    hm = d["alg_heatmaps"].astype(np.float32).reshape(B * N, J, H, W) * d["alg_multiplier"]
    xy, _ = restate_np.integrate_tensor_2d(hm, True)
    kp2 = xy.reshape(B, N, J, 2) * np.array([384 / W, 384 / H])
    assert max_rel(kp2, d["alg_kp2d64"]) <= 1e-6
    conf = d["alg_conf"].astype(np.float64)
    conf = conf / conf.sum(1, keepdims=True) + 1e-5
    x64 = restate_np.triangulate_batch_of_points(d["alg_proj"], kp2, conf)
    assert max_rel(x64, d["alg_kp3d64"]) <= 1e-6
    assert max_rel(d["alg_kp3d"], d["alg_kp3d64"]) <= 1e-3     # the f32 reference's own SVD error


@pytest.mark.parametrize("method,ac,bf16", [("sum", 0, False), ("softmax", 1, False), ("conf", 0, False),
                                            ("max", 0, True)])
def test_oracle_under_address_sanitizer(golden, tmp_path, method, ac, bf16):
    """SURVEY.md §5 (sanitizers): the C oracle built with -fsanitize=address,undefined
    (oracle/asan_driver.c, every array in a malloc block of exactly its size) runs the golden
    inputs — unprojection (out-of-image taps, behind-camera voxels, non-square maps), the
    soft-argmax of its first channels and every DLT design matrix — with no sanitizer report,
    and its outputs equal the regular build's (and, for sum, the reference golden) bit for bit."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    exe = os.path.join(ROOT, "oracle", "_build", "oracle_asan")
    g = golden("unproject_small.npz")
    feat = g["feat_bf16_bits"] if bf16 else g["feat"]
    P, coords, conf = g["proj"], g["coords"], g["conf"]
    B, N, C, H, W = feat.shape
    Vx, Vy, Vz = coords.shape[1:4]
    J = 3
    rng = np.random.default_rng(7)
    pts = rng.uniform(0, 20, (B, N, J, 2)).astype(np.float32)
    pconf = rng.uniform(0.1, 1, (B, N, J)).astype(np.float32)
    hdr = np.array([B, N, C, H, W, Vx, Vy, Vz, capi.agg_code(method), ac, int(bf16), J], np.int32)
    blob = b"".join(np.ascontiguousarray(a).tobytes() for a in (hdr, feat, P, coords, conf, pts, pconf))
    (tmp_path / "in.bin").write_bytes(blob)
    r = subprocess.run([exe, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True, text=True,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), np.float32)
    nv = Vx * Vy * Vz
    vol = out[:B * C * nv].reshape(B, C, Vx, Vy, Vz)
    ref = capi.unproject(feat, P, coords, method, conf, align_corners=bool(ac), feat_bf16_bits=bf16)
    np.testing.assert_array_equal(vol, ref)
    if method == "sum" and not bf16:
        np.testing.assert_array_equal(vol, g[f"sum_ac{ac}"])
    o = B * C * nv
    xyz = out[o:o + B * J * 3].reshape(B, J, 3)
    ref_xyz, ref_sv = capi.softargmax3d(np.ascontiguousarray(ref[:, :J]), coords, True, 1.0)
    np.testing.assert_array_equal(xyz, ref_xyz)
    o += B * J * 3
    np.testing.assert_array_equal(out[o:o + B * J * nv].reshape(ref_sv.shape), ref_sv)
    o += B * J * nv
    A = out[o:].reshape(B, J, 2 * N, 4)
    for b in range(B):
        for j in range(J):
            np.testing.assert_array_equal(A[b, j], capi.dlt_design(P, pts, pconf, b, j))


@pytest.mark.parametrize("method", METHODS)
def test_c_oracle_nan_features_follow_torch(golden, method):
    """NaN feature pixels: the C oracle propagates them as the reference's ATen ops do —
    through sums and the view softmax, and in 'max' with torch.max(dim)'s order (NaN above
    every number, ties to the first view)."""
    d = golden("unproject_small.npz")
    feat = d["feat"].copy()
    feat.reshape(-1)[np.random.default_rng(0).choice(feat.size, 40, replace=False)] = np.nan
    out = capi.unproject(feat, d["proj"], d["coords"], method, d["conf"], False)
    ref = restate_torch.unproject_heatmaps(torch.from_numpy(feat), torch.from_numpy(d["proj"]),
                                           torch.from_numpy(d["coords"]), method, torch.from_numpy(d["conf"])).numpy()
    assert np.isnan(ref).sum() > 50
    assert_parity_with_nans(out, ref, method, tol=1e-6)


def test_backward_golden_is_the_exact_sum_of_forward_tap_products(golden):
    """The element-wise backward golden (the reference's own autograd, captured in the build
    container) equals the exact sum of the forward's f32 tap products per element within
    1e-6 relative: the reference's 'sum' feature gradient on that host is that sum, which is
    what the GPU's deterministic backward is checked to reproduce (test_gpu_backward.py)."""
    from oracle import restate_np
    d = golden("unproject_bwd_elementwise.npz")
    ref = d["grad_feat_sum"].astype(np.float64)
    ex = restate_np.unproject_sum_feature_grad(d["feat"].shape, d["proj"], d["coords"], d["grad_out_sum"])
    assert np.array_equal(ex == 0, ref == 0)
    nz = ref != 0
    assert (np.abs(ex[nz] - ref[nz]) / np.abs(ref[nz])).max() <= 1e-6
