"""The chunk-staged unprojection kernel (csrc/unproject_x4.hip: chunked staging, packed f32
arithmetic; 4 views with 4-channel LDS slots, 8 views with 2-channel slots) against the generic tiled kernel (bit for bit, every aggregation, dtype and
layout) and against the C oracle, on every staging path (one LDS pass, several passes,
global-gather fallback) and on coordinate volumes that are not affine grids.  MI355X only."""
import numpy as np
import pytest
import torch

from conftest import assert_bits_equal, assert_parity_with_nans, max_rel
from oracle import capi

pytestmark = pytest.mark.gpu

METHODS = ("sum", "max", "softmax", "conf")


def _bits(t):
    return t.contiguous().view(torch.int32) if t.dtype == torch.float32 else t.contiguous().view(torch.int16)


def _run(vb_feat, proj, coords, method, conf, out_dtype=None, **knobs):
    from mvn_rocm import _lib, op
    with _lib.unproject_knobs(**knobs):
        return op.unproject_heatmaps(vb_feat, proj, coords, method, conf, out_dtype=out_dtype)


def _batch(device, seed, heatmap=64, volume=32, channels=8, dtype=torch.float32, n_views=4):
    from mvn_rocm import synth
    vb = synth.volumetric_batch(2, n_views=n_views, channels=channels, heatmap=heatmap, volume=volume, seed=seed)
    conf = torch.from_numpy(np.random.default_rng(seed).uniform(0.05, 1.0, (2, n_views, channels)).astype(np.float32))
    return vb, conf


# (views, channels): 4 views / 4-channel slots; 8 views / 2-channel slots, also with a channel
# count that is not a multiple of 4
VIEWS = ((4, 8), (8, 8), (8, 6))


@pytest.mark.parametrize("views", VIEWS, ids=lambda v: f"{v[0]}v{v[1]}c")
@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("dt", ("f32", "bf16", "bf16->f32"))
def test_x4_equals_generic_kernel_and_oracle(device, method, dt, views):
    vb, conf = _batch(device, 70, n_views=views[0], channels=views[1])
    feat = vb.features.to(device)
    od = None
    if dt != "f32":
        feat = feat.to(torch.bfloat16)
        od = torch.float32 if dt == "bf16->f32" else None
    P, X, cf = vb.proj.to(device), vb.coords.to(device), conf.to(device)
    a = _run(feat, P, X, method, cf, od)
    b = _run(feat, P, X, method, cf, od, generic=True)
    assert torch.equal(_bits(a), _bits(b))
    bits = feat.cpu().view(torch.int16).numpy().view(np.uint16) if feat.dtype == torch.bfloat16 else None
    ref = capi.unproject(bits if bits is not None else vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy(),
                         method, conf.numpy(), feat_bf16_bits=bits is not None)
    got = a.float().cpu().numpy()
    if a.dtype == torch.bfloat16:
        np.testing.assert_allclose(got, ref, rtol=2 ** -8, atol=2 ** -8 * np.abs(ref).max())
    elif method == "softmax":
        assert max_rel(got, ref) <= 1e-5
    else:
        assert_bits_equal(got, ref)


def _tile_areas(proj, coords, H, W, tile=(4, 8, 16)):
    from test_gpu_parity import tile_footprints
    return tile_footprints(proj, coords, H, W, tile)


@pytest.mark.parametrize("n_views,dt", ((4, "f32"), (4, "bf16"), (8, "f32")))
@pytest.mark.parametrize("path", ("multipass", "fallback"))
@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_x4_staging_paths(device, path, method, n_views, dt):
    """LDS budgets that force several staging passes of whole views, and single views
    larger than the budget (global-gather fallback) — against the oracle (bf16 maps: on
    the same bf16 bits, f32 out)."""
    vb, conf = _batch(device, 71, heatmap=64, volume=32, channels=8, n_views=n_views)
    # X4Shape tiles: 4 views f32 4x8x16, 4 views bf16 8x8x8, 8 views 4x8x8
    tile = (4, 8, 8) if n_views == 8 else (8, 8, 8) if dt == "bf16" else (4, 8, 16)
    areas = _tile_areas(vb.proj.numpy(), vb.coords.numpy(), 64, 64, tile)
    if path == "multipass":
        budget = int(areas.max()) + 64
        assert (areas.sum(1) + 1 > budget).any()
    else:
        budget = int(np.median(areas[areas > 0]))
        assert (areas.max(1) > budget - 1).any() and (areas.max(1) <= budget - 1).any()
    feat = vb.features.to(torch.bfloat16) if dt == "bf16" else vb.features
    out = _run(feat.to(device), vb.proj.to(device), vb.coords.to(device), method, None, out_dtype=torch.float32,
               lds_slots=budget)
    bits = feat.view(torch.int16).numpy().view(np.uint16) if dt == "bf16" else feat.numpy()
    ref = capi.unproject(bits, vb.proj.numpy(), vb.coords.numpy(), method, feat_bf16_bits=dt == "bf16")
    if method == "softmax":
        assert max_rel(out.cpu().numpy(), ref) <= 1e-5
    else:
        assert_bits_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("n_views", (4, 8))
@pytest.mark.parametrize("method", ("sum", "softmax"))
def test_x4_non_affine_coordinates(device, method, n_views):
    """op.py:99 accepts ANY coordinate volume: jittered and shuffled voxel coordinates (not
    an affine grid) must still match the oracle."""
    vb, _ = _batch(device, 72, heatmap=64, volume=32, channels=8, n_views=n_views)
    rng = np.random.default_rng(72)
    X = vb.coords.numpy().copy()
    X += rng.normal(0, 40.0, X.shape).astype(np.float32)               # jitter (~1 voxel)
    flat = X.reshape(2, -1, 3)
    for b in range(2):                                                   # a few far-flung voxels
        idx = rng.choice(flat.shape[1], 200, replace=False)
        flat[b, idx] = flat[b, rng.permutation(idx)]
    out = _run(vb.features.to(device), vb.proj.to(device), torch.from_numpy(X).to(device), method, None)
    ref = capi.unproject(vb.features.numpy(), vb.proj.numpy(), X, method)
    if method == "softmax":
        assert max_rel(out.cpu().numpy(), ref) <= 1e-5
    else:
        assert_bits_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("channels", (32, 12, 20))
@pytest.mark.parametrize("dt", (torch.float32, torch.bfloat16))
def test_x4_channels_last_and_cuboids_equal_generic(device, dt, channels):
    """Channels-last output (config 5) and in-kernel cuboid coordinates through the
    four-view kernel, bit-identical to the generic kernel (12 / 20 channels: a channel
    group count that is not a multiple of the bf16 store grouping)."""
    from mvn_rocm import _lib, synth, v2v, volumetric
    vb = synth.volumetric_batch(2, n_views=4, channels=channels, heatmap=96, volume=8, seed=73)
    rng = np.random.default_rng(73)
    base = rng.uniform(-500, 500, (2, 3)) + np.array([0, 0, 900.0])
    cub = volumetric.build_cuboids(base, 2500.0, 32, rng.uniform(0, 2 * np.pi, 2), "coco", False, device=device)
    feat, P = vb.features.to(device).to(dt), vb.proj.to(device)
    a = v2v.unproject_channels_last(feat, P, cub, "softmax", out_dtype=dt)
    with _lib.unproject_knobs(generic=True):
        b = v2v.unproject_channels_last(feat, P, cub, "softmax", out_dtype=dt)
    assert torch.equal(_bits(a), _bits(b))


@pytest.mark.parametrize("n_views", (4, 8))
@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("dt", ("f32", "bf16", "bf16->f32"))
def test_x4_partial_tiles(device, method, dt, n_views):
    """A volume that is not a multiple of either tile (20 x 28 x 36 of a 40^3 grid): edge
    tiles with inactive voxels next to full ones — bitwise against the generic kernel, and
    against the oracle."""
    vb, conf = _batch(device, 74, heatmap=64, volume=40, channels=8, n_views=n_views)
    X = vb.coords[:, 2:22, 5:33, 1:37].contiguous()
    feat = vb.features.to(device)
    od = None
    if dt != "f32":
        feat = feat.to(torch.bfloat16)
        od = torch.float32 if dt == "bf16->f32" else None
    P, Xd, cf = vb.proj.to(device), X.to(device), conf.to(device)
    a = _run(feat, P, Xd, method, cf, od)
    b = _run(feat, P, Xd, method, cf, od, generic=True)
    assert a.shape == (2, 8, 20, 28, 36)
    assert torch.equal(_bits(a), _bits(b))
    bits = feat.cpu().view(torch.int16).numpy().view(np.uint16) if feat.dtype == torch.bfloat16 else None
    ref = capi.unproject(bits if bits is not None else vb.features.numpy(), vb.proj.numpy(), X.numpy(),
                         method, conf.numpy(), feat_bf16_bits=bits is not None)
    got = a.float().cpu().numpy()
    if a.dtype == torch.bfloat16:
        np.testing.assert_allclose(got, ref, rtol=2 ** -8, atol=2 ** -8 * np.abs(ref).max())
    elif method == "softmax":
        assert max_rel(got, ref) <= 1e-5
    else:
        assert_bits_equal(got, ref)


@pytest.mark.parametrize("dt", ("f32", "bf16"))
def test_x4_repeat_launches_bit_identical_full_size(device, dt):
    """Config-size volumes (4 x 32 x 96^2 -> 64^3) launched three times in each layout are
    bit-identical, and the channels-last volume is the NCDHW one transposed.  Guards the
    store-data hazard class (a >8-byte store whose data registers the next instruction
    overwrites: nondeterministic channels)."""
    from mvn_rocm import op, synth, v2v
    dtype = torch.bfloat16 if dt == "bf16" else torch.float32
    vb = synth.volumetric_batch(1, dtype=dtype, device=device, seed=57)
    nc = [op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax") for _ in range(3)]
    cl = [v2v.unproject_channels_last(vb.features, vb.proj, vb.coords, "softmax", out_dtype=dtype) for _ in range(3)]
    for t in nc[1:]:
        assert torch.equal(_bits(t), _bits(nc[0]))
    for t in cl[1:]:
        assert torch.equal(_bits(t), _bits(cl[0]))
    assert torch.equal(_bits(cl[0]), _bits(nc[0].permute(0, 2, 3, 4, 1)))


@pytest.mark.parametrize("n_views", (4, 8))
@pytest.mark.parametrize("method", ("sum", "max", "softmax", "conf"))
def test_x4_non_square_maps_and_align_corners(device, n_views, method):
    """Non-square maps on the chunk-staged kernel (W % 4 == 0, H != W: op.py:127-130 divides
    x by H and y by W — the reference's quirk) under both grid_sample conventions, against
    the oracle, and bit-identical to the generic kernel."""
    from mvn_rocm import synth
    rng = np.random.default_rng(90 + n_views)
    B, C, H, W = 2, 8, 56, 80
    vb = synth.volumetric_batch(B, n_views=n_views, channels=C, heatmap=max(H, W), volume=24, seed=90 + n_views)
    feat = rng.standard_normal((B, n_views, C, H, W)).astype(np.float32)
    proj = vb.proj.numpy()
    proj[:, :, 0] *= W / max(H, W)
    proj[:, :, 1] *= H / max(H, W)
    coords = vb.coords.numpy()
    conf = rng.uniform(0.05, 1.0, (B, n_views, C)).astype(np.float32)
    from mvn_rocm import _lib, op
    F, P, X, cf = (torch.from_numpy(a).to(device) for a in (feat, proj, coords, conf))
    for ac in (False, True):
        a = op.unproject_heatmaps(F, P, X, method, cf, align_corners=ac)
        with _lib.unproject_knobs(generic=True):
            b = op.unproject_heatmaps(F, P, X, method, cf, align_corners=ac)
        assert torch.equal(_bits(a), _bits(b)), ac
        ref = capi.unproject(feat, proj, coords, method, conf, ac)
        if method == "softmax":
            assert max_rel(a.cpu().numpy(), ref) <= 1e-5
        else:
            assert_bits_equal(a.cpu().numpy(), ref)


@pytest.mark.parametrize("n_views", (4, 8, 9))
@pytest.mark.parametrize("method", METHODS)
def test_nan_features_follow_the_reference(device, n_views, method):
    """NaN feature pixels on every kernel (chunk-staged x4 at 4 / 8 views, the generic tiled
    kernel, the simple kernel at 9 views): the outputs hold NaN exactly where the oracle
    (pinned to torch's ops, tests/test_oracle.py) does — 'max' in torch.max(dim)'s order."""
    from mvn_rocm import _lib, op
    vb, conf = _batch(device, 75, heatmap=64, volume=24, channels=8, n_views=n_views)
    feat = vb.features.numpy().copy()
    feat.reshape(-1)[np.random.default_rng(75).choice(feat.size, 300, replace=False)] = np.nan
    ref = capi.unproject(feat, vb.proj.numpy(), vb.coords.numpy(), method, conf.numpy())
    assert np.isnan(ref).any()
    F, P, X, cf = (torch.from_numpy(a).to(device) for a in (feat, vb.proj.numpy(), vb.coords.numpy(), conf.numpy()))
    for generic in (False, True):
        with _lib.unproject_knobs(generic=generic):
            out = op.unproject_heatmaps(F, P, X, method, cf)
        assert_parity_with_nans(out.cpu().numpy(), ref, method)
