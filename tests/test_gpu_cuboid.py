"""In-kernel coordinate volumes (mvn_unproject_cuboid /
mvn_softargmax3d_cuboid) on the MI355X.

The reference builds coord_volumes per frame (triangulation.py:280-341) and feeds the same
tensor to unproject_heatmaps (op.py:99) and integrate_tensor_3d_with_coordinates (op.py:84).
The cuboid entry points form the coordinates inside the kernels with the same f32 op order
as mvn_coord_volumes (cuboid_coord, csrc/common.hpp), so the bar is bit-identity with the
tensor path fed the materialised volume, and the oracle on the numpy restatement of the
coordinate volume (restate_np.coord_volumes, pinned by the reference's coord-volume goldens).
"""
import numpy as np
import pytest
import torch

from conftest import assert_bits_equal, max_rel
from oracle import capi, restate_np

pytestmark = pytest.mark.gpu


def _frames(B, V, seed, kind="coco", transfer=False):
    from mvn_rocm import volumetric
    rng = np.random.default_rng(seed)
    base = rng.uniform(-500, 500, (B, 3)) + np.array([0, 0, 900.0])
    thetas = rng.uniform(0, 2 * np.pi, B)
    cub = volumetric.build_cuboids(base, 2500.0, V, thetas, kind, transfer, device="cuda:0")
    ref_coords = restate_np.coord_volumes(base, 2500.0, V, thetas, kind, transfer)
    return cub, ref_coords


def _bits(t):
    return t.view(torch.int32) if t.dtype == torch.float32 else t.view(torch.int16)


@pytest.mark.parametrize("n_views", (1, 3, 4, 8))
@pytest.mark.parametrize("method", ("sum", "max", "softmax", "conf"))
@pytest.mark.parametrize("V,kind,transfer", ((16, "coco", False), (20, "mpii", True), (64, "coco", False)))
def test_unproject_cuboid_is_bit_identical_to_the_volume_path(device, n_views, method, V, kind, transfer):
    from mvn_rocm import op, synth
    B = 2
    vb = synth.volumetric_batch(B, n_views=n_views, channels=8, volume=8, seed=3)
    cub, ref_coords = _frames(B, V, seed=V + n_views, kind=kind, transfer=transfer)
    coords = cub.coord_volumes()
    np.testing.assert_array_equal(coords.cpu().numpy(), ref_coords)
    feat, proj = vb.features.to(device), vb.proj.to(device)
    conf = torch.rand((B, n_views, 8), generator=torch.Generator().manual_seed(1)).to(device)
    a = op.unproject_heatmaps(feat, proj, cub, method, conf)
    b = op.unproject_heatmaps(feat, proj, coords, method, conf)
    assert a.shape == (B, 8, V, V, V)
    assert torch.equal(_bits(a), _bits(b))
    if V <= 20:
        ref = capi.unproject(vb.features.numpy(), vb.proj.numpy(), ref_coords, method, conf.cpu().numpy())
        if method == "softmax":
            assert max_rel(a.cpu().numpy(), ref) <= 1e-5
        else:
            assert_bits_equal(a.cpu().numpy(), ref)


def test_unproject_cuboid_bf16_and_every_kernel_path(device):
    from mvn_rocm import op, synth
    B, V = 2, 24
    vb = synth.volumetric_batch(B, n_views=4, channels=8, volume=8, seed=5)
    cub, _ = _frames(B, V, seed=9)
    coords = cub.coord_volumes()
    feat, proj = vb.features.to(device).to(torch.bfloat16), vb.proj.to(device)
    from mvn_rocm import _lib
    for budget in (0, 300, 40):        # one pass, several passes, global-gather fallback
        with _lib.unproject_knobs(budget):
            for od in (None, torch.float32):
                a = op.unproject_heatmaps(feat, proj, cub, "softmax", out_dtype=od)
                b = op.unproject_heatmaps(feat, proj, coords, "softmax", out_dtype=od)
                assert torch.equal(_bits(a), _bits(b)), budget


def test_unproject_cuboid_more_than_8_views_materialises(device):
    from mvn_rocm import op, synth
    vb = synth.volumetric_batch(1, n_views=9, channels=4, volume=8, seed=2)
    cub, _ = _frames(1, 12, seed=2)
    feat, proj = vb.features.to(device), vb.proj.to(device)
    a = op.unproject_heatmaps(feat, proj, cub, "sum")
    b = op.unproject_heatmaps(feat, proj, cub.coord_volumes(), "sum")
    assert torch.equal(a, b)


@pytest.mark.parametrize("softmax", (True, False))
@pytest.mark.parametrize("V,kind,transfer", ((16, "coco", False), (20, "mpii", True), (64, "coco", False)))
def test_softargmax_cuboid_is_bit_identical_to_the_volume_path(device, softmax, V, kind, transfer):
    from mvn_rocm import op, synth
    B = 2
    cub, ref_coords = _frames(B, V, seed=V, kind=kind, transfer=transfer)
    coords = cub.coord_volumes()
    vol = synth.blob_volumes(coords.cpu(), 17, seed=V).to(device)
    for dt in (torch.float32, torch.bfloat16):
        v = vol.to(dt)
        xa, oa = op.integrate_tensor_3d_with_coordinates(v, cub, softmax, multiplier=1.3)
        xb, ob = op.integrate_tensor_3d_with_coordinates(v, coords, softmax, multiplier=1.3)
        assert torch.equal(_bits(xa), _bits(xb)) and torch.equal(_bits(oa), _bits(ob))
    if V <= 20:
        rx, rv = capi.softargmax3d(vol.cpu().numpy(), ref_coords, softmax, 1.3)
        xa, oa = op.integrate_tensor_3d_with_coordinates(vol, cub, softmax, multiplier=1.3)
        assert max_rel(xa.cpu().numpy(), rx) <= 1e-5 and max_rel(oa.cpu().numpy(), rv) <= 1e-5


def test_softargmax_cuboid_channel_slice(device):
    """A channel slice of an unprojected volume (batch / joint strides, no copy)."""
    from mvn_rocm import op, synth
    B, V = 2, 32
    vb = synth.volumetric_batch(B, n_views=4, channels=20, volume=8, seed=6)
    cub, _ = _frames(B, V, seed=6)
    vol = op.unproject_heatmaps(vb.features.to(device), vb.proj.to(device), cub, "softmax")
    xa, oa = op.integrate_tensor_3d_with_coordinates(vol[:, :17], cub)
    xb, ob = op.integrate_tensor_3d_with_coordinates(vol[:, :17], cub.coord_volumes())
    assert torch.equal(xa, xb) and torch.equal(oa, ob)


def test_cuboid_gradients_match_the_volume_path(device):
    from mvn_rocm import op, synth
    B, V = 1, 16
    vb = synth.volumetric_batch(B, n_views=4, channels=17, volume=8, seed=7)
    cub, _ = _frames(B, V, seed=7)
    coords = cub.coord_volumes()
    grads = []
    for c in (cub, coords):
        feat = vb.features.to(device).requires_grad_(True)
        vol = op.unproject_heatmaps(feat, vb.proj.to(device), c, "softmax")
        xyz, _ = op.integrate_tensor_3d_with_coordinates(vol, c)
        (xyz.square().sum()).backward()
        grads.append(feat.grad)
    # the unprojection backward scatters with float atomics (csrc/unproject_bwd.hip): its
    # summation order, not the coordinates, varies between runs
    assert max_rel(grads[0].cpu().numpy(), grads[1].cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("n_views", (4, 8))
@pytest.mark.parametrize("dt", (torch.float32, torch.bfloat16))
def test_channels_last_cuboid_is_bit_identical(device, dt, n_views):
    """Config 5's channels-last unprojection (V2V front input) with in-kernel coordinates:
    bit-identical to the coordinate-volume path and a transpose of the NCDHW output, for
    the 4- and 8-view instantiations (8 views: 2-channel packed stores) and on every
    staging path (one LDS pass, several passes, global-gather fallback)."""
    from mvn_rocm import _lib, op, synth, v2v
    B, V = 2, 32
    vb = synth.volumetric_batch(B, n_views=n_views, channels=32, volume=8, seed=8)
    cub, _ = _frames(B, V, seed=8)
    feat, proj = vb.features.to(device).to(dt), vb.proj.to(device)
    for budget in (0, 300, 40):
        with _lib.unproject_knobs(budget):
            for od in ((torch.bfloat16, torch.float32) if dt == torch.bfloat16 else (torch.float32,)):
                a = v2v.unproject_channels_last(feat, proj, cub, "softmax", out_dtype=od)
                b = v2v.unproject_channels_last(feat, proj, cub.coord_volumes(), "softmax", out_dtype=od)
                assert a.shape == (B, V, V, V, 32) and torch.equal(_bits(a), _bits(b)), budget
                c = op.unproject_heatmaps(feat, proj, cub, "softmax", out_dtype=od)
                assert torch.equal(_bits(a), _bits(c.permute(0, 2, 3, 4, 1).contiguous())), budget
