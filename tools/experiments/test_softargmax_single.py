# ARCHIVED with tools/experiments/softargmax_single.hip (not kept, profiles/r17_ab_softargmax_single.txt);
# needs that kernel built in place of csrc/softargmax.hip plus its debug hook in the C ABI.
"""Single-pass 3D soft-argmax (csrc/softargmax.hip softargmax_single) vs the three-launch path
and the oracle (MI355X only).

The single pass keeps each (frame, 1024-voxel) unit's values in registers while the frame's
last arriving block folds the partials, so the volume is read once.  Its partials are
per-block (four wave partials merged) instead of pass 1's per-wave partials, so it is not
bit-identical to the three-launch path; both are held to the oracle bars of
tests/test_gpu_parity.py (coordinates and volumes <= 1e-5 max-rel, op.py:84-96) and to
each other at 1e-6.  Repeated calls are bit-identical (the partials are folded by index,
not in arrival order), and the control words are re-zeroed every call.
"""
import numpy as np
import pytest
import torch

from conftest import max_rel
from oracle import capi

pytestmark = pytest.mark.gpu


def _op():
    from mvn_rocm import op
    return op


def _three_pass():
    from mvn_rocm import _lib
    return _lib.softargmax_knobs(three_pass=True)


def _inputs(B, J, V, seed, dtype=torch.float32, scale=4.0):
    from mvn_rocm import synth
    vb = synth.volumetric_batch(B, channels=1, volume=V, seed=seed)
    vol = torch.randn((B, J, V, V, V), generator=torch.Generator().manual_seed(seed)) * scale
    return vol.to(dtype), vb.coords


@pytest.mark.parametrize("dtype", (torch.float32, torch.bfloat16))
@pytest.mark.parametrize("softmax", (True, False))
@pytest.mark.parametrize("B,J,V", ((2, 17, 64), (3, 20, 20), (1, 5, 16), (2, 24, 24)))
def test_single_pass_matches_oracle_and_three_pass(device, dtype, softmax, B, J, V):
    vol, coords = _inputs(B, J, V, seed=B * 100 + J + V, dtype=dtype)
    xyz, out = _op().integrate_tensor_3d_with_coordinates(vol.to(device), coords.to(device), softmax, multiplier=1.3)
    with _three_pass():
        xyz3, out3 = _op().integrate_tensor_3d_with_coordinates(vol.to(device), coords.to(device), softmax,
                                                                multiplier=1.3)
    ref_xyz, ref_vol = capi.softargmax3d(vol.float().numpy(), coords.numpy(), softmax, 1.3)
    assert out.dtype == dtype
    assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-5
    assert max_rel(xyz.cpu().numpy(), xyz3.cpu().numpy()) <= 1e-6
    if dtype == torch.float32:
        assert max_rel(out.cpu().numpy(), ref_vol) <= 1e-5
        assert max_rel(out.cpu().numpy(), out3.cpu().numpy()) <= 1e-6
    else:                                   # bf16 output: within one bf16 ulp of the oracle
        np.testing.assert_allclose(out.float().cpu().numpy(), ref_vol, rtol=2 ** -8, atol=1e-30)
        # each within one ulp of the oracle, so within two of each other (a value near a
        # rounding boundary can round to either side in the two paths)
        np.testing.assert_allclose(out.float().cpu().numpy(), out3.float().cpu().numpy(), rtol=2 ** -7, atol=1e-30)


def test_single_pass_channel_slice_many_frames(device):
    """The bench's operand (channels [0:17] of a (B, 32, 64^3) volume, no copy) with more
    units than the chip holds at once (the persistent loop takes several tickets per block)."""
    B, V = 24, 64
    from mvn_rocm import synth
    vb = synth.volumetric_batch(B, channels=1, volume=V, seed=5, device=device)
    big = torch.randn((B, 32, V, V, V), device=device, generator=torch.Generator(device).manual_seed(5)) * 3
    sl = big[:, :17]
    assert not sl.is_contiguous()
    xyz, out = _op().integrate_tensor_3d_with_coordinates(sl, vb.coords, multiplier=1.1)
    with _three_pass():
        xyz3, out3 = _op().integrate_tensor_3d_with_coordinates(sl, vb.coords, multiplier=1.1)
    assert max_rel(xyz.cpu().numpy(), xyz3.cpu().numpy()) <= 1e-6
    assert max_rel(out.cpu().numpy(), out3.cpu().numpy()) <= 1e-6
    # two frames against the oracle
    for b in (0, B - 1):
        ref_xyz, ref_vol = capi.softargmax3d(sl[b:b + 1].cpu().numpy(), vb.coords[b:b + 1].cpu().numpy(), True, 1.1)
        assert max_rel(xyz[b:b + 1].cpu().numpy(), ref_xyz) <= 1e-5
        assert max_rel(out[b:b + 1].cpu().numpy(), ref_vol) <= 1e-5
    # repeated calls: bit-identical (partials folded by index; control words re-zeroed per call)
    for _ in range(3):
        xyz_r, out_r = _op().integrate_tensor_3d_with_coordinates(sl, vb.coords, multiplier=1.1)
        torch.testing.assert_close(xyz_r, xyz, rtol=0, atol=0)
        torch.testing.assert_close(out_r, out, rtol=0, atol=0)


def test_single_pass_fallbacks(device):
    """Shapes the single pass leaves to the three launches: J > 24, unaligned voxel counts."""
    for B, J, V in ((1, 30, 16), (2, 7, 17)):
        vol, coords = _inputs(B, J, V, seed=J + V)
        xyz, out = _op().integrate_tensor_3d_with_coordinates(vol.to(device), coords.to(device), multiplier=0.9)
        ref_xyz, ref_vol = capi.softargmax3d(vol.numpy(), coords.numpy(), True, 0.9)
        assert max_rel(xyz.cpu().numpy(), ref_xyz) <= 1e-5
        assert max_rel(out.cpu().numpy(), ref_vol) <= 1e-5


def test_single_pass_without_volume_and_cuboids(device):
    from mvn_rocm import volumetric
    B, J, V = 3, 17, 32
    vol = (torch.randn((B, J, V, V, V), generator=torch.Generator().manual_seed(2)) * 5).to(device)
    base = np.array([[100.0, -50.0, 950.0], [0.0, 0.0, 900.0], [-300.0, 200.0, 1000.0]])
    theta = np.array([0.3, 1.9, 4.0])
    cub = volumetric.build_cuboids(base, 2500.0, V, theta, device=device)
    xyz, out = _op().integrate_tensor_3d_with_coordinates(vol, cub, multiplier=1.0)
    with _three_pass():
        xyz3, out3 = _op().integrate_tensor_3d_with_coordinates(vol, cub, multiplier=1.0)
    assert max_rel(xyz.cpu().numpy(), xyz3.cpu().numpy()) <= 1e-6
    assert max_rel(out.cpu().numpy(), out3.cpu().numpy()) <= 1e-6
    xyz_n, none = _op().integrate_tensor_3d_with_coordinates(vol, cub, multiplier=1.0, return_volumes=False)
    assert none is None
    torch.testing.assert_close(xyz_n, xyz, rtol=0, atol=0)
