"""Capture golden input/output vectors from the REFERENCE implementation.

Run in the build container only (it needs /root/reference; the GPU box never runs it):

    python -B tests/golden/make_golden.py [softargmax2d|coord_volumes|ce_loss|v2v_front|chains|dlt_degenerate|bwd_elementwise]   (argument: only that fixture)

The reference (learnable-triangulation-pytorch, mvn/utils/op.py and
mvn/utils/multiview.py) is imported read-only with two in-memory accommodations:
  * ``cv2`` is not installed: an empty module is placed in sys.modules.  op.py only
    uses img.to_numpy / to_torch, which never touch cv2.
  * ``align_corners=True`` goldens (the torch 1.0.1 semantics the reference pins,
    requirements.txt:20) are captured by temporarily binding F.grid_sample with
    align_corners=True around the reference call; all other goldens use torch 2.10's
    default (False), exactly as op.py:134 calls it.
Only data (inputs and the reference's outputs / gradients) is written, as .npz files
next to this script.  Nothing from the reference's source is copied.
"""
from __future__ import annotations

import contextlib
import functools
import math
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "learnable-triangulation-pytorch_amd"))

from mvn_rocm import synth  # noqa: E402  (pure numpy/torch; no GPU needed)


def import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, REF)
    from mvn.utils import op, multiview  # noqa: WPS433
    return op, multiview


@contextlib.contextmanager
def grid_sample_align_corners(flag: bool):
    orig = F.grid_sample
    F.grid_sample = functools.partial(orig, align_corners=flag)
    try:
        yield
    finally:
        F.grid_sample = orig


def meta():
    return dict(torch_version=np.array(torch.__version__),
                cpu_capability=np.array(torch.backends.cpu.get_cpu_capability()))


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays, **meta())
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB")


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)


# ----------------------------------------------------------------------------- inputs
def small_unproject_inputs(seed=0):
    """B=2 frames, N=3 views, C=5, non-square 17x23 maps, non-cubic V=(8,9,10).
    Frame 0: axis-aligned grid with exact coordinates and an axis-aligned camera whose
    depth is exactly 0 on the z=900 plane (exercises the w==0 guard, op.py:123) and
    negative below it (the depth mask, op.py:121).  Frame 1: rotated grid, one camera
    inside the cuboid (half the voxels behind it)."""
    rng = np.random.default_rng(seed)
    H, W = 17, 23
    Vx, Vy, Vz = 8, 9, 10
    B, N, C = 2, 3, 5
    coords = np.zeros((B, Vx, Vy, Vz, 3), np.float32)
    gx, gy, gz = np.meshgrid(np.arange(Vx), np.arange(Vy), np.arange(Vz), indexing="ij")
    coords[0, ..., 0] = -400.0 + 100.0 * gx
    coords[0, ..., 1] = -450.0 + 100.0 * gy
    coords[0, ..., 2] = 500.0 + 100.0 * gz          # includes z == 900 exactly
    rot = synth.rotation_matrix([0.3, 1.0, 0.2], 0.7)
    pts = np.stack([gx, gy, gz], -1).reshape(-1, 3) * 120.0 - np.array([420.0, 480.0, 540.0])
    coords[1] = (pts @ rot.T + np.array([50.0, -30.0, 900.0])).reshape(Vx, Vy, Vz, 3)

    proj = np.zeros((B, N, 3, 4), np.float64)
    for b in range(B):
        cams = synth.ring_cameras(N, rng)
        for v, cam in enumerate(cams):
            K = cam.K.copy()
            K[0, 0] *= W / 384.0
            K[0, 2] *= W / 384.0
            K[1, 1] *= H / 384.0
            K[1, 2] *= H / 384.0
            proj[b, v] = K @ np.hstack([cam.R, cam.t])
    f = 40.0
    proj[0, 2] = np.array([[f, 0.0, 11.5, -11.5 * 900.0], [0.0, f, 8.5, -8.5 * 900.0], [0.0, 0.0, 1.0, -900.0]])
    # frame 1, view 1: camera 300 mm from the cuboid centre looking along +x
    R = np.array([[0.0, 1.0, 0.0], [0.0, 0.0, -1.0], [1.0, 0.0, 0.0]])
    centre = np.array([-250.0, -30.0, 900.0])
    K = np.array([[30.0, 0.0, 11.5], [0.0, 30.0, 8.5], [0.0, 0.0, 1.0]])
    proj[1, 1] = K @ np.hstack([R, (-R @ centre).reshape(3, 1)])
    feat = rng.standard_normal((B, N, C, H, W)).astype(np.float32)
    conf = rng.uniform(0.05, 1.0, size=(B, N, C)).astype(np.float32)
    return feat, proj.astype(np.float32), coords, conf


def golden_softargmax2d(op):
    """integrate_tensor_2d (op.py:11-47): small non-square maps, softmax / relu, the
    caller's heatmap_multiplier (triangulation.py:164), gradients; and a config-shaped
    slice (4 views x 17 joints of 96^2 blob heatmaps)."""
    rng = np.random.default_rng(21)
    hm = (rng.standard_normal((2, 5, 17, 23)) * 3.0).astype(np.float32)
    sa = {}
    for softmax in (True, False):
        for mult in (1.0, 1.7):
            h = torch.from_numpy(hm).requires_grad_(True)
            xy, maps = op.integrate_tensor_2d(h * mult, softmax)
            key = f"sm{int(softmax)}_m{mult}"
            sa[f"xy_{key}"] = xy.detach().numpy()
            sa[f"maps_{key}"] = maps.detach().numpy()
            gxy = torch.from_numpy(rng.standard_normal(xy.shape).astype(np.float32))
            gm = torch.from_numpy((rng.standard_normal(maps.shape) * 1e-2).astype(np.float32))
            torch.autograd.backward([xy, maps], [gxy, gm])
            sa[f"grad_xy_{key}"] = gxy.numpy()
            sa[f"grad_maps_{key}"] = gm.numpy()
            sa[f"grad_in_{key}"] = h.grad.numpy()
    # config-shaped: (B*N, J, 96, 96) Gaussian blobs at random centres
    H = W = 96
    yy, xx = np.mgrid[0:H, 0:W]
    cx, cy = rng.uniform(5, W - 5, (4, 17)), rng.uniform(5, H - 5, (4, 17))
    blob = np.exp(-((xx - cx[..., None, None]) ** 2 + (yy - cy[..., None, None]) ** 2) / (2 * 2.0 ** 2))
    cfg = (blob * 10.0).astype(np.float32)
    xy, _ = op.integrate_tensor_2d(torch.from_numpy(cfg) * 1.0, True)
    save("softargmax2d.npz", hm=hm, cfg=cfg, cfg_xy=xy.numpy(), **sa)


def golden_coord_volumes():
    """Coordinate volumes of triangulation.py:280-341.  The grid/centring is the loop's
    own ATen op sequence (restated in oracle/restate_torch.py: that code is inline in the
    model's forward, not a function); the rotation is the reference's own
    volumetric.rotate_coord_volume (volumetric.py:103-114), called here."""
    from mvn.utils import volumetric  # noqa: WPS433 (reference, imported above)
    sys.path.insert(0, REPO)
    from oracle import restate_torch
    rng = np.random.default_rng(33)
    base = np.stack([rng.uniform(-500, 500, 3) + np.array([0, 0, 900.0]) for _ in range(3)])
    cases = {"coco_eval": ("coco", [0.0, 0.0, 0.0], False), "coco_train": ("coco", [1.234, 4.5, 0.3], False),
             "mpii_cmu": ("mpii", [0.7, 2.2, 5.9], True)}
    out = {"base": base}
    for name, (kind, thetas, cmu) in cases.items():
        cv = restate_torch.build_coord_volumes(base, 2500.0, 16, thetas, kind, cmu, rotate=volumetric.rotate_coord_volume)
        out[f"cv_{name}"] = cv.numpy()
        out[f"theta_{name}"] = np.asarray(thetas)
    save("coord_volumes.npz", **out)


def golden_ce_loss():
    """VolumetricCELoss (loss.py:52-80): loss value and d loss / d volumes, which is
    non-zero exactly at the reference's argmin voxels (so it pins them)."""
    from mvn.models.loss import VolumetricCELoss  # noqa: WPS433 (reference)
    vb = synth.volumetric_batch(2, n_views=4, channels=1, volume=16, seed=17)
    rng = np.random.default_rng(17)
    kps = (vb.coords.reshape(2, -1, 3)[:, rng.integers(0, 16 ** 3, 17)].numpy()
           + rng.normal(0, 30.0, (2, 17, 3))).astype(np.float32)
    logits = torch.from_numpy(rng.standard_normal((2, 17, 16 ** 3)).astype(np.float32) * 3)
    vol = torch.softmax(logits, dim=2).reshape(2, 17, 16, 16, 16).contiguous().requires_grad_(True)
    validity = (rng.uniform(size=(2, 17, 1)) > 0.2).astype(np.float32)
    loss = VolumetricCELoss()(vb.coords, vol, torch.from_numpy(kps), torch.from_numpy(validity))
    loss.backward()
    save("ce_loss.npz", coords=vb.coords.numpy(), vol=vol.detach().numpy(), kps=kps, validity=validity,
         loss=loss.detach().numpy(), grad_vol=vol.grad.numpy())


def golden_v2v_front():
    """V2VModel.front_layers[0] = Basic3DBlock(32, 16, 7) (v2v.py:7-17) in eval mode with
    seeded parameters; conv weights and the input volume rounded to bf16 (the MFMA operand
    type), so the kernel and the reference differ only in f32 accumulation order."""
    from mvn.models.v2v import Basic3DBlock  # noqa: WPS433 (reference)
    g = torch.Generator().manual_seed(41)
    blk = Basic3DBlock(32, 16, 7).eval()
    with torch.no_grad():
        conv, bn = blk.block[0], blk.block[1]
        conv.weight.copy_((torch.randn(conv.weight.shape, generator=g) * 0.02).bfloat16().float())
        conv.bias.copy_(torch.randn(16, generator=g) * 0.1)
        bn.weight.copy_(torch.rand(16, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(16, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(16, generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(16, generator=g) + 0.5)
        x = torch.randn((2, 32, 16, 16, 16), generator=g).bfloat16().float()
        y = blk(x)
    save("v2v_front.npz", x=x.numpy(), weight=conv.weight.detach().numpy(), bias=conv.bias.detach().numpy(),
         bn_weight=bn.weight.detach().numpy(), bn_bias=bn.bias.detach().numpy(), bn_mean=bn.running_mean.numpy(),
         bn_var=bn.running_var.numpy(), eps=np.float64(bn.eps), y=y.numpy())


class _Cfg(dict):
    """dict with attribute access (the reference's configs are EasyDicts; easydict is absent)."""
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v


def _cfg(d):
    return _Cfg({k: _cfg(v) if isinstance(v, dict) else v for k, v in d.items()})


class _FixedBackbone(torch.nn.Module):
    """Stands in for PoseResNet: returns fixed (heatmaps, features, alg_conf, vol_conf)."""

    def __init__(self, outs):
        super().__init__()
        self.outs = outs

    def forward(self, images):
        return self.outs


class _ChannelSlice(torch.nn.Module):
    """Stands in for V2VModel(32, 17): channels [0:17] of the unprojected volume (the bench's
    V2V stand-in); keeps its input so the unprojection is pinned too."""

    def forward(self, v):
        self.last_input = v.detach().clone()
        return v[:, :17]


def golden_chains():
    """End-to-end caller chains of the two models (last row), run through the
    reference's own forward() with the backbone replaced by fixed outputs:
      * AlgebraicTriangulationNet.forward (triangulation.py:149-200): integrate_tensor_2d of
        heatmaps * 100 -> confidence normalisation -> upscale to image px -> DLT; also a
        float64 re-run of the same forward (solver precision only);
      * VolumetricTriangulationNet.forward (triangulation.py:245-355), training mode (random
        cuboid rotation, seeded), kind 'mpii', softmax aggregation: camera resize ->
        projections, coordinate volumes, process_features (a 1x1 conv set to pass channels
        0..31 through exactly), unproject, V2V replaced by the channel slice [0:17],
        soft-argmax with volume_multiplier."""
    from copy import deepcopy
    from mvn.models.triangulation import AlgebraicTriangulationNet, VolumetricTriangulationNet  # noqa: WPS433
    from mvn.utils.multiview import Camera  # noqa: WPS433
    bb = dict(name="resnet18", style="simple", init_weights=False, checkpoint="", num_joints=17, num_layers=18)
    B, N, J = 2, 4, 17
    out = {}

    # --- algebraic: blob heatmaps at the projected joints (+ noise), GAP-head confidences
    ab = synth.algebraic_batch(B, N, J, seed=40, noise_px=0.0)
    rng = np.random.default_rng(40)
    Hm = 96
    uv = ab.points.numpy() / (384 / Hm) + rng.normal(0, 0.7, (B, N, J, 2))
    yy, xx = np.mgrid[0:Hm, 0:Hm]
    d2 = (xx - uv[..., 0, None, None]) ** 2 + (yy - uv[..., 1, None, None]) ** 2
    # float16-representable values (stored as float16: the fixture stays small, exact in f32)
    hm = (np.exp(-d2 / (2 * 2.0 ** 2)) + 0.02 * rng.standard_normal(d2.shape)).astype(np.float16).astype(np.float32)
    conf = rng.uniform(0.2, 1.0, (B * N, J)).astype(np.float32)
    cfg = _cfg(dict(model=dict(use_confidences=True, heatmap_softmax=True, heatmap_multiplier=100.0, backbone=bb)))
    net = AlgebraicTriangulationNet(cfg, device="cpu").eval()
    images = torch.zeros((B, N, 3, 384, 384))
    for prec, dt in (("", torch.float32), ("64", torch.float64)):
        net.backbone = _FixedBackbone((torch.from_numpy(hm).reshape(B * N, J, Hm, Hm).to(dt), None,
                                       torch.from_numpy(conf).to(dt), None))
        with torch.no_grad():
            kp3, kp2, _, confn = net(images, ab.proj.to(dt), None)
        out[f"alg_kp3d{prec}"] = kp3.numpy()
        out[f"alg_kp2d{prec}"] = kp2.numpy()
        out[f"alg_conf_norm{prec}"] = confn.numpy()
    out.update(alg_heatmaps=hm.reshape(B, N, J, Hm, Hm).astype(np.float16), alg_conf=conf.reshape(B, N, J), alg_proj=ab.proj.numpy(),
               alg_multiplier=np.float32(100.0))

    # --- volumetric
    V, Hv, side = 32, 32, 2500.0
    cfg = _cfg(dict(model=dict(kind="mpii", volume_aggregation_method="softmax", volume_softmax=True,
                               volume_multiplier=1.0, volume_size=V, cuboid_side=side, use_gt_pelvis=False,
                               heatmap_softmax=True, heatmap_multiplier=100.0, backbone=bb)))
    net = VolumetricTriangulationNet(cfg, device="cpu")
    net.train()                     # random cuboid rotation (triangulation.py:318-321), seeded below
    with torch.no_grad():
        w = torch.zeros_like(net.process_features[0].weight)
        w[torch.arange(32), torch.arange(32)] = 1.0            # pass channels 0..31 through
        net.process_features[0].weight.copy_(w)
        net.process_features[0].bias.zero_()
    net.volume_net = _ChannelSlice()
    feat32 = rng.standard_normal((B, N, 32, Hv, Hv)).astype(np.float32)
    feats = np.zeros((B * N, 256, Hv, Hv), np.float32)
    feats[:, :32] = feat32.reshape(B * N, 32, Hv, Hv)
    net.backbone = _FixedBackbone((torch.zeros((B * N, J, Hv, Hv)), torch.from_numpy(feats), None, None))
    cams = [[None] * B for _ in range(N)]
    for b in range(B):
        for v, c in enumerate(synth.ring_cameras(N, np.random.default_rng([41, b]))):
            cams[v][b] = Camera(c.R, c.t, c.K)
    pred = (np.array([0.0, 0.0, 900.0]) + rng.uniform(-300, 300, (B, J, 3)))
    batch = {"cameras": cams, "pred_keypoints_3d": pred}
    np.random.seed(42)
    thetas = np.array([np.random.uniform(0.0, 2 * np.pi) for _ in range(B)])
    np.random.seed(42)
    with torch.no_grad():
        kp3, _, vols, _, _, cv, base = net(torch.zeros((B, N, 3, 384, 384)), None, batch)
    new = deepcopy(cams)
    for v in range(N):
        for b in range(B):
            new[v][b].update_after_resize((384, 384), (Hv, Hv))
    P = np.stack([np.stack([new[v][b].projection for v in range(N)]) for b in range(B)]).astype(np.float32)
    sub = (slice(None), slice(None), slice(None, None, 4), slice(None, None, 4), slice(None, None, 4))
    out.update(vol_features=feat32, vol_proj=P, vol_base=pred[:, 6], vol_thetas=thetas, vol_side=np.float64(side),
               vol_coords=cv.numpy(), vol_kp3d=kp3.numpy(), vol_volumes_sub=vols.numpy()[sub],
               vol_unprojected_sub=net.volume_net.last_input.numpy()[sub], vol_base_points=base.numpy())
    save("chains.npz", **out)


def golden_dlt_degenerate(multiview):
    """Degenerate DLT inputs (SURVEY.md §5 failure row): a joint with all-zero confidences
    (A = 0) and cameras whose projection ignores z (third column of every P zero, so A has an
    exactly zero column and X[3] = 0).  The outputs are whatever the reference's torch.svd
    (LAPACK) returns on THIS host: zeros for A = 0; (nan, nan, +-inf) for the zero column here,
    while another host's LAPACK may return a non-exact null vector (finite values)."""
    rng = np.random.default_rng(0)
    P = torch.from_numpy(rng.normal(size=(2, 4, 3, 4)).astype(np.float32))
    pts = torch.from_numpy(rng.normal(size=(2, 4, 3, 2)).astype(np.float32))
    conf = torch.from_numpy(rng.uniform(0.2, 1, (2, 4, 3)).astype(np.float32))
    conf[0, :, 1] = 0.0
    conf[1, :, 2] = 0.0
    out_zero_conf = multiview.triangulate_batch_of_points(P, pts, conf)
    P2 = P.clone()
    P2[:, :, :, 2] = 0.0
    out_zero_col = multiview.triangulate_batch_of_points(P2, pts, None)
    save("dlt_degenerate.npz", proj=P.numpy(), points=pts.numpy(), conf=conf.numpy(), proj_zero_col=P2.numpy(),
         out_zero_conf=out_zero_conf.numpy(), out_zero_col=out_zero_col.numpy())


def golden_unproject_backward_elementwise(op):
    """The reference's own autograd gradient of unproject_heatmaps (op.py:99-163: ATen's
    grid_sampler_2d / softmax backward on THIS host) for the element-wise backward parity
    test: the upstream gradients span 1e-12 ... 1e8 (frame 1 x 1e8, frame 0 channel 2 x
    1e-12).  Captured here, with the forward goldens, because ATen's CPU backward is not the
    same function of its inputs on every host: on the GPU box's EPYC it recomputes the
    sampling coordinate with a different rounding (profiles/r20_bwd_host_probe_epyc.txt:
    9.3e-4 element-wise vs 2.9e-7 on this Xeon), so a gradient recomputed there is not the
    reference's."""
    vb = synth.volumetric_batch(2, n_views=4, channels=4, heatmap=32, volume=16, seed=8)
    res = {}
    gout = torch.rand((2, 4, 16, 16, 16), generator=torch.Generator().manual_seed(6))
    gout[1] *= 1e8
    gout[0, 2] *= 1e-12
    g_sm = torch.randn((2, 4, 16, 16, 16), generator=torch.Generator().manual_seed(7))
    g_sm[1] *= 1e8
    for method, feat_scale, g in (("sum", 1.0, gout), ("softmax", 20.0, g_sm)):
        f = (vb.features * feat_scale).clone().requires_grad_(True)
        op.unproject_heatmaps(f, vb.proj, vb.coords, method).backward(g)
        res[f"grad_out_{method}"] = g.numpy()
        res[f"grad_feat_{method}"] = f.grad.numpy()
    save("unproject_bwd_elementwise.npz", feat=vb.features.numpy(), proj=vb.proj.numpy(), coords=vb.coords.numpy(),
         **res)


def main():
    op, multiview = import_reference()
    if len(sys.argv) > 1 and sys.argv[1] == "bwd_elementwise":
        golden_unproject_backward_elementwise(op)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "v2v_front":
        golden_v2v_front()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "ce_loss":
        golden_ce_loss()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "softargmax2d":
        golden_softargmax2d(op)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "coord_volumes":
        golden_coord_volumes()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "dlt_degenerate":
        return golden_dlt_degenerate(import_reference()[1])
    if len(sys.argv) > 1 and sys.argv[1] == "chains":
        golden_chains()
        return
    torch.manual_seed(0)

    # --- unproject: small, every aggregation, both align_corners, f32 and bf16-rounded input
    feat, proj, coords, conf = small_unproject_inputs()
    out = {}
    grads = {}
    for method in ("sum", "max", "softmax", "conf"):
        for ac in (False, True):
            h = torch.from_numpy(feat).requires_grad_(True)
            c = torch.from_numpy(conf).requires_grad_(True)
            with grid_sample_align_corners(ac):
                vol = op.unproject_heatmaps(h, torch.from_numpy(proj), torch.from_numpy(coords), method,
                                            c if method == "conf" else None)
            key = f"{method}_ac{int(ac)}"
            out[key] = vol.detach().numpy()
            g = torch.from_numpy(np.random.default_rng(7).standard_normal(vol.shape).astype(np.float32))
            vol.backward(g)
            grads[f"grad_out_{key}"] = g.numpy()
            grads[f"grad_feat_{key}"] = h.grad.numpy()
            if method == "conf":
                grads[f"grad_conf_{key}"] = c.grad.numpy()
    fb = torch.from_numpy(feat).to(torch.bfloat16)
    for method in ("sum", "softmax"):
        vol = op.unproject_heatmaps(fb.float(), torch.from_numpy(proj), torch.from_numpy(coords), method)
        out[f"bf16in_{method}_ac0"] = vol.numpy()
    save("unproject_small.npz", feat=feat, feat_bf16_bits=bf16_bits(torch.from_numpy(feat)), proj=proj,
         coords=coords, conf=conf, **out, **grads)

    # --- unproject: config-shaped slice (4 views, 96^2, 8 channels, V=16, softmax + sum)
    vb = synth.volumetric_batch(1, n_views=4, channels=8, volume=16, seed=11)
    res = {}
    for method in ("softmax", "sum"):
        res[method] = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, method).numpy()
    save("unproject_cfg.npz", feat=vb.features.numpy(), proj=vb.proj.numpy(), coords=vb.coords.numpy(),
         **{f"{k}_ac0": v for k, v in res.items()})

    # --- soft-argmax: small non-cubic (softmax / relu, multiplier fused by the caller) + blob
    rng = np.random.default_rng(3)
    vol = (rng.standard_normal((2, 3, 8, 9, 10)) * 3.0).astype(np.float32)
    sa = {}
    for softmax in (True, False):
        for mult in (1.0, 1.7):
            v = torch.from_numpy(vol).requires_grad_(True)
            xyz, vols = op.integrate_tensor_3d_with_coordinates(v * mult, torch.from_numpy(coords), softmax=softmax)
            key = f"sm{int(softmax)}_m{mult}"
            sa[f"xyz_{key}"] = xyz.detach().numpy()
            sa[f"vol_{key}"] = vols.detach().numpy()
            gx = torch.from_numpy(rng.standard_normal(xyz.shape).astype(np.float32))
            gv = torch.from_numpy((rng.standard_normal(vols.shape) * 1e-2).astype(np.float32))
            torch.autograd.backward([xyz, vols], [gx, gv])
            sa[f"grad_xyz_{key}"] = gx.numpy()
            sa[f"grad_vol_{key}"] = gv.numpy()
            sa[f"grad_in_{key}"] = v.grad.numpy()
    save("softargmax_small.npz", vol=vol, coords=coords, **sa)

    vb = synth.volumetric_batch(1, n_views=4, channels=1, volume=16, seed=5)
    blob = synth.blob_volumes(vb.coords, n_joints=17, seed=5)
    xyz, vols = op.integrate_tensor_3d_with_coordinates(blob, vb.coords, softmax=True)
    save("softargmax_blob.npz", vol=blob.numpy(), coords=vb.coords.numpy(), xyz=xyz.numpy(), vol_out=vols.numpy())

    # --- DLT: config 1 (B=1, 4 views, 17 joints, confidences), None-confidence and 8-view cases
    dl = {}
    cases = {
        "cfg1": synth.algebraic_batch(1, 4, 17, seed=0),
        "b3n3": synth.algebraic_batch(3, 3, 5, seed=1),
        "n8": synth.algebraic_batch(2, 8, 17, seed=2),
    }
    for name, ab in cases.items():
        for use_conf in (True, False):
            conf_t = ab.confidences if use_conf else None
            P = ab.proj.clone()
            pts = ab.points.clone().requires_grad_(True)
            ct = conf_t.clone().requires_grad_(True) if use_conf else None
            X = multiview.triangulate_batch_of_points(P, pts, ct)
            key = f"{name}_c{int(use_conf)}"
            dl[f"out_{key}"] = X.detach().numpy()
            g = torch.from_numpy(np.random.default_rng(9).standard_normal(X.shape).astype(np.float32))
            X.backward(g)
            dl[f"grad_out_{key}"] = g.numpy()
            dl[f"grad_pts_{key}"] = pts.grad.numpy()
            if use_conf:
                dl[f"grad_conf_{key}"] = ct.grad.numpy()
            # float64 re-run of the same reference code (solver precision only)
            X64 = multiview.triangulate_batch_of_points(P.double(), ab.points.double(),
                                                        conf_t.double() if use_conf else None)
            dl[f"out64_{key}"] = X64.numpy()
        dl[f"proj_{name}"] = ab.proj.numpy()
        dl[f"points_{name}"] = ab.points.numpy()
        dl[f"conf_{name}"] = ab.confidences.numpy()
        dl[f"gt_{name}"] = ab.points_3d.numpy()
    save("dlt.npz", **dl)

    golden_softargmax2d(op)
    golden_coord_volumes()
    golden_ce_loss()
    golden_v2v_front()
    golden_chains()


if __name__ == "__main__":
    main()
