"""The op layer's eager bypass (mvn_rocm._ops.call) must not hide the custom ops from
tracers: under make_fx with fake tensors every drop-in function records its
torch.ops.mvn_rocm op (shape-only fake kernels; no GPU, no library call)."""
import torch
from torch.fx.experimental.proxy_tensor import make_fx


def _targets(gm):
    return {str(n.target) for n in gm.graph.nodes if n.op == "call_function"}


def test_make_fx_records_the_custom_ops():
    from mvn_rocm import multiview, op
    feat = torch.randn(2, 4, 8, 16, 16)
    proj = torch.randn(2, 4, 3, 4)
    coords = torch.randn(2, 8, 8, 8, 3)

    def path(feat, proj, coords):
        vol = op.unproject_heatmaps(feat, proj, coords, "softmax")
        xyz, sm = op.integrate_tensor_3d_with_coordinates(vol[:, :3], coords)
        return vol, xyz, sm

    gm = make_fx(path, tracing_mode="fake")(feat, proj, coords)
    t = _targets(gm)
    assert "mvn_rocm.unproject.default" in t and "mvn_rocm.softargmax3d.default" in t, t
    pts = torch.randn(2, 4, 5, 2)
    gm = make_fx(lambda p, x: multiview.triangulate_batch_of_points(p, x), tracing_mode="fake")(proj, pts)
    assert "mvn_rocm.dlt.default" in _targets(gm)
    hm = torch.randn(3, 5, 16, 16)
    gm = make_fx(lambda h: op.integrate_tensor_2d(h), tracing_mode="fake")(hm)
    assert "mvn_rocm.softargmax2d.default" in _targets(gm)


def test_eager_call_on_cpu_tensors_fails_loudly():
    """The bypass runs the op's own body, which refuses CPU tensors (no CPU fallback)."""
    import pytest
    from mvn_rocm import op
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        op.unproject_heatmaps(torch.randn(1, 4, 4, 8, 8), torch.randn(1, 4, 3, 4), torch.randn(1, 4, 4, 4, 3))


def test_tracers_and_transforms_route_through_the_dispatcher():
    """_ops.call takes the eager bypass only when nothing records or transforms the call:
    torch.jit.trace and functorch transforms (vmap) must see the registered ops."""
    from mvn_rocm import _ops
    seen = []

    def f(x):
        seen.append(_ops._tracing())
        return x + 1

    f(torch.randn(2))
    assert seen == [False]
    seen.clear()
    torch.jit.trace(f, torch.randn(2), check_trace=False)
    assert seen and all(seen), seen
    seen.clear()
    torch.func.vmap(f)(torch.randn(3, 2))
    assert seen == [True], seen
