"""install() rebinds the reference's hot-path module attributes (no GPU needed: only the
library load and the rebinding are exercised)."""
import types

from mvn_rocm import install, multiview, op


def test_install_rebinds_every_hot_path_function():
    ref_op = types.SimpleNamespace(unproject_heatmaps=object(), integrate_tensor_3d_with_coordinates=object(),
                                   integrate_tensor_2d=object())
    ref_mv = types.SimpleNamespace(triangulate_batch_of_points=object())
    before = dict(vars(ref_op), **vars(ref_mv))
    prev = install(ref_op, ref_mv)
    assert prev == before
    assert ref_op.unproject_heatmaps is op.unproject_heatmaps
    assert ref_op.integrate_tensor_3d_with_coordinates is op.integrate_tensor_3d_with_coordinates
    assert ref_op.integrate_tensor_2d is op.integrate_tensor_2d
    assert ref_mv.triangulate_batch_of_points is multiview.triangulate_batch_of_points


REF = "/root/reference"


def test_install_on_the_real_reference_modules():
    """install() on the reference's own modules (build container only: /root/reference is
    imported read-only with an empty cv2 module, as tests/golden/make_golden.py does).  After
    install(), the names mvn/models/triangulation.py resolves at its call sites
    (op.unproject_heatmaps :349, op.integrate_tensor_3d_with_coordinates :353,
    op.integrate_tensor_2d :164, multiview.triangulate_batch_of_points :188) are mvn_rocm's.
    Run in a subprocess so the reference never enters this test process's modules."""
    import os
    import subprocess
    import sys
    import pytest
    if not os.path.isdir(os.path.join(REF, "mvn")):
        pytest.skip("the reference is not present (GPU box)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys, types
sys.dont_write_bytecode = True
sys.modules.setdefault("cv2", types.ModuleType("cv2"))
sys.path.insert(0, {REF!r})
sys.path.insert(0, {os.path.join(root, "learnable-triangulation-pytorch_amd")!r})
from mvn.models import triangulation as T
import mvn_rocm
from mvn_rocm import op, multiview
prev = mvn_rocm.install()
assert T.op.unproject_heatmaps is op.unproject_heatmaps
assert T.op.integrate_tensor_3d_with_coordinates is op.integrate_tensor_3d_with_coordinates
assert T.op.integrate_tensor_2d is op.integrate_tensor_2d
assert T.multiview.triangulate_batch_of_points is multiview.triangulate_batch_of_points
assert prev["unproject_heatmaps"].__module__ == "mvn.utils.op"
assert prev["triangulate_batch_of_points"].__module__ == "mvn.utils.multiview"
print("ok")
"""
    r = subprocess.run([sys.executable, "-B", "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]
