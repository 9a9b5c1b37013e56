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
