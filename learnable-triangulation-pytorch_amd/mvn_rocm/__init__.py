"""mvn_rocm — MI355X-native volumetric / algebraic triangulation hot path.

Drop-in replacements for the three hot-path functions of learnable-triangulation-pytorch:

    mvn_rocm.op.unproject_heatmaps                    <- mvn/utils/op.py:99-163
    mvn_rocm.op.integrate_tensor_3d_with_coordinates  <- mvn/utils/op.py:84-96
    mvn_rocm.multiview.triangulate_batch_of_points    <- mvn/utils/multiview.py:162-174
    mvn_rocm.op.integrate_tensor_2d                   <- mvn/utils/op.py:11-47 (algebraic path)

backed by hand-written gfx950 HIP kernels in libmvn_hip.so (C ABI: include/mvn_hip.h).
``install()`` rebinds them inside an importable ``mvn`` package so that
VolumetricTriangulationNet / AlgebraicTriangulationNet call them unchanged.
"""
from __future__ import annotations

from . import _lib
from . import op, multiview

__all__ = ["op", "multiview", "install", "library_path", "set_unproject_precision"]

library_path = _lib.LIB_PATH
set_unproject_precision = op.set_unproject_precision


def install(mvn_op=None, mvn_multiview=None):
    """Rebind the reference's hot-path functions to the HIP implementations.

    The reference calls them by attribute lookup on the modules
    (``from mvn.utils import op, multiview`` in mvn/models/triangulation.py:11), so
    replacing the module attributes is a true drop-in.  Returns the previous bindings.
    """
    if mvn_op is None or mvn_multiview is None:
        import importlib
        mvn_op = mvn_op or importlib.import_module("mvn.utils.op")
        mvn_multiview = mvn_multiview or importlib.import_module("mvn.utils.multiview")
    _lib.load()   # fail loudly now, not at the first forward
    previous = {
        "unproject_heatmaps": mvn_op.unproject_heatmaps,
        "integrate_tensor_3d_with_coordinates": mvn_op.integrate_tensor_3d_with_coordinates,
        "triangulate_batch_of_points": mvn_multiview.triangulate_batch_of_points,
        "integrate_tensor_2d": mvn_op.integrate_tensor_2d,
    }
    mvn_op.unproject_heatmaps = op.unproject_heatmaps
    mvn_op.integrate_tensor_3d_with_coordinates = op.integrate_tensor_3d_with_coordinates
    mvn_multiview.triangulate_batch_of_points = multiview.triangulate_batch_of_points
    mvn_op.integrate_tensor_2d = op.integrate_tensor_2d
    return previous
