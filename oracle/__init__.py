"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference hot path (learnable-triangulation-pytorch,
mvn/utils/op.py:84-163 and mvn/utils/multiview.py:132-174), used exclusively as the
checker by tests/, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
bench.py.  Nothing in the product package (learnable-triangulation-pytorch_amd/)
imports this package.

    oracle.capi          ctypes wrapper of the plain-C restatement (mvn_oracle.c)
    oracle.restate_torch op-for-op torch-CPU restatement (same ATen calls, same B x N /
                         B x J Python loops) — bit-exact with the reference, and the
                         timed CPU baseline on the GPU box
    oracle.restate_np    float64 numpy restatement of the DLT (LAPACK SVD)

Pinning: every restatement is checked against tests/golden/*.npz, vectors captured by
importing the reference itself in the build container (tests/golden/make_golden.py).
"""
