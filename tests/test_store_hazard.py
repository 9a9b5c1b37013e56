"""tools/check_store_hazard.py (run by __graft_entry__.build() on libmvn_hip.so): it flags a
>8-byte VMEM store whose data VGPRs the next vector instruction overwrites, and passes the
padded form and unrelated registers.  CPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_store_hazard  # noqa: E402

BAD = """_Zk:
\tbuffer_store_dwordx4 v[4:7], v97, s[40:43], s8 offen
\tv_mov_b32_e32 v7, v3
\tglobal_store_dwordx4 v[2:3], v[8:11], off
\tv_add_f32_e32 v9, v1, v2
"""
GOOD = """_Zk:
\tbuffer_store_dwordx4 v[4:7], v97, s[40:43], s8 offen
\ts_nop 1
\tv_mov_b32_e32 v7, v3
\tbuffer_store_dwordx2 v[4:5], v97, s[40:43], s8 offen
\tv_mov_b32_e32 v5, v3
\tbuffer_store_dwordx4 v[4:7], v97, s[40:43], s8 offen
\tv_mov_b32_e32 v8, v3
"""


def test_flags_overwritten_store_data(tmp_path):
    p = tmp_path / "bad.s"
    p.write_text(BAD)
    assert check_store_hazard.check([str(p)]) == 2


def test_passes_padded_and_unrelated(tmp_path):
    p = tmp_path / "good.s"
    p.write_text(GOOD)
    assert check_store_hazard.check([str(p)]) == 0


def test_built_library_is_clean():
    lib = os.path.join(ROOT, "learnable-triangulation-pytorch_amd", "mvn_rocm", "libmvn_hip.so")
    if not (os.path.exists(lib) and os.path.exists(os.path.join(check_store_hazard.LLVM, "llvm-objdump"))):
        import pytest
        pytest.skip("library or llvm-objdump not present")
    assert check_store_hazard.check([lib]) == 0
