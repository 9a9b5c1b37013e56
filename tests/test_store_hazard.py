"""tools/check_store_hazard.py (run by __graft_entry__.build() on libmvn_hip.so): it flags a
>8-byte VMEM store whose data VGPRs a vector instruction overwrites within two wait states
(the next instruction, or the one after a single intervening instruction / `s_nop 0`), and
passes the padded form (`s_nop 1` = two wait states), writes three instructions later and
unrelated registers.  CPU only."""
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
ONE_GAP = """_Zk:
\tbuffer_store_dwordx4 v[4:7], v97, s[40:43], s8 offen
\tv_add_u32_e32 v20, v21, v22
\tv_mov_b32_e32 v6, v3
\tbuffer_store_dwordx3 v[8:10], v97, s[40:43], s8 offen
\ts_nop 0
\tv_mov_b32_e32 v10, v3
\tbuffer_store_dwordx4 v[12:15], v97, s[40:43], s8 offen
\ts_waitcnt lgkmcnt(0)
\tv_mov_b32_e32 v13, v3
"""
FAR = """_Zk:
\tbuffer_store_dwordx4 v[4:7], v97, s[40:43], s8 offen
\tv_add_u32_e32 v20, v21, v22
\ts_add_u32 s4, s4, 1
\tv_mov_b32_e32 v6, v3
\tbuffer_store_dwordx4 v[4:7], v97, s[40:43], s8 offen
\ts_nop 0
\ts_nop 0
\tv_mov_b32_e32 v6, v3
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


def test_flags_a_write_one_instruction_later(tmp_path):
    p = tmp_path / "gap.s"
    p.write_text(ONE_GAP)
    assert check_store_hazard.check([str(p)]) == 3


def test_passes_writes_after_two_wait_states(tmp_path):
    p = tmp_path / "far.s"
    p.write_text(FAR)
    assert check_store_hazard.check([str(p)]) == 0


def test_passes_padded_and_unrelated(tmp_path):
    p = tmp_path / "good.s"
    p.write_text(GOOD)
    assert check_store_hazard.check([str(p)]) == 0


def test_built_library_is_clean():
    lib = os.path.join(ROOT, "learnable-triangulation-pytorch_amd", "mvn_rocm", "libmvn_hip.so")
    assert os.path.exists(os.path.join(check_store_hazard.LLVM, "llvm-objdump")), "llvm-objdump missing"
    if not os.path.exists(lib):
        import pytest
        pytest.skip("library not built")
    assert check_store_hazard.check([lib]) == 0
