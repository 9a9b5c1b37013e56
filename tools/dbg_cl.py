"""Debug aid (r14): bitwise comparison of the config-5-sized unprojection (bf16, 1 frame) between
two builds of libmvn_hip.so, repeat-launch determinism of each, and channels-last vs NCDHW.
    python tools/dbg_cl.py libA.so [libB.so]   (default: the in-tree library twice)"""
import ctypes, os, sys
sys.path.insert(0, "learnable-triangulation-pytorch_amd")
import torch
from mvn_rocm import _lib, synth
LIBS = (sys.argv[1:] + ["learnable-triangulation-pytorch_amd/mvn_rocm/libmvn_hip.so"] * 2)[:2]
dev = torch.device("cuda:0")
vb = synth.volumetric_batch(1, dtype=torch.bfloat16, device=dev, seed=55)
res = {}
for path in LIBS:
    lib = ctypes.CDLL(os.path.abspath(path))
    for n in ("mvn_unproject_ex", "mvn_unproject"):
        if n in _lib.SIGNATURES:
            r_, a_ = _lib.SIGNATURES[n]; getattr(lib, n).restype, getattr(lib, n).argtypes = r_, a_
    st = torch.cuda.current_stream().cuda_stream
    nc = torch.empty((1, 32, 64, 64, 64), dtype=torch.bfloat16, device=dev)
    r = lib.mvn_unproject(vb.features.data_ptr(), 1, vb.proj.data_ptr(), vb.coords.data_ptr(), None, nc.data_ptr(), 1, 1, 4, 32, 96, 96, 64, 64, 64, 2, 0, st)
    assert r == 0
    torch.cuda.synchronize()
    res[path] = nc.clone()
a, b = list(res.values())
d = (a != b)
print("NCDHW differs:", int(d.sum()), "of", d.numel())
if d.any():
    idx = d.nonzero()
    print("channels:", torch.unique(idx[:, 1]).tolist()[:40])
    print("first:", idx[:10].tolist())
    print("a", a[d][:10].float().tolist()); print("b", b[d][:10].float().tolist())
# determinism of the current build, and channels-last vs NCDHW for each build
for path in LIBS:
    lib = ctypes.CDLL(os.path.abspath(path))
    for n in ("mvn_unproject_ex", "mvn_unproject"):
        r_, a_ = _lib.SIGNATURES[n]; getattr(lib, n).restype, getattr(lib, n).argtypes = r_, a_
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for k in range(3):
        nc = torch.empty((1, 32, 64, 64, 64), dtype=torch.bfloat16, device=dev)
        assert lib.mvn_unproject(vb.features.data_ptr(), 1, vb.proj.data_ptr(), vb.coords.data_ptr(), None, nc.data_ptr(), 1, 1, 4, 32, 96, 96, 64, 64, 64, 2, 0, st) == 0
        outs.append(nc)
    cls = []
    for k in range(3):
        cl = torch.empty((1, 64, 64, 64, 32), dtype=torch.bfloat16, device=dev)
        assert lib.mvn_unproject_ex(vb.features.data_ptr(), 1, vb.proj.data_ptr(), vb.coords.data_ptr(), None, cl.data_ptr(), 1, 1, 1, 4, 32, 96, 96, 64, 64, 64, 2, 0, st) == 0
        cls.append(cl)
    torch.cuda.synchronize()
    print(path, "NCDHW repeat-equal:", all(torch.equal(outs[0], o) for o in outs), "CL repeat-equal:", all(torch.equal(cls[0], o) for o in cls))
    p = outs[0].permute(0, 2, 3, 4, 1).contiguous()
    d = p != cls[0]
    print("  CL vs NCDHW differ:", int(d.sum()))
    if d.any():
        idx = d.nonzero()
        print("  channels:", torch.unique(idx[:, 4]).tolist(), "x:", torch.unique(idx[:, 1]).tolist()[:20])
