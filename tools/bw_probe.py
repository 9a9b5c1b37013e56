"""Achievable HBM bandwidth on this box for the hot path's access shapes (torch kernels):
read-only (sum), write-only (fill), copy, at the config-3 sizes (537 MB volume)."""
import torch


def t(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


dev = torch.device("cuda:0")
n = 32 * 32 * 64 ** 3                    # config 3 unprojection output, bf16: 537 MB
x = torch.randn(n, device=dev).to(torch.bfloat16)
y = torch.empty_like(x)
for name, fn, nbytes in (("write (fill_) 537 MB", lambda: y.fill_(1.0), 2 * n),
                         ("read (sum) 537 MB", lambda: x.sum(dtype=torch.float32), 2 * n),
                         ("copy 537 MB -> 537 MB", lambda: y.copy_(x), 4 * n)):
    sec = t(fn)
    print(f"{name:26s} {sec * 1e6:8.1f} us  {nbytes / sec / 1e12:5.2f} TB/s", flush=True)
