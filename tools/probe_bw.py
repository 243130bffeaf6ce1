"""HBM streaming probes on this box (torch kernels): copy, a + b -> c, and a 3-read 1-write pattern at the trunk's
layer-1 tensor sizes, to calibrate what the HBM-bound passes can reach. usage: python tools/probe_bw.py"""
import torch

dev = "cuda"


def t(f, n=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


M, C = 3211264, 256
x = torch.randn(M, C, device=dev).to(torch.bfloat16)
y = torch.randn(M, C, device=dev).to(torch.bfloat16)
z = torch.empty_like(x)
a64 = torch.randn(M, 64, device=dev).to(torch.bfloat16)
nb = x.numel() * 2
us = t(lambda: z.copy_(x))
print(f"copy {nb / 1e9:.2f} GB: {us:8.1f} us  {2 * nb / us / 1e3:5.2f} TB/s (read + write)")
us = t(lambda: torch.add(x, y, out=z))
print(f"add  (2 reads + 1 write): {us:8.1f} us  {3 * nb / us / 1e3:5.2f} TB/s")
us = t(lambda: x.sum(dtype=torch.float32))
print(f"sum  (read only): {us:8.1f} us  {nb / us / 1e3:5.2f} TB/s")
xf = x.view(torch.int16)
us = t(lambda: torch.bitwise_or(xf, y.view(torch.int16), out=z.view(torch.int16)))
print(f"or   (2 reads + 1 write): {us:8.1f} us  {3 * nb / us / 1e3:5.2f} TB/s")
