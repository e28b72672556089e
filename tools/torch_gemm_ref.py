"""rocBLAS/hipBLASLt (torch.mm, fp32) timing at the block's GEMM shapes, for comparison."""
import torch
shapes = [("preconv", 5440, 512, 384), ("qkv", 12288, 288, 170), ("gtu7", 32640, 64, 224), ("dX7", 65280, 32, 448),
          ("dWp", 512, 384, 5440), ("sat_dW", 192, 512, 5440), ("big", 4096, 4096, 2048)]
torch.backends.cuda.matmul.allow_tf32 = False
for name, M, N, K in shapes:
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    for _ in range(5):
        torch.mm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 50
    for _ in range(n):
        torch.mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    print(f"{name:8s} {M}x{N}x{K}: {us:8.1f} us  {2 * M * N * K / us / 1e6:7.1f} TF/s")
