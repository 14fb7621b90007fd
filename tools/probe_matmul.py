"""Probe: does torch's fp32 GEMM with K=6 ([100,6] @ [6,P]) agree with an element-wise build?"""
import numpy as np
import torch

dev = torch.device("cuda", 0)
for P in (65536, 1 << 20, 2160 * 3840):
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.rand((6, P), generator=g, device=dev) * 100 - 50
    B = torch.rand((100, 6), generator=g, device=dev)
    I = B @ a
    J = torch.zeros_like(I)
    for j in range(6):
        J.add_(B[:, j:j + 1] * a[j:j + 1])
    ref = (B.double() @ a.double()).float()
    print(P, "gemm vs fp64:", float((I - ref).abs().max()), " elementwise vs fp64:", float((J - ref).abs().max()),
          flush=True)
