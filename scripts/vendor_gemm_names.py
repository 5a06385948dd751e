"""Run the encoder's GEMM shapes (B = 8 large-v3: M = 12000) through torch.matmul (hipBLASLt) so a
rocprofv3 kernel trace names the vendor kernels (macro tile, MFMA shape, depth) this build is
measured against.  usage (GPU box): rocprofv3 --kernel-trace --stats -d gpurun_out/vn -- python3 scripts/vendor_gemm_names.py"""
import torch

M = 12000
shapes = {"qkv": (1280, 3840), "fc1": (1280, 5120), "fc2": (5120, 1280), "out": (1280, 1280)}
for name, (K, N) in shapes.items():
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(20):
        c = a @ w.t()
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1000 / 20
    print(f"{name} {M}x{N}x{K}: {us:.1f} us = {2 * M * N * K / us / 1e6:.0f} TF/s", flush=True)
