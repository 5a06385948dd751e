"""Vendor-library reference points for the encoder's shapes on this GPU (not product code):
torch.nn.functional.linear (hipBLASLt) for the four encoder GEMMs and scaled_dot_product_attention
for the encoder attention, timed with HIP events.  Prints one JSON line per op."""
import json

import torch
import torch.nn.functional as F


def tm(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it  # us


import sys

dev = "cuda"
if "--parakeet" in sys.argv:
    # Parakeet-V3 encoder GEMMs in f16 at the C5 streaming pass (64 x 13 frames) and offline (8 x 375)
    for M in (832, 3000):
        for name, N, K in [("ff1", 4096, 1024), ("qkv", 3072, 1024), ("pw1", 2048, 1024), ("out", 1024, 1024),
                           ("ff2", 1024, 4096)]:
            a = torch.randn(M, K, device=dev, dtype=torch.float16)
            w = torch.randn(N, K, device=dev, dtype=torch.float16)
            b = torch.randn(N, device=dev, dtype=torch.float16)
            us = tm(lambda: F.linear(a, w, b))
            fl = 2.0 * M * N * K
            print(json.dumps({"op": f"hipblaslt_linear_pk_{name}", "M": M, "N": N, "K": K, "us": round(us, 2),
                              "TFLOP/s": round(fl / us / 1e6, 1), "frac_of_2500": round(fl / us / 1e6 / 2500, 3)}),
                  flush=True)
    sys.exit(0)
M, d = 8 * 1500, 1280
for name, N, K in [("qkv", 3 * d, d), ("out", d, d), ("fc1", 4 * d, d), ("fc2", d, 4 * d), ("cross_kv", 64 * d, d)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    us = tm(lambda: F.linear(a, w, b))
    fl = 2.0 * M * N * K
    print(json.dumps({"op": f"hipblaslt_linear_{name}", "M": M, "N": N, "K": K, "us": round(us, 2),
                      "TFLOP/s": round(fl / us / 1e6, 1), "frac_of_2500": round(fl / us / 1e6 / 2500, 3)}), flush=True)
q = torch.randn(8, 20, 1500, 64, device=dev, dtype=torch.bfloat16)
k = torch.randn_like(q)
v = torch.randn_like(q)
us = tm(lambda: F.scaled_dot_product_attention(q, k, v))
fl = 4.0 * 8 * 20 * 1500 * 1500 * 64
print(json.dumps({"op": "torch_sdpa_encoder_attention", "shape": [8, 20, 1500, 64], "us": round(us, 2),
                  "TFLOP/s": round(fl / us / 1e6, 1), "frac_of_2500": round(fl / us / 1e6 / 2500, 3)}), flush=True)
# the residual projections as the encoder needs them: bf16 operands, f32 residual C = D (beta = 1)
# and bias, through hipBLASLt's mixed-precision path (torch.addmm(..., out_dtype=float32))
for name, N, K in [("out_resid_f32", d, d), ("fc2_resid_f32", d, 4 * d)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    x = torch.randn(M, N, device=dev, dtype=torch.float32)
    b = torch.randn(N, device=dev, dtype=torch.float32)
    try:
        us = tm(lambda: x.copy_(torch.addmm(x, a, w.t(), out_dtype=torch.float32)).add_(b))
        fl = 2.0 * M * N * K
        print(json.dumps({"op": f"hipblaslt_addmm_{name}", "M": M, "N": N, "K": K, "us": round(us, 2),
                          "TFLOP/s": round(fl / us / 1e6, 1), "note": "includes a copy-back and a bias add"}), flush=True)
    except Exception as e:  # noqa: BLE001 -- a missing mixed-precision solution is a result too
        print(json.dumps({"op": f"hipblaslt_addmm_{name}", "error": str(e)[:200]}), flush=True)
