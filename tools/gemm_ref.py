#!/usr/bin/env python3
"""Library GEMM ceiling for the detector's conv shapes: times torch.mm (hipBLASLt) on
fp16 [M,K] x [K,N] with M = batch*oh*ow, N = cout, K = cin*k*k for each
yolov4-tiny@608 b64 conv that runs on conv_glds_f16, so the implicit-GEMM kernel
can be judged against what the vendor GEMM reaches on the same (M,N,K) with the
im2col matrix given for free.  python tools/gemm_ref.py"""
import torch

SHAPES = [("L6", 369664, 128, 576), ("L8", 92416, 256, 1152), ("L10", 23104, 512, 2304),
          ("L12", 23104, 1024, 4608), ("L13", 23104, 256, 1024), ("L14", 23104, 512, 2304),
          ("L21", 92416, 256, 3456), ("L28", 369664, 128, 2304)]
torch.manual_seed(0)
tot_us = 0.0
for name, m, n, k in SHAPES:
    a = torch.randn(m, k, device="cuda", dtype=torch.float16)
    b = torch.randn(k, n, device="cuda", dtype=torch.float16)
    for _ in range(3):
        torch.mm(a, b)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        torch.mm(a, b)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    tot_us += us
    print(f"{name}: M={m} N={n} K={k} {us:8.1f} us {2*m*n*k/us/1e6:8.1f} TFLOP/s", flush=True)
print(f"total {tot_us:.1f} us")
