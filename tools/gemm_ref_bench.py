"""Known-good reference for the conv GEMM shapes: hipBLASLt (torch.mm, bf16
in, fp32 accumulate) on the implicit-GEMM dimensions of representative
Inception-v3 layers at B = 64, timed with HIP events on random operands.
Diagnostic only (methodology rule: a ceiling comes from a known-good kernel
on the same box, never from our own attempts).
  python tools/gemm_ref_bench.py"""
import torch

SHAPES = {  # name: (M, N, K)  fwd M = B*Ho*Wo, N = c_out, K = kh*kw*c_in
    "conv5 fwd 73^2 3x3 80->192": (322624, 192, 720),
    "conv5 wgrad": (720, 192, 322624),
    "conv3 fwd 147^2 3x3 32->64": (1382976, 64, 288),
    "35^2 3x3 64->96 fwd": (78400, 96, 576),
    "35^2 1x1 288->176 fwd": (78400, 176, 288),
    "17^2 1x1 768->512 fwd": (18496, 512, 768),
    "17^2 1x7 192->192 fwd": (18496, 192, 1344),
    "17^2 1x7 wgrad": (1344, 192, 18496),
    "8^2 1x1 2048->1152 fwd": (4096, 1152, 2048),
    "8^2 3x3 448->384 fwd": (4096, 384, 4032),
    "square 8192": (8192, 8192, 8192),
}


def main():
    torch.manual_seed(0)
    print(f"{'shape':32s} {'M':>8s} {'N':>6s} {'K':>7s} {'us':>9s} {'TF/s':>8s} {'frac':>6s}")
    for name, (M, N, K) in SHAPES.items():
        a = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(K, N, device="cuda", dtype=torch.bfloat16) * 2 - 1
        for _ in range(3):
            torch.mm(a, b)
        torch.cuda.synchronize()
        reps = 20 if M * N * K < 1e11 else 5
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                torch.mm(a, b)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / reps * 1e3)
        us = min(ts)
        tf = 2.0 * M * N * K / us / 1e6
        print(f"{name:32s} {M:8d} {N:6d} {K:7d} {us:9.1f} {tf:8.1f} {tf / 2500:6.3f}", flush=True)


if __name__ == "__main__":
    main()
