"""Diagnostic: time jr_bn_relu_bwd (reduce + finalize + apply) on the
Inception-v3 BN shapes (B=64, 299^2) for the libjr named by $JR_LIB.
Prints per-shape µs and the step total weighted by how many layers have
that shape.   python tools/bnbench.py [dtype f32|bf16]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402

from jr import _ffi  # noqa: E402

_ffi.init(0)
L = _ffi.load()
DT = _ffi.JR_BF16 if len(sys.argv) > 1 and sys.argv[1] == "bf16" else _ffi.JR_F32
TD = torch.bfloat16 if DT == _ffi.JR_BF16 else torch.float32
B = 64
# (h, c, layers with this BN shape) over the 94 conv2d_bn of App. A
SHAPES = [(149, 32, 1), (147, 32, 1), (147, 64, 1), (73, 80, 1), (71, 192, 1),
          (35, 64, 12), (35, 48, 2), (35, 96, 9), (35, 32, 1), (17, 384, 1), (17, 192, 18), (17, 128, 6),
          (17, 160, 12), (8, 320, 3), (8, 192, 3), (8, 384, 8), (8, 448, 2), (17, 96, 1)]
tot = tot_apply = 0.0
for h, c, cnt in SHAPES:
    m = B * h * h
    x = torch.randn(m * c, device="cuda").to(TD)
    dy = torch.randn(m * c, device="cuda").to(TD)
    dx = torch.empty_like(x)
    mean = torch.randn(c, device="cuda") * 0.1
    invstd = torch.rand(c, device="cuda") + 0.5
    beta = torch.randn(c, device="cuda") * 0.1
    dbeta = torch.empty(c, device="cuda")
    ws = torch.empty(L.jr_bn_workspace_size(m, c), dtype=torch.uint8, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run():
        _ffi.check("jr_bn_relu_bwd", L.jr_bn_relu_bwd(DT, P(dy), 0, c, P(x), 0, c, m, c, P(mean), P(invstd),
                                                      P(beta), P(dx), P(dbeta), P(ws), ws.numel(), None))
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    gbs = 3 * m * c * x.element_size() / us / 1e3     # algorithmic: read x, dy once; write dx

    def fwd():
        _ffi.check("jr_bn_relu_apply", L.jr_bn_relu_apply(DT, P(x), 0, c, m, c, P(mean), P(invstd), P(beta),
                                                          P(dx), 0, c, None))
    for _ in range(5):
        fwd()
    e0.record()
    for _ in range(n):
        fwd()
    e1.record()
    torch.cuda.synchronize()
    ua = e0.elapsed_time(e1) * 1e3 / n
    tot += us * cnt
    tot_apply += ua * cnt
    print(f"{h:4d}^2 x {c:4d}  x{cnt:2d}: bwd {us:8.1f} us  {gbs:7.0f} GB/s (3 passes) | apply {ua:7.1f} us "
          f"{2 * m * c * x.element_size() / ua / 1e3:7.0f} GB/s")
print(f"weighted total bwd {tot:.1f} us, apply {tot_apply:.1f} us  [{os.path.basename(_ffi.LIB_PATH)}]")
