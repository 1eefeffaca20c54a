"""One BN backward launch set (jr_bn_relu_bwd: k_bn_reduce, k_bn_finalize*,
k_bn_relu_bwd_apply) per Inception-v3 BN shape at B=64, 299^2, after one
warm-up of each, for rocprofv3 --pmc passes (tools/bn_pmc.sh); the order of
the measured dispatches is SHAPES order (tools/bn_pmc_summary.py).
  python tools/bn_pmc_run.py [f32|bf16]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402

from jr import _ffi  # noqa: E402

from bnbench_shapes import SHAPES  # noqa: E402

_ffi.init(0)
L = _ffi.load()
DT = _ffi.JR_BF16 if len(sys.argv) > 1 and sys.argv[1] == "bf16" else _ffi.JR_F32
TD = torch.bfloat16 if DT == _ffi.JR_BF16 else torch.float32
B = 64
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
bufs = []
for h, c, _ in SHAPES:
    m = B * h * h
    t = dict(x=torch.randn(m * c, device="cuda").to(TD), dy=torch.randn(m * c, device="cuda").to(TD),
             mean=torch.randn(c, device="cuda") * 0.1, invstd=torch.rand(c, device="cuda") + 0.5,
             beta=torch.randn(c, device="cuda") * 0.1, dbeta=torch.empty(c, device="cuda"),
             ws=torch.empty(L.jr_bn_workspace_size(m, c), dtype=torch.uint8, device="cuda"))
    t["dx"] = torch.empty_like(t["x"])
    bufs.append((m, c, t))


def run(m, c, t):
    _ffi.check("jr_bn_relu_bwd", L.jr_bn_relu_bwd(DT, P(t["dy"]), 0, c, P(t["x"]), 0, c, m, c, P(t["mean"]),
                                                  P(t["invstd"]), P(t["beta"]), P(t["dx"]), P(t["dbeta"]),
                                                  P(t["ws"]), t["ws"].numel(), None))


for m, c, t in bufs:        # warm-up, then the measured pass (dispatch order = SHAPES order)
    run(m, c, t)
torch.cuda.synchronize()
for m, c, t in bufs:
    run(m, c, t)
torch.cuda.synchronize()
print("done", len(bufs), "shapes")
