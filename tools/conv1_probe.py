"""conv2d_1 forward + fused BN statistics at 299^2 B=64 (the first layer:
c_in 3 stored 4 fp32 / 8 bf16 wide, 3x3 stride 2 valid, 32 out), timed with
HIP events over back-to-back calls: the pinned GEMM tile vs the direct VALU
kernel (JR_CONV1_DIRECT is read once per process: run twice).
python tools/conv1_probe.py [x8|bf16] [cfg]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "x8"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else -1
_ffi.init(0)
L = _ffi.load()
code = _ffi.JR_F32_X8 if dt == "x8" else _ffi.JR_BF16
q, et = (4, torch.float32) if dt == "x8" else (8, torch.bfloat16)
n, h, ho = 64, 299, 149
d = _ffi.ConvDesc(n, h, h, 3, 32, 3, 3, 2, 2, 0, 0, ho, ho, 0, q, 0, 32)
if cfg >= 0:
    _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, code, 0, cfg))
x = torch.rand(n * h * h * q, device="cuda").to(et)
w = (torch.randn(32 * 9 * 8 if dt == "bf16" else 27 * 32, device="cuda") * 0.2).to(et)
y = torch.zeros(n * ho * ho * 32, device="cuda", dtype=et)
st = torch.zeros(64, device="cuda")
wsb = 8 * L.jr_conv2d_workspace_size(ctypes.byref(d), 0, code)   # (forced split-K factors need more)
ws = torch.zeros(wsb // 4 + 64, device="cuda")


def run():
    _ffi.check("fwd", L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), code, x.data_ptr(), w.data_ptr(), y.data_ptr(), 1e-3,
                                               st.data_ptr(), st.data_ptr() + 128, ws.data_ptr(), wsb, None))


for _ in range(5):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 50
mb = (x.numel() * x.element_size() + y.numel() * y.element_size()) / 1e6
print(f"{dt} cfg {L.jr_conv2d_get_config(ctypes.byref(d), 0, code, 0)} direct={os.environ.get('JR_CONV1_DIRECT', '1')}: "
      f"{us:.1f} us per conv + statistics ({mb:.0f} MB moved: {mb / us:.2f} TB/s)")
