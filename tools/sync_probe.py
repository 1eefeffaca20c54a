"""Cost of HIP stream synchronisation on the GPU (run under rocprofv3
--kernel-trace; tools/sync_probe_gaps.py prints the gaps per segment).
Segments (each between two tagging fill kernels, 40 elementwise kernels):
  a  plain back-to-back on one stream
  b  + a torch event (hipEventDisableTiming) recorded after each
  c  ping-pong between two streams through torch events
  d  + a wait on a long-complete torch event before each
  e  + an event created DisableTiming | DisableSystemFence recorded after each
  f  ping-pong through DisableSystemFence events
  g  + hipStreamWriteValue32 after each
  h  ping-pong through hipStreamWriteValue32 / hipStreamWaitValue32
"""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
hip.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint]
hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]


def nev(flags):
    e = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), flags) == 0
    return e


N = 8 << 20
x = torch.ones(N, device="cuda")
y = torch.ones(N, device="cuda")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
A, B = ctypes.c_void_p(sa.cuda_stream), ctypes.c_void_p(sb.cuda_stream)
tev = [torch.cuda.Event() for _ in range(64)]
fev = [nev(0x2 | 0x20000000) for _ in range(64)]
flag = torch.zeros(64, dtype=torch.int32, device="cuda")
R = 40


def mark():
    with torch.cuda.stream(sa):
        torch.empty(1000, device="cuda").fill_(0)


def pingpong(rec, wait):
    for i in range(R):
        s, t = (sa, x) if i % 2 == 0 else (sb, y)
        if i:
            wait(s, i - 1)
        with torch.cuda.stream(s):
            t.mul_(1.0)
        rec(s, i)


for rep in range(2):
    torch.cuda.synchronize()
    mark()
    with torch.cuda.stream(sa):
        for _ in range(R):
            x.mul_(1.0)
    mark()
    with torch.cuda.stream(sa):
        for i in range(R):
            x.mul_(1.0)
            tev[i % 64].record(sa)
    mark()
    torch.cuda.synchronize()
    pingpong(lambda s, i: tev[i % 64].record(s), lambda s, i: s.wait_event(tev[i % 64]))
    torch.cuda.synchronize()
    mark()
    tev[0].record(sb)
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        for i in range(R):
            sa.wait_event(tev[0])
            x.mul_(1.0)
    mark()
    with torch.cuda.stream(sa):
        for i in range(R):
            x.mul_(1.0)
            hip.hipEventRecord(fev[i % 64], A)
    mark()
    torch.cuda.synchronize()
    pingpong(lambda s, i: hip.hipEventRecord(fev[i % 64], ctypes.c_void_p(s.cuda_stream)),
             lambda s, i: hip.hipStreamWaitEvent(ctypes.c_void_p(s.cuda_stream), fev[i % 64], 0))
    torch.cuda.synchronize()
    mark()
    flag.zero_()
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        for i in range(R):
            x.mul_(1.0)
            hip.hipStreamWriteValue32(A, ctypes.c_void_p(flag.data_ptr() + 4 * (i % 64)), rep * 1000 + i + 1, 0)
    mark()
    torch.cuda.synchronize()
    flag.zero_()
    torch.cuda.synchronize()
    pingpong(lambda s, i: hip.hipStreamWriteValue32(ctypes.c_void_p(s.cuda_stream),
                                                    ctypes.c_void_p(flag.data_ptr() + 4 * (i % 64)), 7, 0),
             lambda s, i: hip.hipStreamWaitValue32(ctypes.c_void_p(s.cuda_stream),
                                                   ctypes.c_void_p(flag.data_ptr() + 4 * (i % 64)), 7, 0, 0xffffffff))
    torch.cuda.synchronize()
    mark()
    torch.cuda.synchronize()
print("done")
