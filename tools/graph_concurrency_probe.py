"""Probe: does a captured HIP graph run independent branches (forked
streams) concurrently on this ROCm?  Times N small kernels on 1 stream vs the
same kernels split over 2 / 4 forked streams, eager and graph-replayed."""
import time
import torch

dev = torch.device("cuda", 0)
N = 400
bufs = [torch.randn(64 * 1024, device=dev) for _ in range(4)]
big = [torch.randn(2048, 2048, device=dev) for _ in range(4)]


def work(k, i, kind):
    if kind == "small":
        bufs[k].mul_(1.0001)
    else:
        torch.mm(big[k], big[k], out=big[(k + 1) % 4] if False else None)


def run(nstreams, kind, main):
    streams = [main] + [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]
    for s in streams[1:]:
        s.wait_stream(main)
    for i in range(N):
        k = i % nstreams
        with torch.cuda.stream(streams[k]):
            work(k, i, kind)
    for s in streams[1:]:
        main.wait_stream(s)


for kind, n in (("small", N), ("mm", 64)):
    N = n
    for ns in (1, 2, 4):
        main = torch.cuda.Stream(dev)
        with torch.cuda.stream(main):
            run(ns, kind, main)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(main):
            for _ in range(5):
                run(ns, kind, main)
        torch.cuda.synchronize()
        te = (time.perf_counter() - t0) / 5
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main):
            run(ns, kind, main)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        tg = (time.perf_counter() - t0) / 5
        print(f"{kind:5s} kernels={N} streams={ns}: eager {te*1e3:7.2f} ms  graph {tg*1e3:7.2f} ms", flush=True)
