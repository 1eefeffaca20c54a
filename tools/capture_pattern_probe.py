"""Which cross-stream wait pattern crashes HIP graph capture (ROCm 7.2)?
Each pattern runs in a child process: tiny torch kernels on three streams
A (origin), B, C inside torch.cuda.graph, then one replay."""
import subprocess, sys
if len(sys.argv) > 1:
    import torch
    p = sys.argv[1]
    A = torch.cuda.Stream(); B = torch.cuda.Stream(); C = torch.cuda.Stream()
    x = [torch.zeros(1024, device="cuda") for _ in range(3)]
    def k(s, i):
        with torch.cuda.stream(s):
            x[i].add_(1)
    def wait(dst, src):
        e = torch.cuda.Event(); e.record(src); dst.wait_event(e)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=A):
        wait(B, A); wait(C, A)                  # fork
        k(C, 2)
        if p == "double":                       # C's node waited by A and by B
            wait(A, C); k(A, 0); wait(B, C); k(B, 1)
        elif p == "fresh":                      # B waits on a newer C node
            wait(A, C); k(A, 0); k(C, 2); wait(B, C); k(B, 1)
        elif p == "chain":                      # B waits on A (which waited on C)
            wait(A, C); k(A, 0); wait(B, A); k(B, 1)
        elif p == "double_nowork":              # double wait, A has no work after
            wait(A, C); wait(B, C); k(B, 1); k(A, 0)
        wait(A, B); wait(A, C)                  # join
    g.replay(); torch.cuda.synchronize()
    print(p, "ok", x[0][0].item(), x[1][0].item(), x[2][0].item())
    sys.exit(0)
for p in ("chain", "fresh", "double", "double_nowork"):
    r = subprocess.run([sys.executable, __file__, p], capture_output=True, text=True, timeout=120)
    print(p, "rc", r.returncode, r.stdout.strip()[-80:], flush=True)
