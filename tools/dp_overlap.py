"""Bucket / backward overlap of the data-parallel step from a rocprofv3
kernel trace (bench.py --dp on): per training step (delimited by the
optimizer kernel), every RCCL kernel's start and end relative to the END of
the step's last backward conv kernel (negative = the all-reduce ran while the
backward was still computing), and the gap between that conv and the
optimizer.
  python tools/dp_overlap.py run_kernel_trace.csv [nsteps]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kind"] == "KERNEL_DISPATCH"]
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
opt = [i for i, r in enumerate(rows) if "nesterov" in r["Kernel_Name"].lower()]
is_rccl = lambda n: "nccl" in n.lower() or "rccl" in n.lower()  # noqa: E731
is_conv = lambda n: "conv" in n.lower() or "wgrad_reduce" in n.lower()  # noqa: E731
print(f"{len(rows)} kernels, {len(opt)} optimizer launches, "
      f"{sum(1 for r in rows if is_rccl(r['Kernel_Name']))} RCCL kernels")
steps = list(zip(opt, opt[1:]))[-nlast:]
for a, b in steps:
    seg = rows[a + 1:b + 1]
    convs = [r for r in seg if is_conv(r["Kernel_Name"])]
    rccl = [r for r in seg if is_rccl(r["Kernel_Name"])]
    if not convs:
        continue
    t_end = max(int(r["End_Timestamp"]) for r in convs)
    t0 = int(seg[0]["Start_Timestamp"])
    t_opt = int(seg[-1]["Start_Timestamp"])
    print(f"step: {(t_opt - t0) / 1e3:.1f} us from first kernel to optimizer; last backward conv ends at "
          f"{(t_end - t0) / 1e3:.1f} us; optimizer starts {(t_opt - t_end) / 1e3:+.1f} us after it")
    for r in rccl:
        s, e = int(r["Start_Timestamp"]) - t_end, int(r["End_Timestamp"]) - t_end
        print(f"  {r['Kernel_Name'][:60]:60s} start {s / 1e3:+9.1f} us  end {e / 1e3:+9.1f} us "
              f"({'overlapped' if s < 0 else 'after backward'})")
