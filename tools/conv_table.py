"""Map k_conv_f32 dispatches of a rocprofv3 kernel trace to (layer, op) and
print per-call achieved TFLOP/s for the last training step in the trace."""
import csv, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
from jr.inception import build_inception_v3

trace = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
rows = [r for r in csv.DictReader(open(trace)) if r["Kind"] == "KERNEL_DISPATCH"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
g = build_inception_v3()
seq = [(n, "fwd") for n in g.convs]
for n in reversed(g.convs):
    seq.append((n, "wgrad"))
    if n.idx != 0:
        for ph in range(n.stride * n.stride):   # one GEMM per stride phase
            seq.append((n, "dgrad" if n.stride == 1 else f"dg{ph}"))
conv = []
i = 0
while i < len(rows):
    r = rows[i]
    if "k_conv" in r["Kernel_Name"] and "splitk" not in r["Kernel_Name"]:
        t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        j = i + 1
        if j < len(rows) and "splitk_reduce" in rows[j]["Kernel_Name"]:
            t2 = int(rows[j]["End_Timestamp"]) - int(rows[j]["Start_Timestamp"])
        else:
            t2 = 0
        conv.append((r, t, t2))
    i += 1
last = conv[-len(seq):]
tot_t = 0; tot_f = 0
out = []
for (n, op), (r, t, t2) in zip(seq, last):
    f = 2 * n.macs_per_image() * B / (n.stride * n.stride if op.startswith("dg") and op != "dgrad" else 1)
    tot_t += t + t2; tot_f += f
    name = r["Kernel_Name"]; cfg = name[name.index("<"):name.index(">") + 1]
    out.append((t + t2, f"{n.name:10s} {op:5s} {n.kh}x{n.kw}/{n.stride} {n.h:3d}x{n.w:<3d} {n.cin:4d}->{n.cout:4d} "
                f"{cfg:24s} grid={r['Grid_Size_X']:>7s}x{r['Grid_Size_Z']:<4s} {t/1e3:8.1f}+{t2/1e3:6.1f}us {f/(t+t2)/1e3:7.1f} TF/s"))
for t, s in sorted(out, reverse=True)[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(s)
print(f"total conv {tot_t/1e6:.2f} ms, {tot_f/tot_t/1e3:.1f} TF/s")

# ---- whole-step breakdown: kernels between the last two optimizer launches
opt = [i for i, r in enumerate(rows) if "k_nesterov" in r["Kernel_Name"] or "k_sgd" in r["Kernel_Name"]]
if len(opt) >= 2:
    a, b = opt[-2] + 1, opt[-1] + 1
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"]); t1 = int(step[-1]["End_Timestamp"])
    from collections import defaultdict
    cat = defaultdict(float)
    for r in step:
        n = r["Kernel_Name"]
        key = n.split("(")[0].replace("void ", "")
        key = key.split("<")[0]
        cat[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    busy = sum(cat.values())
    print(f"\nlast step: wall {(t1 - t0)/1e6:.2f} ms, kernel-busy {busy:.2f} ms, {len(step)} kernels")
    for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
        print(f"  {v:8.3f} ms  {k}")

# ---- split-K reduce launches of the last step, largest first
red = sorted(((t2, s) for (t, s), (_, _, t2) in zip(out, last) if t2 > 0), reverse=True)
print(f"\nsplit-K reduces: {len(red)} launches, {sum(t for t, _ in red)/1e6:.3f} ms")
for t2, s in red[:int(sys.argv[4]) if len(sys.argv) > 4 else 10]:
    print(f"  {t2/1e3:7.1f}us  {s[:60]}")

# ---- rocprofv3-style stats restricted to the last complete steps (the
# process-wide run_kernel_stats.csv also holds autotuning and warm-up calls)
if len(sys.argv) > 5 and len(opt) >= 2:
    nsteps = min(int(sys.argv[6]) if len(sys.argv) > 6 else 3, len(opt) - 1)
    a, b = opt[-1 - nsteps] + 1, opt[-1] + 1
    per = defaultdict(list)
    for r in rows[a:b]:
        per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in per.values())
    with open(sys.argv[5], "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "CallsPerStep"])
        for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), round(sum(v) / len(v), 1), round(100 * sum(v) / tot, 2), min(v), max(v),
                        round(len(v) / nsteps, 2)])
    print(f"\nwrote step-window stats over {nsteps} steps to {sys.argv[5]}")
