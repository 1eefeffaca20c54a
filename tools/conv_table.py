"""Map the conv GEMM dispatches of the last training step in a rocprofv3
kernel trace to (launch, op) of the engine's plan (jr.plan: fused sibling
groups included) and print per-call achieved TFLOP/s, then a whole-step
kernel-family breakdown.
  python tools/conv_table.py trace.csv [B] [top] [split_top] [stats.csv] [nsteps] [res] [--unfused]"""
import csv, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
from jr.inception import build_inception_v3
from jr.plan import build_plan

args = [a for a in sys.argv[1:] if not a.startswith("--")]
trace = args[0]
B = int(args[1]) if len(args) > 1 else 64
res = int(args[6]) if len(args) > 6 else 299
sys.argv = [sys.argv[0]] + args
rows = [r for r in csv.DictReader(open(trace)) if r["Kind"] == "KERNEL_DISPATCH"]
# host issue order (Dispatch_Id), not start time: with several lanes the GPU
# starts kernels of different streams out of issue order, and matching by start
# time mislabels the launches of parallel branches (round-3 tables before r03e)
rows.sort(key=lambda r: int(r["Dispatch_Id"]) if r.get("Dispatch_Id") else int(r["Start_Timestamp"]))
g = build_inception_v3(res, res)
plan = build_plan(g, "--unfused" not in sys.argv[0:] and "--unfused" not in os.environ.get("CONV_TABLE", ""))


def phases(u):
    s, k = u.stride, []
    for py in range(s):
        for px in range(s):
            hc = (u.h - py + s - 1) // s if py < u.h else 0
            wc = (u.w - px + s - 1) // s if px < u.w else 0
            r0, c0 = (py + u.pad_h) % s, (px + u.pad_w) % s
            na = (u.kh - r0 + s - 1) // s if r0 < u.kh else 0
            nb = (u.kw - c0 + s - 1) // s if c0 < u.kw else 0
            if hc and wc:
                k.append((f"dg{py * s + px}" if s > 1 else "dgrad", 2 * B * hc * wc * u.cin * na * nb * u.cout))
    return k


# plan order: the forward GEMMs, then per unit in reverse its backward group
# (filter gradient + data-gradient phases, in whatever order the engine issues
# them: matched below by the OP template argument of the kernel name)
groups = [[(u, "fwd", 2 * u.macs_per_image() * B)] for u in plan.units]
for u in reversed(plan.units):
    grp = [(u, "wgrad", 2 * u.macs_per_image() * B)]
    if u.x != g.input_buf:
        grp += [(u, op, f) for op, f in phases(u)]
    groups.append(grp)
seq = [e for grp in groups for e in grp]


def op_of(name):
    """0 fwd / 1 dgrad / 2 wgrad from the kernel name (halo kernels: fwd)."""
    if "k_conv_halo<" in name:
        return 0
    a = name[name.index("<") + 1:]
    return int(a.split(",")[0].split(">")[0].strip())

opt = [i for i, r in enumerate(rows) if "k_nesterov" in r["Kernel_Name"] or "k_sgd" in r["Kernel_Name"]]
step_rows = rows[opt[-2] + 1:opt[-1] + 1] if len(opt) >= 2 else rows
FAMILY = ("k_splitk_reduce", "k_stats_finalize")
conv = []
i = 0
while i < len(step_rows):
    r = step_rows[i]
    nm = r["Kernel_Name"]
    if ("k_conv<" in nm or "k_conv_bf16<" in nm or "k_conv_halo<" in nm):
        t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        t2 = 0
        j = i + 1
        while j < len(step_rows) and any(f in step_rows[j]["Kernel_Name"] for f in FAMILY):
            t2 += int(step_rows[j]["End_Timestamp"]) - int(step_rows[j]["Start_Timestamp"])
            j += 1
        conv.append((r, t, t2))
        i = j
        continue
    i += 1
if len(conv) != len(seq):
    print(f"warning: {len(conv)} conv GEMMs in the step, plan expects {len(seq)}", file=sys.stderr)
last = conv[-len(seq):]
# within each backward group, give the filter gradient the OP=2 launch and
# the data-gradient phases the OP=1 launches in issue order
aligned, k = [], 0
for grp in groups:
    ks = last[k:k + len(grp)]
    k += len(grp)
    w = [c for c in ks if op_of(c[0]["Kernel_Name"]) == 2]
    d = [c for c in ks if op_of(c[0]["Kernel_Name"]) == 1]
    f = [c for c in ks if op_of(c[0]["Kernel_Name"]) == 0]
    for (u, op, fl) in grp:
        src = f if op == "fwd" else w if op == "wgrad" else d
        if not src:
            print(f"warning: no OP match for {u.name} {op}", file=sys.stderr)
            src = [c for c in (f, w, d) if c][0]
        aligned.append(src.pop(0))
last = aligned
# per-call floor: max(flops at the dense bf16 MFMA peak, compulsory HBM bytes
# at 8 TB/s) -- bf16 kernels only (fp32 kernels: the x8 / fp32-MFMA peaks differ)
PEAK_TF, PEAK_GBS = 2500.0, 8000.0


def floor_us(u, op, f, name):
    if "bf16" not in name and "halo" not in name:
        return None
    e = 2   # bytes per bf16 element
    x = B * u.h * u.w * u.cin * e
    y = B * u.ho * u.wo * u.cout * e
    wt = u.kh * u.kw * u.cin * u.cout * e
    byts = {"fwd": x + y + wt, "wgrad": x + y + 2 * wt}.get(op, y + x + wt)   # dgrad phases: dy + dx + w
    if op.startswith("dg") and op != "dgrad":
        byts /= u.stride * u.stride
    return max(f / PEAK_TF / 1e6, byts / PEAK_GBS / 1e3)


tot_t = 0; tot_f = 0; tot_floor = 0.0
out = []
for (u, op, f), (r, t, t2) in zip(seq, last):
    tot_t += t + t2; tot_f += f
    name = r["Kernel_Name"]; cfg = name[name.index("<"):name.index(">") + 1]
    fl = floor_us(u, op, f, name)
    tot_floor += fl or 0.0
    ftxt = f"  floor {fl:6.1f}us ({fl * 1e3 / max(t + t2, 1):4.2f})" if fl is not None else ""
    out.append((t + t2, f"{u.name:14s} {op:5s} {u.kh}x{u.kw}/{u.stride} {u.h:3d}x{u.w:<3d} {u.cin:4d}->{u.cout:4d} "
                f"{cfg:24s} grid={r['Grid_Size_X']:>7s}x{r['Grid_Size_Z']:<4s} {t/1e3:8.1f}+{t2/1e3:6.1f}us {f/max(t+t2, 1)/1e3:7.1f} TF/s"
                + ftxt))
for t, s in sorted(out, reverse=True)[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(s)
print(f"total conv {tot_t/1e6:.2f} ms, {tot_f/max(tot_t, 1)/1e3:.1f} TF/s"
      + (f"; sum of per-call floors {tot_floor/1e3:.2f} ms ({tot_floor*1e3/max(tot_t, 1):.2f} of the time)"
         if tot_floor else ""))

# ---- whole-step breakdown: kernels between the last two optimizer launches
opt = [i for i, r in enumerate(rows) if "k_nesterov" in r["Kernel_Name"] or "k_sgd" in r["Kernel_Name"]]
if len(opt) >= 2:
    a, b = opt[-2] + 1, opt[-1] + 1
    step = rows[a:b]
    t0 = min(int(r["Start_Timestamp"]) for r in step); t1 = max(int(r["End_Timestamp"]) for r in step)
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
