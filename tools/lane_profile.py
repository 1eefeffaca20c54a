"""Where a two-lane training step spends its wall time, from a rocprofv3
kernel trace: every instant of the last `steps` steps is classified by how
many kernels run (0 = gap, 1 = alone, 2+ = overlapped) and the time a
kernel runs ALONE is charged to its family -- the serial part of the step,
which is what shortening a kernel buys back.

python tools/lane_profile.py <run_kernel_trace.csv> [steps] [top]
"""
import csv
import re
import sys
from collections import defaultdict


def family(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"(?:jr::)?(\w+)(<[^,>]*)?", n)
    if not m:
        return n[:40]
    base = m.group(1)
    if base in ("k_conv", "k_conv_bf16", "k_conv_halo"):
        op = (m.group(2) or "<?").lstrip("<")
        return f"{base}<{ {'0': 'fwd', '1': 'dgrad', '2': 'wgrad'}.get(op, op)}>"
    return base


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if "k_nesterov" in r[2]]
    if len(opt) < nsteps + 1:
        sys.exit(f"need {nsteps + 1} optimizer launches, found {len(opt)}")
    t0, t1 = rows[opt[-nsteps - 1]][1], rows[opt[-1]][1]
    win = [r for r in rows[opt[-nsteps - 1] + 1:opt[-1] + 1]]
    ev = []
    for k, (s, e, n) in enumerate(win):
        ev.append((max(s, t0), 1, k))
        ev.append((min(e, t1), -1, k))
    ev.sort()
    running = set()
    last = t0
    alone = defaultdict(float)
    over = defaultdict(float)
    gap = both = single = 0.0
    for t, d, k in ev:
        dt = t - last
        if dt > 0:
            if not running:
                gap += dt
            elif len(running) == 1:
                single += dt
                alone[family(win[next(iter(running))][2])] += dt
            else:
                both += dt
                for j in running:
                    over[family(win[j][2])] += dt / len(running)
        last = t
        if d > 0:
            running.add(k)
        else:
            running.discard(k)
    if t1 > last and not running:
        gap += t1 - last
    wall = (t1 - t0) / nsteps / 1e3
    print(f"wall {wall:.3f} us/step over {nsteps} steps: one kernel running {single / nsteps / 1e3:.1f} us, "
          f"2+ overlapped {both / nsteps / 1e3:.1f} us, nothing {gap / nsteps / 1e3:.1f} us")
    print(f"{'family':34s} {'alone us/step':>14s} {'overlapped (shared) us/step':>28s}")
    for fam in sorted(set(alone) | set(over), key=lambda f: -(alone.get(f, 0) + over.get(f, 0)))[:top]:
        print(f"{fam:34s} {alone.get(fam, 0) / nsteps / 1e3:14.1f} {over.get(fam, 0) / nsteps / 1e3:28.1f}")


if __name__ == "__main__":
    main()
