"""Per-step kernel time by family from a rocprofv3 kernel trace.

python tools/kernel_families.py <run_kernel_trace.csv> [steps]

Over the last `steps` complete training steps (delimited by the optimizer
launch), sums kernel durations per family: the kernel name up to its first
template argument (so conv forward / data-grad / filter-grad, which differ
in the first argument OP = 0 / 1 / 2, stay apart), in ms per step, with the
launch count per step.
"""
import csv
import re
import sys
from collections import defaultdict


def family(name: str) -> str:
    m = re.search(r"jr::(\w+)(<[^,>]*)?", name)
    if not m:
        return name.split("(")[0][:48]
    return m.group(1) + (m.group(2) + ">" if m.group(2) else "")


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if "k_nesterov" in r[2]]
    # whole training steps only: bench.py's per-family rate replays after the
    # timed region also launch the optimizer alone, so keep the windows
    # between optimizer launches that hold conv kernels
    steps = [(a, b) for a, b in zip(opt, opt[1:])
             if any("k_conv" in rows[i][2] for i in range(a + 1, b))]
    if len(steps) < nsteps:
        sys.exit(f"need {nsteps} whole steps, found {len(steps)}")
    win = [r for a, b in steps[-nsteps:] for r in rows[a + 1:b + 1]]
    t = defaultdict(int)
    c = defaultdict(int)
    for s, e, n in win:
        k = family(n)
        t[k] += e - s
        c[k] += 1
    tot = sum(t.values())
    print(f"{'family':40s} {'ms/step':>9s} {'calls':>6s}")
    for k in sorted(t, key=lambda k: -t[k]):
        print(f"{k:40s} {t[k] / 1e6 / nsteps:9.3f} {c[k] / nsteps:6.1f}")
    print(f"{'total':40s} {tot / 1e6 / nsteps:9.3f} {len(win) / nsteps:6.1f}")


if __name__ == "__main__":
    main()
