"""Where a training step's idle GPU time sits, from a rocprofv3 kernel trace:
every interval of the last `steps` steps in which NO kernel runs, classified
by the kernel that closed the busy period before it and the one that opened
the next (same hardware queue = an in-order launch gap, other queue = a
cross-lane hand-off), with a duration histogram.

python tools/gap_profile.py <run_kernel_trace.csv> [steps] [top]
"""
import csv
import sys
from collections import defaultdict

from lane_profile import family


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"])))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if "k_nesterov" in r[2]]
    if len(opt) < nsteps + 1:
        sys.exit(f"need {nsteps + 1} optimizer launches, found {len(opt)}")
    win = rows[opt[-nsteps - 1] + 1:opt[-1] + 1]
    # busy periods: sweep in start order, tracking the latest end seen
    gaps = []   # (duration ns, prev kernel, next kernel)
    cur_end, cur_k = win[0][1], win[0]
    for k in win[1:]:
        if k[0] > cur_end:
            gaps.append((k[0] - cur_end, cur_k, k))
        if k[1] > cur_end:
            cur_end, cur_k = k[1], k
    total = sum(g[0] for g in gaps)
    wall = (win[-1][1] - win[0][0]) / nsteps
    print(f"wall {wall / 1e3:.1f} us/step; idle {total / nsteps / 1e3:.1f} us/step in {len(gaps) / nsteps:.0f} "
          f"intervals/step ({len(win) / nsteps:.0f} kernels/step, queues {sorted(set(r[3] for r in win))})")
    same = [g for g in gaps if g[1][3] == g[2][3]]
    cross = [g for g in gaps if g[1][3] != g[2][3]]
    for name, gs in (("same queue (in-order launch gap)", same), ("other queue (cross-lane hand-off)", cross)):
        t = sum(g[0] for g in gs)
        print(f"  {name:36s} {t / nsteps / 1e3:8.1f} us/step  {len(gs) / nsteps:5.0f}/step  "
              f"mean {t / max(len(gs), 1) / 1e3:6.2f} us")
    edges = [0, 1e3, 2e3, 5e3, 10e3, 20e3, 50e3, 1e12]
    print("  histogram (us): " + "  ".join(
        f"[{edges[i] / 1e3:g},{edges[i + 1] / 1e3:g}): {sum(1 for g in gaps if edges[i] <= g[0] < edges[i + 1]) / nsteps:.0f}"
        f" / {sum(g[0] for g in gaps if edges[i] <= g[0] < edges[i + 1]) / nsteps / 1e3:.0f}us"
        for i in range(len(edges) - 1)))
    pairs = defaultdict(lambda: [0.0, 0])
    for d, a, b in gaps:
        key = (family(a[2]), family(b[2]), "same" if a[3] == b[3] else "cross")
        pairs[key][0] += d
        pairs[key][1] += 1
    print(f"  {'before':28s} {'after':28s} {'queue':6s} {'us/step':>8s} {'n/step':>7s}")
    for (a, b, q), (d, n) in sorted(pairs.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"  {a:28s} {b:28s} {q:6s} {d / nsteps / 1e3:8.1f} {n / nsteps:7.1f}")


if __name__ == "__main__":
    main()
