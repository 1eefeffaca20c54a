"""GPU occupancy of a training step from a rocprofv3 kernel trace.

python tools/busy_union.py <run_kernel_trace.csv> [steps]

Steps are delimited by the optimizer launch (k_nesterov); over the last
`steps` complete steps it prints the wall time per step, the union of the
kernel intervals (time at least one kernel runs), the sum of kernel
durations (> union when lanes overlap), and the idle gaps by size -- i.e.
whether the step is bound by kernel time or by serialisation / launch gaps.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if "k_nesterov" in r[2]]
    if len(opt) < nsteps + 1:
        sys.exit(f"need {nsteps + 1} optimizer launches, found {len(opt)}")
    lo, hi = opt[-nsteps - 1] + 1, opt[-1] + 1
    win = rows[lo:hi]
    t0, t1 = rows[opt[-nsteps - 1]][1], rows[opt[-1]][1]
    wall = t1 - t0
    busy = tot = 0
    cur_s, cur_e = None, None
    gaps = []
    for s, e, _ in win:
        tot += e - s
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            elif s > t0:
                gaps.append(s - t0)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    ms = lambda ns: ns / 1e6 / nsteps  # noqa: E731
    print(f"{nsteps} steps, {len(win) // nsteps} kernels/step")
    print(f"wall      {ms(wall):8.3f} ms/step")
    print(f"busy      {ms(busy):8.3f} ms/step (union of kernel intervals, {busy / wall:.3f} of wall)")
    print(f"sum       {ms(tot):8.3f} ms/step (kernel durations; overlap factor {tot / max(busy, 1):.3f})")
    print(f"idle      {ms(wall - busy):8.3f} ms/step in {len(gaps) // nsteps} gaps/step")
    for lo_us, hi_us in ((0, 1), (1, 2), (2, 5), (5, 20), (20, 1e9)):
        g = [x for x in gaps if lo_us * 1e3 <= x < hi_us * 1e3]
        print(f"  gaps {lo_us:>3}-{hi_us if hi_us < 1e9 else 'inf':>3} us: {len(g) / nsteps:7.1f}/step  {ms(sum(g)):7.3f} ms/step")


if __name__ == "__main__":
    main()
