"""Gaps between consecutive kernels of tools/sync_probe.py segments (trace
CSV), per repetition: a b c d e f g h (see tools/sync_probe.py; argv[2]: the
segment letters of another probe, tools/probes/sync_probe2.hip: abcdefg)."""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"])))
rows.sort()
marks = [i for i, r in enumerate(rows) if "Fill" in r[2] or r[2].startswith("tag")]
segs = []
for k in range(len(marks) - 1):
    seg = [r for r in rows[marks[k] + 1:marks[k + 1]] if "Fill" not in r[2] and not r[2].startswith("tag")]
    if len(seg) >= 4:
        segs.append(seg)
names = sys.argv[2] if len(sys.argv) > 2 else "abcdefgh"
for k, seg in enumerate(segs):
    gaps = sorted(b[0] - a[1] for a, b in zip(seg, seg[1:]))
    dur = [r[1] - r[0] for r in seg]
    print(f"rep {k // len(names)} {names[k % len(names)]}: {len(seg)} kernels, queues {sorted(set(r[3] for r in seg))}, mean kernel "
          f"{sum(dur) / len(dur) / 1e3:.1f} us, gap median {gaps[len(gaps) // 2] / 1e3:.2f} mean "
          f"{sum(gaps) / len(gaps) / 1e3:.2f} us")
