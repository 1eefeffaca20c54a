"""Aggregate a conv_table breakdown (tools/conv_table.py output) by op and
kernel size: ms per step and achieved TFLOP/s."""
import collections, re, sys
tot, fl = collections.Counter(), collections.Counter()
for l in open(sys.argv[1]):
    m = re.match(r"(conv2d_[\d+]+)\s+(\w+)\s+(\d)x(\d)/(\d).*grid=\s*\S+\s+([\d.]+)\+\s*([\d.]+)us\s+([\d.]+) TF/s", l)
    if not m:
        continue
    op = 'dgrad' if m.group(2).startswith('dg') else m.group(2)
    key = (op, '1x1' if int(m.group(3)) * int(m.group(4)) == 1 else 'kxk')
    t = float(m.group(6)) + float(m.group(7))
    tot[key] += t
    fl[key] += t * float(m.group(8))
for k in sorted(tot):
    print(f"{k[0]:6s} {k[1]}  {tot[k] / 1e3:7.3f} ms  {fl[k] / tot[k]:6.1f} TF/s")
print(f"total  {sum(tot.values()) / 1e3:7.3f} ms")
