"""List the kernels of the last complete training step of a rocprofv3 kernel
trace (between the last two optimizer launches), optionally filtered by name:
  python tools/kernel_calls.py trace.csv [substring] [limit]"""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if 'nesterov' in r['Kernel_Name']]
a, b = idx[-2], idx[-1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
k = 0
for r in rows[a + 1:b]:
    if pat in r['Kernel_Name']:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        print(f"{d:9.2f} us  grid={int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']):7d}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
              f" vgpr={r['VGPR_Count']} lds={r['LDS_Block_Size']}  {r['Kernel_Name'][:70]}")
        k += 1
        if k >= lim:
            break
