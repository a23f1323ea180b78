"""Print the kernel timeline of the last full step in a rocprofv3 kernel trace (between the last two
launches of a marker kernel) - usage: ktimeline.py TRACE.csv [MARKER] [MAX_LINES]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "k_count_types"
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 80
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = (idx[-2], idx[-1]) if len(idx) >= 2 else (0, len(rows))
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b][:lim]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {r["Grid_Size_X"]:>8} {r["Workgroup_Size_X"]:>5} '
          f'{r["LDS_Block_Size"]:>6} {r["VGPR_Count"]:>4} {r["Kernel_Name"][:80]}')
print("step span us", (int(rows[b - 1]["End_Timestamp"]) - t0) / 1e3)
