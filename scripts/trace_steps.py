"""Print the last N kernels of a rocprofv3 kernel trace with durations and inter-kernel gaps (us)."""
import csv, re, sys

path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))[-n:]
t0, prev = int(rows[0]['Start_Timestamp']), None
for r in rows:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = re.sub(r'\(.*', '', r['Kernel_Name'])[-44:]
    print(f"{(s - t0) / 1e3:8.1f} dur {(e - s) / 1e3:7.1f} gap {((s - prev) / 1e3 if prev else 0):6.1f}  {name}"
          f"  grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} lds={r['LDS_Block_Size']}")
    prev = e
