"""Per-step kernel spans and inter-kernel gaps from a rocprofv3 kernel trace (run_kernel_trace.csv).
Usage: python scripts/trace_gaps.py DIR [first-kernel-substring]"""
import csv, sys, statistics as st
d = sys.argv[1]; first = sys.argv[2] if len(sys.argv) > 2 else "gru_fwd"
rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"]]
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
gaps, spans = {}, []
for a, b in zip(starts[-12:-1], starts[-11:]):
    spans.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    for i in range(a, b):
        k = rows[i]["Kernel_Name"].split("(")[0][-40:]
        g = (int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3
        dur = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
        gaps.setdefault(k, []).append((dur, g))
print(f"  step span median {st.median(spans):.2f} us")
for k, v in gaps.items():
    print(f"  {k:40s} dur {st.median([x[0] for x in v]):7.2f}  gap after {st.median([x[1] for x in v]):5.2f}")
