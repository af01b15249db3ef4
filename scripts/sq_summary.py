"""Per-kernel averages of the SQ counters collected by scripts/gpu_sq.sh (counter_collection.csv)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
cols = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
        "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE"]
print(f"{'kernel':40s} " + " ".join(f"{c[3:13]:>11s}" for c in cols) + "  cyc/wave")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
    n = len(disp[k])
    print(f"{k:40s} " + " ".join(f"{v[c] / n:11.3g}" for c in cols) +
          f"  {4 * v['SQ_WAVE_CYCLES'] / max(v['SQ_WAVES'], 1):9.0f}")
