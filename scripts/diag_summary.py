"""Per-kernel means of a scripts/gpu_diag.sh pass: cycles per wave split into waiting / issue-stalled / active,
LDS instructions and bank-conflict cycles, MFMA / VALU busy against the kernel's GPU-busy cycles."""
import csv
import glob
import sys
from collections import defaultdict

per = defaultdict(lambda: defaultdict(float))
name_of = {}
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        key = (path, r["Dispatch_Id"])
        name_of[key] = r["Kernel_Name"].split("(")[0][:60]
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
acc = defaultdict(lambda: defaultdict(list))
for key, cnt in per.items():
    for c, v in cnt.items():
        acc[name_of[key]][c].append(v)
for name, d in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    busy = m.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024 or 1
    wc = m.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{name}: n={len(next(iter(d.values())))} wave_cycles={wc:.3g} wait={m.get('SQ_WAIT_ANY', 0) / wc:.2f} "
          f"stall={m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} active={m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
          f"lds_insts={m.get('SQ_INSTS_LDS', 0):.3g} lds_conf={m.get('SQ_LDS_BANK_CONFLICT', 0):.3g} "
          f"mfma_busy={m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / busy:.3f} valu_busy={4 * m.get('SQ_ACTIVE_INST_VALU', 0) / busy:.3f}")
