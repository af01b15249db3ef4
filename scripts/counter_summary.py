"""Summarise scripts/gpu_counters.sh passes into profiles/<tag>_pmc_<cfg>.json (per kernel phase, per dispatch).

HBM: hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (kB -> B). gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE = TCC_EA0_RDREQ x 64 B tallies each 128-B memory-side read at 64 B, half the bytes of a coalesced read —
doubled here; WRITE_SIZE is exact for coalesced stores; Infinity-Cache hits count as fetches.

SQ (one pass: 8 SQ + GRBM_GUI_ACTIVE). rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs, so the kernel's GPU-busy
cycles are GRBM_GUI_ACTIVE / 8. With 256 CUs = 1024 SIMDs:
* mfma_busy_pct  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)      (rocprof MfmaUtil, busy cycles)
* valu_busy_pct  = SQ_ACTIVE_INST_VALU * 4 / (1024 * GRBM_GUI_ACTIVE / 8)        (SQ_ACTIVE_INST_* count quad-cycles)
* mfma_f32_flop  = SQ_INSTS_VALU_MFMA_MOPS_F32 * 512                            (rocprof MfmaFlopsF32)
* coexec_pct     = SQ_VALU_MFMA_COEXEC_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)
The summary is stamped with the sha256 of the kernel sources the passes measured (bench.kernel_source_hash, taken on
the GPU box), which bench.py checks before it reports `traffic`.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PHASES = {"Fc1Prob": "fc1", "GiProb": "gi", "gru_fwd": "gru_fwd", "Fc2Prob": "fc2", "HypProb": "hyper",
          "hyper_ws_kernel": "hyper", "hyper_kernel": "hyper", "mix_kernel": "mix", "mix_fast_kernel": "mix",
          "gru_bwd": "gru_bwd", "Dx1Prob": "dx1", "Dw1Prob": "dw1", "DwhProb": "dwh", "dwh_kernel": "dwh", "dwh_red1": "dwh",
          "red_pass": "reduce", "apply_kernel": "apply", "coma_l1": "coma_l1", "coma_head": "coma_head",
          "coma_wgrad": "coma_wgrad", "coma_chain": "coma_chain"}
SIMDS = 1024
XCDS = 8


def phase_of(name):
    for k, v in PHASES.items():
        if k in name:
            return v
    return None


def load(path_glob):
    """{phase: {counter: mean per dispatch}} (counter rows are per dispatch; several rows of one counter in one
    dispatch are summed first)."""
    per = defaultdict(lambda: defaultdict(float))
    ph_of = {}
    for path in glob.glob(path_glob, recursive=True):
        if not path.endswith("counter_collection.csv"):
            continue
        for r in csv.DictReader(open(path)):
            ph = phase_of(r["Kernel_Name"])
            if not ph:
                continue
            key = (path, r["Dispatch_Id"])
            ph_of[key] = ph
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    acc = defaultdict(lambda: defaultdict(list))
    for key, cnt in per.items():
        for c, v in cnt.items():
            acc[ph_of[key]][c].append(v)
    return {ph: {c: sum(v) / len(v) for c, v in d.items()} for ph, d in acc.items()}


def main(tag, cfg, root="gpurun_out"):
    f = load(f"{root}/pmc_{tag}_{cfg}_FETCH_SIZE/**/*.csv")
    w = load(f"{root}/pmc_{tag}_{cfg}_WRITE_SIZE/**/*.csv")
    sq = load(f"{root}/pmc_{tag}_{cfg}_SQ/**/*.csv")
    hpath = f"{root}/src_hash_{tag}_{cfg}.txt"
    out = {"source_sha256": open(hpath).read().strip() if os.path.exists(hpath) else None, "tag": tag,
           "formulas": __doc__.split("\n\n", 1)[1], cfg: {}}
    for ph in sorted(set(f) | set(w) | set(sq)):
        fb = f.get(ph, {}).get("FETCH_SIZE", 0.0)
        wb = w.get(ph, {}).get("WRITE_SIZE", 0.0)
        d = {"FETCH_SIZE_kB": fb, "WRITE_SIZE_kB": wb, "hbm_bytes_per_launch": (2.0 * fb + wb) * 1024.0}
        s = sq.get(ph)
        if s and s.get("GRBM_GUI_ACTIVE"):
            busy = s["GRBM_GUI_ACTIVE"] / XCDS
            d.update({k: s.get(k) for k in sorted(s)})
            d["gpu_busy_cycles"] = busy
            d["mfma_busy_pct"] = 100.0 * s.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (SIMDS * busy)
            d["valu_busy_pct"] = 100.0 * 4.0 * s.get("SQ_ACTIVE_INST_VALU", 0.0) / (SIMDS * busy)
            d["coexec_pct"] = 100.0 * s.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0.0) / (SIMDS * busy)
            d["mfma_f32_flop"] = 512.0 * s.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)
        out[cfg][ph] = d
    os.makedirs("profiles", exist_ok=True)
    path = f"profiles/{tag}_pmc_{cfg}.json"
    json.dump(out, open(path, "w"), indent=1)
    for ph, d in out[cfg].items():
        print(f"{ph:10s} hbm {d['hbm_bytes_per_launch'] / 1e6:8.2f} MB  mfma_busy {d.get('mfma_busy_pct', 0):6.2f}%"
              f"  valu_busy {d.get('valu_busy_pct', 0):6.2f}%  coexec {d.get('coexec_pct', 0):6.2f}%")
    print(path)


if __name__ == "__main__":
    main(*sys.argv[1:3])
