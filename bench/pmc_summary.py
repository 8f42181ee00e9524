#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter CSVs per kernel (last dispatch of each kernel name).
Usage: pmc_summary.py <dir-with-pmc1/pmc2> [out.md]"""
import csv, glob, os, re, sys
sys.path.insert(0, os.path.dirname(__file__))
from prof_summary import short


def load(d):
    res = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"], r["Dispatch_Id"])
            res.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
            res[k]["_dur"] = float(r.get("End_Timestamp", 0)) - float(r.get("Start_Timestamp", 0)) if r.get("End_Timestamp") else 0
    return res


def main():
    d = sys.argv[1]
    per = {}
    for sub in ("pmc1", "pmc2"):
        for (name, disp), c in load(os.path.join(d, sub)).items():
            per.setdefault(short(name), {}).update({k: v for k, v in c.items()})
    cols = ["SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU",
            "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
            "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"]
    lines = ["| kernel | MFMA | VALU | LDS | VMEM rd | VALU/MFMA | wait_inst% | wait_any% | MFMA busy% | LDS bank-confl% | LDS active / GUI cycle |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    rows = []
    for k, c in per.items():
        if c.get("SQ_INSTS_MFMA", 0) + c.get("SQ_INSTS_VALU", 0) < 1e5:
            continue
        wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
        mf = c.get("SQ_INSTS_MFMA", 0)
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(c.get("GRBM_GUI_ACTIVE", 1) * 256 * 4 / 8, 1)
        rows.append((c.get("SQ_WAVE_CYCLES", 0), f"| `{k[:70]}` | {mf:.3g} | {c.get('SQ_INSTS_VALU',0):.3g} | "
                     f"{c.get('SQ_INSTS_LDS',0):.3g} | {c.get('SQ_INSTS_VMEM_RD',0):.3g} | "
                     f"{c.get('SQ_INSTS_VALU',0)/max(mf,1):.1f} | {100*c.get('SQ_WAIT_INST_ANY',0)/wc:.0f} | "
                     f"{100*c.get('SQ_WAIT_ANY',0)/wc:.0f} | {100*busy:.1f} | "
                     f"{100*c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_LDS_IDX_ACTIVE',1),1):.1f} | "
                     f"{c.get('SQ_LDS_IDX_ACTIVE',0)/max(c.get('GRBM_GUI_ACTIVE',1),1):.1f} |"))
    rows.sort(key=lambda r: -r[0])
    out = "\n".join(lines + [r[1] for r in rows])
    print(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(out + "\n")


if __name__ == "__main__":
    main()
