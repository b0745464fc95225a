"""Summarise tools/sq_counters.sh's two rocprofv3 --pmc passes: per xdrg
kernel (name + grid), the per-dispatch mean of every SQ counter (rocprofv3
reports them summed over the chip), plus derived figures: VALU wave
instructions per CU, their issue time at 2.4 GHz, LDS conflict cycles per LDS
instruction, the fraction of wave cycles spent waiting.

  python tools/sq_summary.py gpurun_out/sq_TAG > summary.json"""
import csv
import glob
import json
import os
import statistics
import sys


def load(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "xdrg::" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("xdrg::", "")
            key = f"{name} grid={r['Grid_Size']}"
            out.setdefault(key, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return out


def main(root):
    merged = {}
    for p in ("p1", "p2"):
        for k, cs in load(os.path.join(root, p)).items():
            for c, vals in cs.items():
                merged.setdefault(k, {})[c] = statistics.mean(vals)
    for k, c in merged.items():
        if "SQ_INSTS_VALU" in c:
            c["valu_wave_instr_per_cu"] = round(c["SQ_INSTS_VALU"] / 256)
            # (a wave64 VALU instruction holds its 16-lane SIMD 4 cycles: one per CU per cycle)
            c["valu_issue_ms_at_2.4GHz"] = round(c["SQ_INSTS_VALU"] / 256 / 2.4e6, 3)
        if c.get("SQ_INSTS_LDS"):
            c["lds_conflict_cycles_per_lds_instr"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"], 3)
        if c.get("SQ_WAVE_CYCLES"):
            c["wait_fraction"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
    json.dump({"source": f"rocprofv3 --pmc, two passes ({root}); per-dispatch means summed over the chip",
               "kernels": merged}, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
