"""Median counters per (kernel, grid size) over rocprofv3 --pmc output dirs:
python tools/pmc_grid.py 'k_fr_' gpurun_out/fr_sq1 gpurun_out/fr_sq2 ...
FETCH_SIZE is reported x2 (gfx950 tallies 128-B requests at 64 B), sizes in bytes."""
import collections
import csv
import statistics
import sys

flt = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[2:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if flt not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"].split("(")[0].replace("void ", "").replace("xdrg::", ""), int(r["Grid_Size"]))
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["_us"].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
for k, d in sorted(agg.items()):
    m = {c: statistics.median(v) for c, v in d.items()}
    if "FETCH_SIZE" in m:
        m["FETCH_SIZE"] *= 2048
    if "WRITE_SIZE" in m:
        m["WRITE_SIZE"] *= 1024
    print(k, {c: (round(v) if v > 100 else round(v, 2)) for c, v in sorted(m.items())})
