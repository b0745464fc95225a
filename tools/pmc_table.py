"""Per-kernel, per-grid counter averages from rocprofv3 --pmc runs:
python tools/pmc_table.py DIR [DIR ...] [--filter k_fr_]
(each DIR holds a run_counter_collection.csv; values are summed over the
dimensions of one dispatch, then averaged over dispatches of the same kernel
and grid size)."""
import collections
import csv
import glob
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = "xdrg::"
if "--filter" in sys.argv:
    flt = sys.argv[sys.argv.index("--filter") + 1]
    args.remove(flt)
per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, grid, dispatch) -> counter -> sum
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if flt not in k:
                continue
            name = k.split("(")[0].replace("void ", "").replace("xdrg::", "")
            g = int(r.get("Grid_Size", 0) or r.get("Grid_Size_X", 0))
            per[(name, g, d, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for (name, g, d, disp), cs in per.items():
    for c, v in cs.items():
        agg[(name, g)][c].append(v)
for (name, g), cs in sorted(agg.items()):
    print(f"{name} grid {g}")
    for c, v in sorted(cs.items()):
        print(f"    {c:24s} {sum(v) / len(v):16.0f}  (n {len(v)})")
