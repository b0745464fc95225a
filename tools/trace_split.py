"""Per-kernel, per-grid-size average durations from a rocprofv3 kernel trace:
python tools/trace_split.py gpurun_out/fr_trace/run_kernel_trace.csv [name-filter]"""
import collections
import csv
import sys

d = collections.defaultdict(list)
flt = sys.argv[2] if len(sys.argv) > 2 else "xdrg::"
for r in csv.DictReader(open(sys.argv[1])):
    if flt not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("xdrg::", "")
    d[(k, int(r["Grid_Size_X"]) if "Grid_Size_X" in r else int(r.get("Grid_Size", 0)))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, g), v in sorted(d.items()):
    print(f"{k:40s} grid {g:>10d} n {len(v):4d} avg {sum(v) / len(v):9.1f} us  min {min(v):9.1f}")
