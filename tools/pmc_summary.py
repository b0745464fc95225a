"""Summarise rocprofv3 outputs into the committed profiles/ files.

  python tools/pmc_summary.py <tag> <trace_dir> <fetch_dir> <write_dir> <records>

* <trace_dir>/run_kernel_stats.csv -> profiles/<tag>_kernel_stats.csv (xdrg kernels)
* FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md §HBM):
  per-dispatch KB; FETCH doubled (gfx950 reports half of a wide streaming
  read), WRITE exact for 16-B streaming stores -> profiles/pmc_traffic.json
  bytes_per_launch per kernel (median over dispatches).
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n.replace("xdrg::", "")


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if "xdrg::" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return out


def main():
    tag, trace, fetch, write, records = sys.argv[1:6]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    rows = [r for r in csv.DictReader(open(os.path.join(trace, "run_kernel_stats.csv")))
            if "xdrg::" in r["Name"]]
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"], r["AverageNs"],
                        r["MinNs"], r["MaxNs"]])
    fe = per_kernel(os.path.join(fetch, "run_counter_collection.csv"), "FETCH_SIZE")
    wr = per_kernel(os.path.join(write, "run_counter_collection.csv"), "WRITE_SIZE")
    path = os.path.join(prof, "pmc_traffic.json")
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        doc = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                         "bench.py; KB per dispatch; FETCH x2 (gfx950 reports half of a wide "
                         "streaming read), WRITE as reported; median over dispatches",
               "kernels": {}}
    for k in sorted(set(fe) & set(wr)):
        base = k.split("<")[0]
        fkb, wkb = statistics.median(fe[k]), statistics.median(wr[k])
        doc["kernels"][base] = {"instance": k, "records": int(records), "tag": tag,
                                "fetch_kb_raw": fkb, "write_kb": wkb,
                                "bytes_per_launch": int(round((2 * fkb + wkb) * 1024)),
                                "dispatches": len(fe[k])}
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
