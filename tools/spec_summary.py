"""Summarise tools/spec_bench.sh: frame-walk kernel averages (rocprofv3 stats)
and the receive legs' frame_scan figures of framed configs 2 and 4."""
import csv
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/spec_b1"


def recv(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    for e in [d] + d.get("extra_configs", []):
        if isinstance(e, dict) and e.get("receive"):
            r = e["receive"]
            return {"receive_ms": r["ms_per_step"], "frame_scan_ms": r["frame_scan"]["avg_ms"],
                    "frac": r["frame_scan"]["frac"]}
    return None


for c in ("c2f", "c4f"):
    out = {"config": c}
    ks = os.path.join(D, c, "run_kernel_stats.csv")
    if os.path.exists(ks):
        for r in csv.DictReader(open(ks)):
            n = r["Name"]
            if "k_fs" in n or "k_fr" in n:
                out[n.split("(")[0].replace("void ", "").replace("xdrg::", "")] = round(float(r["AverageNs"]) / 1e3, 1)
    for tag in ("", "_exact"):
        p = os.path.join(D, c + tag + ".json")
        if os.path.exists(p):
            out["spec" if not tag else "exact"] = recv(p)
    print(json.dumps(out))
