"""Summarise rocprofv3 outputs into the committed profiles/ files.

  python tools/pmc_summary.py <tag> <trace_dir> <fetch_dir> <write_dir> <records>

* <trace_dir>/run_kernel_stats.csv -> profiles/<tag>_kernel_stats.csv (xdrg kernels)
* FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md §HBM):
  per-dispatch KB; FETCH doubled (gfx950 reports half of a wide streaming
  read), WRITE exact for 16-B streaming stores -> profiles/pmc_traffic.json
  bytes_per_launch per kernel and grid (median over dispatches), and per
  bench.py config the bytes of its dominant launch (CONFIGS below: the place
  kernels of one direction summed, encode and decode averaged, as bench.py's
  roofline `achieved` averages their launches).
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


# bench.py config -> (records, encode kernels, decode kernels) as (name, grid)
CONFIGS = {
    "2": (67108864, [("k_stream_bswap", "134217728")], [("k_stream_bswap", "134217728")]),
    "2f": (67108864, [("k_stream_framed_enc_lean", "150994944")], [("k_stream_framed_dec_lean", "134217728")]),
    "3": (16777216, [("k_enc_place_g", "4194304"), ("k_enc_payload", "1073741824")],
          [("k_dec_place_g", "4194304"), ("k_dec_payload", "1073741824")]),
    "4": (33554432, [("k_enc_stage_rm|k_enc_ostage|k_enc_stage", "8388608"), ("k_enc_place_g?", "8388608")],
          [("k_dec_sweep|k_dec_stage", "8388608"), ("k_dec_place_g?", "8388608")]),
    "4f": (33554432, [("k_enc_stage_rm|k_enc_ostage|k_enc_stage", "8388608"), ("k_enc_place_g?", "8388608")],
           [("k_dec_sweep|k_dec_stage", "8388608"), ("k_dec_place_g?", "8388608")]),
}
# (a name "a|b" takes the first of the alternatives the profile holds: the
# staged kernels' variants replace them when the tuning selects them; a name
# ending in "?" is dropped when the profile does not hold it: the one-pass
# derived-count decode launches no group kernel for big-record blocks)


def resolve(ks, table):
    out = []
    for name, grid in ks:
        opt = name.endswith("?")
        for alt in name.rstrip("?").split("|"):
            if (alt, grid) in table:
                out.append((alt, grid))
                break
        else:
            if not opt:
                out.append((name, grid))
    return out


def by_grid(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if "xdrg::" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        out.setdefault((short(r["Kernel_Name"]).split("<")[0], r["Grid_Size"]), []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def _trace_stats(path):
    """rocprofv3 kernel stats rows of the xdrg kernels."""
    return [r for r in csv.DictReader(open(path)) if "xdrg::" in r["Name"]]


def per_config(tag, root):
    """Per-config evidence (tools/profile_configs.sh): root/c<key>/{trace,fetch,write}
    of one bench.py workload each -> profiles/<tag>_configs/c<key>_kernel_stats.csv
    and pmc_traffic.json configs[key] from that config's own launches, with the
    phase averages that reproduce bench.py's roofline fraction."""
    prof = os.path.join(ROOT, "profiles")
    out_dir = os.path.join(prof, f"{tag}_configs")
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(prof, "pmc_traffic.json")
    doc = json.load(open(path))
    for key, (recs, enc, dec) in CONFIGS.items():
        d = os.path.join(root, f"c{key}")
        tr = os.path.join(d, "trace", "run_kernel_stats.csv")
        if not os.path.exists(tr):
            print("no trace for", key)
            continue
        rows = _trace_stats(tr)
        with open(os.path.join(out_dir, f"c{key}_kernel_stats.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
            for r in rows:
                w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["MinNs"], r["MaxNs"]])
        # a kernel's template variants share its base name: the one with the most
        # time is the phase's launch (a derived-count decode's rerun variants
        # are few-microsecond no-ops)
        avg, tot = {}, {}
        for r in rows:
            b = short(r["Name"]).split("<")[0]
            if float(r["TotalDurationNs"]) > tot.get(b, -1.0):
                tot[b] = float(r["TotalDurationNs"])
                avg[b] = float(r["AverageNs"])
        fg = by_grid(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
        wg = by_grid(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
        enc, dec = resolve(enc, fg), resolve(dec, fg)
        sides = []
        for ks in (enc, dec):
            if not all(k in fg and k in wg for k in ks):
                break
            sides.append((sum(2 * fg[k] * 1024 for k in ks), sum(wg[k] * 1024 for k in ks)))
        # a phase's launch = its kernels back to back (bench.py times the phase)
        phase_ns = [sum(avg.get(k[0], 0.0) for k in ks) for ks in (enc, dec)]
        e = {"records": recs, "tag": tag, "encode": [k[0] for k in enc], "decode": [k[0] for k in dec],
             "kernel_stats": os.path.relpath(os.path.join(out_dir, f"c{key}_kernel_stats.csv"), ROOT),
             "phase_avg_ns": [round(x, 1) for x in phase_ns]}
        if len(sides) == 2:
            e.update({"fetch_bytes": [int(x[0]) for x in sides], "write_bytes": [int(x[1]) for x in sides],
                      "bytes_per_launch": int(round(sum(x[0] + x[1] for x in sides) / 2))})
        doc["configs"][key] = e
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(json.dumps(doc["configs"], indent=1))


def main():
    if sys.argv[1] == "--per-config":
        per_config(sys.argv[2], sys.argv[3])
        return
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
    fg = by_grid(os.path.join(fetch, "run_counter_collection.csv"), "FETCH_SIZE")
    wg = by_grid(os.path.join(write, "run_counter_collection.csv"), "WRITE_SIZE")
    doc["configs"] = {}
    for key, (recs, enc, dec) in CONFIGS.items():
        sides = []
        enc, dec = resolve(enc, fg), resolve(dec, fg)
        for ks in (enc, dec):
            if not all(k in fg and k in wg for k in ks):
                break
            f_b = sum(2 * fg[k] * 1024 for k in ks)
            w_b = sum(wg[k] * 1024 for k in ks)
            sides.append((f_b, w_b))
        if len(sides) == 2:
            doc["configs"][key] = {"records": recs, "tag": tag, "encode": [k[0] for k in enc],
                                   "decode": [k[0] for k in dec],
                                   "fetch_bytes": [int(x[0]) for x in sides],
                                   "write_bytes": [int(x[1]) for x in sides],
                                   "bytes_per_launch": int(round(sum(x[0] + x[1] for x in sides) / 2))}
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
