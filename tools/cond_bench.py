"""Throughput of conditional tapes (rpcgen unions / optional data; DESIGN.md
§8f2, §8f4) on three builder-designed shapes:

* RELEASE: lease_cache.x RELEASE(lease_key, lease_state) argument batches,
  4 Mi records (unsigned hyper, string<1024> of 8..64 B, an int union whose
  arms are opaque<64> / unsigned int / void);
* READDIRPLUS: plus_types.x `plus_res` replies (the reply union, optional
  directory attributes, a verifier and a `plus_entry *next` list whose every
  element carries an optional attribute union and an optional handle union),
  512 Ki records of 0..12 entries;
* chunk map: chunk_map.x `chunk_map` replies (a `chunk_ent *next` list whose
  every element holds `replica copies[2]`, unrolled, each replica with an
  optional checksum and a tag opaque<16>), 1 Mi records of 0..12 entries;
* volume_index.x and acl_tree.x: groups inside group elements, two and four
  group levels.

Device-resident, HIP-event timed encode and decode (median of reps); bytes =
native + XDR per direction, as bench.py counts them; roundtrip_ok = the decode
succeeds and its output re-encodes to the same stream and offsets."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oncrpc4j_amd import abi, engine, rpcgen  # noqa: E402
from oncrpc4j_amd.columns import DeviceBatch, random_batch  # noqa: E402

LEASE = 0x2000F33E


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def discriminants(fields, conds, hb, rng):
    """Realistic arm mixes: bool discriminants 0/1, int discriminants drawn
    from their case values plus one that takes the default arm."""
    for k in sorted({d for _, d, _, _ in conds}):
        rows = hb.arrays[k].shape[0]
        if fields[k][0] == abi.T_BOOL:
            hb.arrays[k][:] = rng.integers(0, 2, rows, dtype=np.uint8)
        else:
            vals = sorted({v for _, d, _, vs in conds if d == k for v in vs})
            pool = np.array(vals + [max(vals) + 1], dtype=np.int64)
            hb.arrays[k][:] = pool[rng.integers(0, pool.size, rows)].astype(hb.arrays[k].dtype)


def run(name, fields, conds, n, dyn_len, group_len=(0, 4)):
    # XDRG_SHAPES=plus,chunk: only the shapes whose name holds one of these (profiling runs)
    want = [w.lower() for w in os.environ.get("XDRG_SHAPES", "").split(",") if w]
    if want and not any(w in name.lower() for w in want):
        return {"shape": name, "skipped": True}
    ctx = engine.Context(0)
    ctx.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
    ctx.set_stream(torch.cuda.current_stream())
    hb = random_batch(fields, n, seed=3, dyn_len=dyn_len, group_len=group_len, special_floats=False)
    discriminants(fields, conds, hb, np.random.default_rng(3))
    sch = engine.Schema(fields, conds)
    db = DeviceBatch.from_host(hb)
    cap = hb.xdr_total() + 64            # every field present: an upper bound
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    cols = db.columns()
    total = ctx.encode(sch, cols, n, out, cap, rec_offsets=ro)
    t_enc = timed(lambda: ctx.encode(sch, cols, n, out, cap, rec_offsets=ro))
    back = DeviceBatch.empty(fields, n, hb.dyn_caps())
    bcols = back.columns()
    t_dec = timed(lambda: ctx.decode(sch, out, total, n, bcols, rec_offsets=ro))
    ok = ctx.decode(sch, out, total, n, bcols, rec_offsets=ro) == (0, n, 0)
    # an output check at full size: the decoded batch re-encodes to the same
    # stream and record offsets (absent arms, lists and counts included)
    out2 = torch.zeros_like(out)
    ro2 = torch.zeros_like(ro)
    ok = ok and ctx.encode(sch, bcols, n, out2, cap, rec_offsets=ro2) == total and \
        bool(torch.equal(out2, out)) and bool(torch.equal(ro2, ro))
    nat = hb.native_bytes()
    per_dir = nat + total
    return {"shape": name, "records": n, "xdr_bytes": total, "native_bytes": nat,
            "encode_ms": round(t_enc, 3), "decode_ms": round(t_dec, 3),
            "encode_GBps": round(per_dir / t_enc / 1e6, 1), "decode_GBps": round(per_dir / t_dec / 1e6, 1),
            "frac_of_8TBps": round(2 * per_dir / (t_enc + t_dec) / 1e6 / 8000, 4),
            "Mrec_s": round(2 * n / (t_enc + t_dec) / 1e3, 1), "roundtrip_ok": ok}


def main():
    g = os.path.join(ROOT, "tests", "golden", "rpcgen")
    lease = rpcgen.parse_file(os.path.join(g, "lease_cache.x"))
    f, c = lease.args_tape(LEASE, 1, 2)
    print(json.dumps(run("RELEASE(lease_key, lease_state) args", f, c, 4 << 20, (8, 64))), flush=True)
    plus = rpcgen.parse_file(os.path.join(g, "plus_types.x"))
    f, c = plus.tape("plus_res")
    print(json.dumps(run("READDIRPLUS plus_res replies", f, c, 512 << 10, (0, 40), (0, 12))), flush=True)
    cmap = rpcgen.parse_file(os.path.join(g, "chunk_map.x"))
    f, c = cmap.tape("chunk_map")
    print(json.dumps(run("chunk_map replies (replica copies[2] in list elements)", f, c, 1 << 20, (0, 16), (0, 12))),
          flush=True)
    vix = rpcgen.parse_file(os.path.join(g, "volume_index.x"))
    f, c = vix.tape("volume_index")
    print(json.dumps(run("volume_index replies (a list and an array inside list elements)", f, c, 512 << 10,
                         (0, 24), (0, 6))), flush=True)
    acl = rpcgen.parse_file(os.path.join(g, "acl_tree.x"))
    f, c = acl.tape("tree_res")
    print(json.dumps(run("acl_tree replies (four group levels: entry list > ace list > who<8> > tags<>)", f, c,
                         256 << 10, (0, 24), (0, 4))), flush=True)


if __name__ == "__main__":
    main()
