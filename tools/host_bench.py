"""Host-inclusive legs of bench.py (XDRG_HOST_PTRS through the C-ABI) on
configs[1], for a few staging-ring shapes: one JSON line per shape."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--records", type=int, default=64 << 20)
    p.add_argument("--shapes", default="4x64,4x256,2x256,8x32", help="slots x MiB, comma separated")
    p.add_argument("--legs", default="staged,staged_dma,mapped,staged_pageable")
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    from oncrpc4j_amd import abi, engine
    sch = engine.Schema([(abi.T_INT, abi.K_SCALAR, 0)] * 8)
    for shape in a.shapes.split(","):
        k, mb = (int(x) for x in shape.split("x"))
        r = bench.host_inclusive(0, sch, a.records, reps=a.reps, slot_bytes=mb << 20, slots=k,
                                 legs=tuple(a.legs.split(",")))
        print(json.dumps({"shape": shape, **r}), flush=True)


if __name__ == "__main__":
    main()
