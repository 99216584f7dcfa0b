#!/usr/bin/env python3
"""Config 2 / 3 legs of bench.py on their own (dev tool), for rocprofv3 kernel summaries:

    rocprofv3 --kernel-trace --stats -d out -o c23 -- python3 tools/config_prof.py [--reps R]

Builds the bench engine (N = 2^16, L = 30, K = 10, scale 40), runs bench.config_legs (warm-up +
timed call per leg, FIPS-verified) R times and prints the legs' JSON."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "aes-fhe_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--legs", default="2,3")
    a = ap.parse_args()
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    args.legs = a.legs
    eng, drv = bench.setup_engine(args, 0, 0)
    for r in range(a.reps):
        t0 = time.perf_counter()
        out = bench.config_legs(args, eng, drv)
        if "h" in a.legs.split(","):
            out["reference_harness"] = bench.reference_harness_leg(args)
        out["wall_s"] = round(time.perf_counter() - t0, 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
