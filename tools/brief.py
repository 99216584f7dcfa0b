#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line: value, ms/step, verified, selected kernel classes
(python tools/brief.py bench.json [label] [class-substring ...])."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
label = sys.argv[2] if len(sys.argv) > 2 else ""
pats = sys.argv[3:] or ["poly2"]
k = (d.get("roofline") or {}).get("kernels") or {}
sel = {n: (k[n].get("avg_us"), k[n].get("dispatches_per_step"), k[n].get("hbm_bytes_per_launch"))
       for n in k if any(p in n for p in pats)}
a10 = d.get("aes128_10_rounds") or {}
print(label, d["value"], d["ms_per_step"], d["config"]["verified"], "frac", d["roofline"]["frac"], sel,
      "aes10", a10.get("value"), a10.get("verified"))
