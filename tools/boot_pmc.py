#!/usr/bin/env python3
"""Per kernel class of a rocprofv3 run (two --pmc passes, FETCH_SIZE and WRITE_SIZE, each with its
kernel trace): dispatches, time, HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction)
and achieved GB/s.  python tools/boot_pmc.py FETCH_DIR WRITE_DIR"""
import collections
import csv
import glob
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import klass  # noqa: E402


def load(d, counter):
    cc = glob.glob(f"{d}/*counter_collection.csv")[0]
    kt = glob.glob(f"{d}/*kernel_trace.csv")[0]
    dur = {}
    for r in csv.DictReader(open(kt)):
        dur[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    val = collections.Counter()
    for r in csv.DictReader(open(cc)):
        if r["Counter_Name"] == counter:
            val[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return dur, val


fd, fv = load(sys.argv[1], "FETCH_SIZE")
wd, wv = load(sys.argv[2], "WRITE_SIZE")
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for i, (name, ns) in fd.items():
    c = klass(name) or name.split("(")[0][:40]
    a = agg[c]
    a[0] += 1
    a[1] += ns
    a[2] += 2048.0 * fv.get(i, 0.0)
wsum = collections.defaultdict(float)
for i, (name, ns) in wd.items():
    wsum[klass(name) or name.split("(")[0][:40]] += 1024.0 * wv.get(i, 0.0)
tot = sum(a[1] for a in agg.values())
print(f"{'class':28s} {'n':>6s} {'ms':>9s} {'share':>6s} {'GB read':>9s} {'GB write':>9s} {'TB/s':>6s}")
for c, (n, ns, rd) in sorted(((c, a[:3]) for c, a in agg.items()), key=lambda kv: -kv[1][1]):
    wr = wsum.get(c, 0.0)
    print(f"{c[:28]:28s} {n:6d} {ns / 1e6:9.1f} {ns / tot:6.3f} {rd / 1e9:9.2f} {wr / 1e9:9.2f} {(rd + wr) / max(ns, 1) / 1e3:6.2f}")
