#!/usr/bin/env python3
"""Per kernel (template instantiation) over rocprofv3 --pmc passes, each with its kernel trace:
dispatches, mean duration, HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction) and
GB/s, SQ fractions (WAIT_ANY, WAIT_INST_ANY, ACTIVE_INST_ANY over WAVE_CYCLES), VALU / SMEM
instructions per wave, L2 hit rate.  python tools/pmc_kernels.py DIR [DIR ...]"""
import collections
import csv
import glob
import re
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name)
    return name.replace("void ", "").replace("aesfhe::", "")[:60]


def load(d):
    cc = glob.glob(f"{d}/*counter_collection.csv")[0]
    kt = glob.glob(f"{d}/*kernel_trace.csv")[0]
    dur = {}
    for r in csv.DictReader(open(kt)):
        dur[int(r["Dispatch_Id"])] = (short(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    val = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(cc)):
        val[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return dur, val


agg = collections.defaultdict(lambda: collections.Counter())
for d in sys.argv[1:]:
    dur, val = load(d)
    first = d == sys.argv[1]
    for did, (name, ns) in dur.items():
        a = agg[name]
        if first:
            a["n"] += 1
            a["ns"] += ns
        for c, v in val.items():
            if did in v:
                a[c] += v[did]
tot = sum(a["ns"] for a in agg.values())
print(f"{'kernel':46s} {'share':>6s} {'n':>5s} {'avg_us':>9s} {'GB/s':>7s} {'wait':>5s} {'wInst':>5s} {'activ':>5s} {'valu/w':>7s} {'smem/w':>6s} {'lds/w':>6s} {'L2hit':>5s} {'MB/disp':>8s} {'salu/w':>6s} {'vmem/w':>6s} {'mfma/w':>6s} {'ldsconf':>7s}")
for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"])[:40]:
    hbm = 2 * a["FETCH_SIZE"] * 1024 + a["WRITE_SIZE"] * 1024  # KB counters
    gbs = hbm / a["ns"] if a["ns"] else 0
    wc = a["SQ_WAVE_CYCLES"] or 1
    waves = a["SQ_WAVES"] or 1
    hit = a["TCC_HIT_sum"] / max(1.0, a["TCC_HIT_sum"] + a["TCC_MISS_sum"])
    print(f"{name[:46]:46s} {a['ns'] / tot * 100:5.1f}% {a['n']:5d} {a['ns'] / max(1, a['n']) / 1e3:9.1f} {gbs:7.0f} "
          f"{a['SQ_WAIT_ANY'] / wc:5.2f} {a['SQ_WAIT_INST_ANY'] / wc:5.2f} {a['SQ_ACTIVE_INST_ANY'] / wc:5.2f} "
          f"{a['SQ_INSTS_VALU'] / waves:7.0f} {a['SQ_INSTS_SMEM'] / waves:6.0f} {a['SQ_INSTS_LDS'] / waves:6.0f} {hit:5.2f} "
          f"{hbm / max(1, a['n']) / 1e6:8.1f} {a['SQ_INSTS_SALU'] / waves:6.0f} "
          f"{(a['SQ_INSTS_VMEM_RD'] + a['SQ_INSTS_VMEM_WR']) / waves:6.0f} {a['SQ_INSTS_MFMA'] / waves:6.0f} "
          f"{a['SQ_LDS_BANK_CONFLICT'] / max(1, a['n']):7.0f}")
