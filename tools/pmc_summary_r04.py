#!/usr/bin/env python3
"""Per kernel class of one bench round step (rocprofv3 --pmc CSVs between the marker fills):
SQ wave / wait cycles and instruction counts, L2 (TCC) hit rate.
python tools/pmc_summary_r04.py SQ.csv TCC.csv > out.txt"""
import collections
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import klass, step_records  # noqa: E402

sq, tcc = step_records(sys.argv[1]), step_records(sys.argv[2])
agg = collections.defaultdict(lambda: collections.Counter())
for recs in (sq, tcc):
    for d, (name, cs) in recs.items():
        c = klass(name) or name.split("(")[0]
        agg[c].update(cs)
        if recs is sq:
            agg[c]["n"] += 1
print("# rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
      "SQ_INSTS_VALU SQ_INSTS_SMEM / --pmc TCC_HIT_sum TCC_MISS_sum, --kernel-trace, one bench round step between")
print("# marker kernels (bench.py --steps 1 --warmup 1 --pmc-marks ...; tools/gpu_r04_pmc.sh).  Wait fractions are of")
print("# SQ_WAVE_CYCLES; VALU / SMEM per wave; L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS).")
print(f"{'class':24s} {'n':>5s} {'waves':>10s} {'wave_cyc':>10s} {'WAIT_ANY':>8s} {'WAIT_INST':>9s} {'ACTIVE':>7s} "
      f"{'VALU/wv':>8s} {'SMEM/wv':>8s} {'L2hit':>6s}")
for c, v in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    wc = v["SQ_WAVE_CYCLES"] or 1
    wv = v["SQ_WAVES"] or 1
    h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
    print(f"{c[:24]:24s} {v['n']:5d} {v['SQ_WAVES']:10.0f} {wc:10.3g} {v['SQ_WAIT_ANY'] / wc:8.2f} "
          f"{v['SQ_WAIT_INST_ANY'] / wc:9.2f} {v['SQ_ACTIVE_INST_ANY'] / wc:7.2f} {v['SQ_INSTS_VALU'] / wv:8.0f} "
          f"{v['SQ_INSTS_SMEM'] / wv:8.1f} {h / (h + m) if h + m else 0:6.2f}")
