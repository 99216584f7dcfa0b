"""Per-kernel PMC summary of tools/gpu_pmc.sh output (dev tool): HBM-side bytes per launch
(FETCH_SIZE x 2 -- the gfx950 correction calibrated on tools/ntt_bench's copy kernel -- plus
WRITE_SIZE; counters are in KiB) and the SQ issue / wait split."""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"


def load(tag):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{d}/pmc_{tag}/p_counter_collection.csv")):
        agg[r["Kernel_Name"].split("(")[0][:44]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


f, w, sq = load("fetch"), load("write"), load("sq")
print(f"{'kernel':44s} {'n':>4s} {'read MB':>8s} {'write MB':>8s} {'VALU/wave-cyc':>13s} {'wait%':>6s} {'issue-stall%':>12s}")
for k in sorted(f, key=lambda k: -sum(f[k]["FETCH_SIZE"])):
    fs = f[k]["FETCH_SIZE"]
    ws = w.get(k, {}).get("WRITE_SIZE", [0])
    s = sq.get(k, {})
    cyc = sum(s.get("SQ_WAVE_CYCLES", [0])) or 1
    print(f"{k:44s} {len(fs):4d} {2 * sum(fs) / len(fs) / 1024:8.1f} {sum(ws) / len(ws) / 1024:8.1f} "
          f"{sum(s.get('SQ_INSTS_VALU', [0])) / cyc * 4:13.3f} {100 * sum(s.get('SQ_WAIT_ANY', [0])) / cyc:6.1f} "
          f"{100 * sum(s.get('SQ_WAIT_INST_ANY', [0])) / cyc:12.1f}")
