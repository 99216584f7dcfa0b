"""Print the top kernels of a rocprofv3 kernel_stats.csv (dev tool)."""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_rows/rows_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.1f} ms")
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
    print(f"{r['Name'][:52]:52s} {int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1e6:8.1f} ms "
          f"{float(r['Percentage']):5.1f}% avg {float(r['AverageNs']) / 1e3:8.1f} us")
