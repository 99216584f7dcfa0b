"""Compare two rocprofv3 kernel_stats.csv files per kernel family (template arguments folded):
total ms, calls, average us (dev tool).   python tools/cmpk.py A.csv B.csv"""
import collections
import csv
import re
import sys


def load(p):
    d = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(p)):
        k = re.sub(r"<[^()]*>", "<>", r["Name"].split("(")[0]).replace("void ", "")[:48]
        d[k][0] += float(r["TotalDurationNs"]) / 1e6
        d[k][1] += int(r["Calls"])
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
print(f"{'kernel':48s} {'A ms':>9s} {'B ms':>9s} {'B/A':>6s} {'A avg us':>9s} {'B avg us':>9s}")
for k in sorted(set(a) | set(b), key=lambda k: -max(a[k][0], b[k][0]))[:18]:
    x, y = a[k], b[k]
    print(f"{k:48s} {x[0]:9.1f} {y[0]:9.1f} {y[0] / x[0] if x[0] else 0:6.3f} "
          f"{1e3 * x[0] / max(x[1], 1):9.1f} {1e3 * y[0] / max(y[1], 1):9.1f}")
print(f"{'TOTAL':48s} {sum(v[0] for v in a.values()):9.1f} {sum(v[0] for v in b.values()):9.1f}")
