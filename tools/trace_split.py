#!/usr/bin/env python3
"""Per-kernel breakdown of a rocprofv3 kernel trace, split into busy segments (dev tool).
Usage: trace_split.py trace.csv [gap_ms] [seg_index ...]"""
import collections
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    gap = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 3e6
    segs, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > gap:
            segs.append(cur)
            cur = []
        cur.append(b)
    segs.append(cur)
    for i, s in enumerate(segs):
        t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
        print(f"seg {i}: {len(s)} kernels, span {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms")
    for i in map(int, sys.argv[3:]):
        per = collections.defaultdict(lambda: [0, 0.0])
        for r in segs[i]:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("aesfhe::", "")
            per[k][0] += 1
            per[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        print(f"--- seg {i}")
        for k, (n, ms) in sorted(per.items(), key=lambda kv: -kv[1][1])[:30]:
            print(f"{ms:9.2f} ms {n:6d} {ms / n * 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main()
