#!/usr/bin/env python3
"""HBM traffic (and fp64 instruction counts) per kernel class of ONE bench round step, from
rocprofv3 --pmc counter CSVs (dev tool; writes the JSON bench.py's roofline.traffic and
roofline.kernels read).

    pmc_traffic.py --fetch F.csv --write W.csv [--f64 S.csv] --bench bench.json --head SHA -o out.json

The runs are `bench.py ... --steps 1 --pmc-marks`: the step's dispatches are the ones between the
two torch fill kernels the bench launches around its timed region.  read = FETCH_SIZE x 2 (the
gfx950 correction, MI355X_MICROARCH.md "HBM"), write = WRITE_SIZE (both in KiB).  f64 FLOPs =
64 lanes x (ADD + MUL + 2 FMA + TRANS) fp64 VALU instructions (SQ_INSTS_VALU_*_F64, per wave)."""
import argparse
import collections
import csv
import json
import re

# kernel name -> engine profile class (engine.hip ProfScope labels)
CLASSES = [
    (r"k_nttf_fwd_cols_spread<", "ntt_fwd_cols_spread"),
    (r"k_nttf_fwd_cols<", "ntt_fwd_cols"),
    (r"k_nttf_fwd_rows_t<true", "ntt_fwd_rows_fin"),
    (r"k_nttf_fwd_rows_t<false", "ntt_fwd_rows"),
    (r"k_nttf_inv_rows<\d+, true", "ntt_inv_rows_prod"),
    (r"k_nttf_inv_rows<\d+, false", "ntt_inv_rows"),
    (r"k_nttf_inv_cols<", "ntt_inv_cols"),
    (r"k_ntt_(fwd|inv)_(rows|cols)<", "ntt_generic"),
    (r"k_nttf_rows_ks_p<\d+, true, 1>", "ks_rows_fin.prod"),  # round 5: the LDS-DMA pipelined rows
    (r"k_nttf_rows_ks_p<\d+, false, 1>", "ks_rows_fin.ks"),
    (r"k_nttf_rows_ks_p<\d+, true, 2>", "ks_rows_inner.prod"),
    (r"k_nttf_rows_ks_p<\d+, false, 2>", "ks_rows_inner.ks"),
    (r"k_nttf_rows_ks_p<\d+, true", "ks_rows_acc.prod"),
    (r"k_nttf_rows_ks_p<", "ks_rows_acc.ks"),
    (r"k_bconv_cols<\d+, true, false", "modup_cols"),  # round 6: conversion + forward column pass
    (r"k_bconv_cols<\d+, true, true", "moddown_cols"),
    (r"k_bconv_mfma<\d+, false", "modup"),  # matrix-core conversions: ModUp (no v slot), ModDown (v)
    (r"k_bconv_mfma<\d+, true", "moddown"),
    (r"k_bsgs_terms<", "bsgs_terms"),
    (r"k_nttf_rows_ks<\d+, \d+, true, 1>", "ks_rows_fin.prod"),
    (r"k_nttf_rows_ks<\d+, \d+, false, 1>", "ks_rows_fin.ks"),
    (r"k_nttf_rows_ks<\d+, \d+, true, 2>", "ks_rows_inner.prod"),
    (r"k_nttf_rows_ks<\d+, \d+, false, 2>", "ks_rows_inner.ks"),
    (r"k_nttf_rows_ks<\d+, \d+, true", "ks_rows_acc.prod"),
    (r"k_nttf_rows_ks<", "ks_rows_acc.ks"),
    (r"k_ks_inner_all<", "ks_inner"),
    (r"k_ks_inner_multi<", "ks_inner_multi"),
    (r"k_modup<", "modup"),
    (r"k_moddown<", "moddown"),
    (r"k_moddown_finish", "moddown_finish"),
    (r"k_poly2_int(_s|_split)?<", "poly2_int"),
    (r"k_poly2\b", "poly2"),
    (r"k_gather_batch", "gather"),
    (r"k_lincomb_many", "lincomb_many"),
    (r"k_lincomb\b", "lincomb"),
    (r"k_dot_pt_ext_multi", "dot_pt_ext_multi"),
    (r"k_dot_pt\b", "dot_pt"),
    (r"k_dot\b", "dot"),
    (r"k_mul_const", "mul_const"),
    (r"k_addsub", "add"),
    (r"k_tensor_fma", "tensor_fma"),
    (r"k_tensor\b", "tensor"),
    (r"k_galois", "galois"),
]
NTT_FAMILY = {"ntt_fwd_cols", "ntt_fwd_cols_spread", "ntt_fwd_rows", "ntt_fwd_rows_fin", "ntt_inv_rows",
              "ntt_inv_rows_prod", "ntt_inv_cols", "ntt_generic"}


def klass(name):
    for pat, c in CLASSES:
        if re.search(pat, name):
            return c
    return None


def step_records(path):
    """{dispatch_id: (kernel name, {counter: value})} of the dispatches between the two marker
    fills (torch FillFunctor kernels)."""
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        rec = per.setdefault(d, [r["Kernel_Name"], {}])
        rec[1][r["Counter_Name"]] = rec[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    marks = [d for d in ids if "FillFunctor" in per[d][0] or "fill" in per[d][0].lower()]
    if len(marks) < 2:
        raise SystemExit(f"{path}: expected two marker fills, found {len(marks)}")
    a, b = marks[-2], marks[-1]
    return {d: per[d] for d in ids if a < d < b}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--f64")
    ap.add_argument("--bench", help="the JSON line of one of the runs (workload shape)")
    ap.add_argument("--head", required=True)
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    f, w = step_records(a.fetch), step_records(a.write)
    s = step_records(a.f64) if a.f64 else {}
    if len(f) != len(w):
        raise SystemExit(f"fetch and write runs differ in dispatches: {len(f)} vs {len(w)}")
    agg = collections.defaultdict(lambda: {"launches": 0, "read": 0.0, "write": 0.0, "f64": 0.0})
    for (df, (nf, cf)), (dw, (nw, cw)) in zip(sorted(f.items()), sorted(w.items())):
        if nf != nw:
            raise SystemExit(f"dispatch order differs: {nf} vs {nw}")
        c = klass(nf) or nf.split("(")[0]
        g = agg[c]
        g["launches"] += 1
        g["read"] += 2.0 * 1024.0 * cf.get("FETCH_SIZE", 0.0)
        g["write"] += 1024.0 * cw.get("WRITE_SIZE", 0.0)
    f64_counted = bool(s)
    for d, (n, cs) in s.items():
        c = klass(n) or n.split("(")[0]
        agg[c]["f64"] += 64.0 * (cs.get("SQ_INSTS_VALU_ADD_F64", 0) + cs.get("SQ_INSTS_VALU_MUL_F64", 0) +
                                 2 * cs.get("SQ_INSTS_VALU_FMA_F64", 0) + cs.get("SQ_INSTS_VALU_TRANS_F64", 0))
    per = {}
    for c, g in sorted(agg.items(), key=lambda kv: -(kv[1]["read"] + kv[1]["write"])):
        n = g["launches"]
        per[c] = {"launches": n, "read_bytes_per_launch": g["read"] / n, "write_bytes_per_launch": g["write"] / n,
                  "hbm_bytes_per_launch": (g["read"] + g["write"]) / n}
        if f64_counted:
            per[c]["f64_flops_per_launch"] = g["f64"] / n
    fam = [per[c] for c in per if c in NTT_FAMILY]
    nl = sum(p["launches"] for p in fam)
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import csrc_sha16
    out = {"head": a.head, "csrc_sha16": csrc_sha16(),
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE" + (" / --pmc SQ_INSTS_VALU_*_F64" if f64_counted else "")
                     + " (separate passes, --kernel-trace) over one bench round step between marker kernels; "
                       "FETCH_SIZE x 2 (gfx950), tools/pmc_traffic.py",
           "ntt_family": {"classes": sorted(c for c in per if c in NTT_FAMILY), "launches": nl,
                          "hbm_bytes_per_launch": sum(p["hbm_bytes_per_launch"] * p["launches"] for p in fam) / max(nl, 1)},
           "per_kernel": per}
    if a.bench:
        r = json.loads(open(a.bench).read().strip().splitlines()[-1])
        cfg = r["config"]
        out["workload"] = {"log_n": cfg["log_n"], "max_level": cfg["max_level"], "special_primes": cfg["special_primes"],
                           "digit_primes": cfg.get("digit_primes", cfg["special_primes"]),
                           "batch": cfg["ciphertext_sets_per_gpu"], "layout": cfg["layout"]}
    text = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
