"""HBM traffic of the NTT pass kernels from rocprofv3 --pmc CSVs (dev tool; writes the JSON that
bench.py's roofline.traffic reads).  Per launch: read = FETCH_SIZE x 2 (the gfx950 correction,
calibrated on tools/ntt_bench's copy kernel whose bytes are known), write = WRITE_SIZE (KiB in
the counters).  Algorithmic bytes per pass launch = 8 N per limb, limbs = Grid_Size / 4096 (16
workgroups of 256 lanes per limb).  Usage: ntt_traffic.py fetch.csv write.csv [out.json]"""
import collections
import csv
import json
import sys

NTT = ("k_nttf_fwd_cols", "k_nttf_fwd_rows_t<false>", "k_nttf_inv_rows", "k_nttf_inv_cols")
N = 1 << 16


def load(path, counter):
    per = collections.defaultdict(list)  # kernel -> [(grid, value)]
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for k in NTT:
            base = k.split("<")[0]
            if (base + "<" + k.split("<")[1][:-1] if "<" in k else base) in name:
                # the product INTT (k_nttf_inv_rows<R, true, ...>) reads two operands: 16 N
                # algorithmic bytes per limb (bench.py / engine ProfScope credit it the same)
                w = 2.0 if base == "k_nttf_inv_rows" and ", true" in name.split("(")[0] else 1.0
                per[k].append((int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024.0, w))
    return per


def main():
    f, w = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    hbm = alg = 0.0
    launches = 0
    per_kernel = {}
    for k in NTT:
        if not f.get(k):
            continue
        rd = [2.0 * v for _, v, _ in f[k]]
        wr = [v for _, v, _ in w.get(k, [])] or [0.0]
        a = sum(8.0 * N * g / 4096 * x for g, _, x in f[k])
        hbm += sum(rd) + sum(wr) * len(rd) / len(wr)
        alg += a
        launches += len(rd)
        per_kernel[k] = {"read_bytes_per_launch": sum(rd) / len(rd),
                         "write_bytes_per_launch": sum(wr) / len(wr),
                         "alg_bytes_per_launch": a / len(rd), "launches": len(rd)}
    out = {"family": "ntt passes (" + ", ".join(per_kernel) + ")", "hbm_bytes": hbm,
           "alg_bytes": alg, "launches": launches, "traffic_over_alg": hbm / alg,
           "per_kernel": per_kernel,
           "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes, --kernel-trace) "
                     "on tools/ks_driver (C ABI, B=16, N=2^16, L=30, ct x ct multiplies: the engine's "
                     "NTT kernels on the bench's parameter set); FETCH_SIZE x 2 per MI355X_MICROARCH.md, "
                     "verified on tools/ntt_bench's copy kernel (tools/ntt_traffic.py)"}
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
