"""HBM traffic per launch of the GEMM family from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE in separate runs, MI355X_MICROARCH.md 'rocprofv3 PMC slots').  Units: KB.  gfx950
correction (MI355X_MICROARCH.md 'HBM'): FETCH_SIZE counts half the bytes of a wide coalesced
read -> doubled; WRITE_SIZE taken as is.
usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> > profiles/<round>_gemm_traffic.json"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "*.db")):  # rocpd output (rocprofv3 default on ROCm 7.2)
        import sqlite3
        c = sqlite3.connect(f)
        for did, name, val in c.execute("select dispatch_id, kernel_name, sum(value) from counters_collection "
                                        "where counter_name = ? group by dispatch_id", (counter,)):
            out[int(did)] = (name, float(val))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]))
    return out


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    fam = "gemm_glds_kernel"  # the fp32 / bf16-in-LDS and the bf16-operand GEMMs are all this template
    fk = [v for n, v in fetch.values() if fam in n]
    wk = [v for n, v in write.values() if fam in n]
    fetch_b = 2.0 * 1024 * sum(fk) / len(fk)
    write_b = 1024 * sum(wk) / len(wk)
    out = {
        "kernel": fam + "<*>", "launches_fetch_pass": len(fk), "launches_write_pass": len(wk),
        "fetch_bytes_per_launch": round(fetch_b), "write_bytes_per_launch": round(write_b),
        "hbm_bytes_per_launch": round(fetch_b + write_b),
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate runs of bench.py --eager --steps 1 "
                  "--warmup 1; FETCH_SIZE x2 (gfx950 wide-read undercount), KB x1024",
    }
    if len(sys.argv) > 3:  # the workload the passes ran (bench.py matches on batch, d, layers, amp)
        out.update(batch=int(sys.argv[3]), workload=sys.argv[4] if len(sys.argv) > 4 else "C2 d=256 12L")
    if len(sys.argv) > 5:
        d, layers, amp = sys.argv[5].split(",")
        out.update(d=int(d), layers=int(layers), amp=amp == "1")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
