"""Per-kernel PMC counter averages from rocpd databases.
usage: python tools/pmc_kernel.py <pmc_dir> [<pmc_dir> ...] [--filter substr]"""
import collections
import glob
import os
import sqlite3
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    if flt in args:
        args.remove(flt)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in args:
        for f in glob.glob(os.path.join(d, "*.db")):
            c = sqlite3.connect(f)
            for did, name, cn, val in c.execute("select dispatch_id, kernel_name, counter_name, sum(value) from "
                                                "counters_collection group by dispatch_id, counter_name"):
                short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                if flt in short:
                    agg[short][cn].append(val)
    for k, cs in agg.items():
        print(k)
        for cn, v in sorted(cs.items()):
            print(f"   {cn:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
