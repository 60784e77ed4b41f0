"""Average the PMC counters of one kernel over its dispatches: python scripts/pmc_sum.py DIR [kernel-substring]"""
import collections, csv, glob, sys
d = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else "pileup"
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f"{f.split('/')[-2]:4s} {k:24s} n={len(v):3d} mean={sum(v)/len(v):.6g}")
