"""Average rocprofv3 PMC counters per kernel from run_counter_collection.csv files."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(d + "/**/run_counter_collection.csv", recursive=True)):
        acc = collections.defaultdict(list)
        for x in csv.DictReader(open(f)):
            acc[(x["Kernel_Name"][:40], x["Counter_Name"])].append(float(x["Counter_Value"]))
        print(f)
        for (k, c), v in sorted(acc.items()):
            print(f"   {k:40s} {c:36s} n={len(v):3d} mean={sum(v)/len(v):.6g}")
