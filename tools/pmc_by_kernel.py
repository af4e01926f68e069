"""Mean per-dispatch PMC counters per kernel instance (full template names,
shortened to the template arguments) from rocprofv3 --pmc output trees.
usage: python tools/pmc_by_kernel.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
        for x in csv.DictReader(open(f)):
            acc[short(x["Kernel_Name"])][x["Counter_Name"]].append(float(x["Counter_Value"]))
for k in sorted(acc):
    print(k)
    for c in sorted(acc[k]):
        v = acc[k][c]
        print(f"   {c:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
