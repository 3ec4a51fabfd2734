"""Per-dispatch counter totals from rocprofv3 --pmc CSV output (the largest dispatch of a kernel)."""
import collections
import csv
import sys

path, kernel = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    if kernel in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
big = max(agg.values(), key=lambda c: max(c.values()))
for k in sorted(big):
    print(f"{k}\t{big[k]:.4e}")
