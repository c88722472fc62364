"""Average PMC counters per dispatch of kernels matching a substring (rocprofv3 csv output)."""
import collections
import csv
import glob
import sys

root, pat = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{root}/*/*counter_collection.csv")):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    for k in sorted(tot):
        print(f"{k:32s} {tot[k] / max(1, len(disp[k])):16.0f}  (per dispatch, {len(disp[k])} dispatches)")
