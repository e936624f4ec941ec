"""Summarise rocprofv3 --pmc CSVs: per-dispatch average of every counter for the k_render kernels."""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in sorted(glob.glob(f"{out}/**/p*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "k_render" not in r["Kernel_Name"]:
            continue
        key = (f, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        names[key] = r["Kernel_Name"]
agg = collections.defaultdict(list)
for key, cs in per.items():
    for c, v in cs.items():
        agg[c].append(v)
summary = {c: sum(v) / len(v) for c, v in agg.items()}
summary["_dispatches_per_pass"] = {c: len(v) for c, v in agg.items()}
summary["_kernels"] = sorted(set(names.values()))
json.dump(summary, open(f"{out}/pmc_summary.json", "w"), indent=1, sort_keys=True)
print(json.dumps(summary, indent=1, sort_keys=True))
