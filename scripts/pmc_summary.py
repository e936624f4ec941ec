"""Summarise rocprofv3 --pmc CSVs: per-dispatch average of every counter for one kernel family.

usage: pmc_summary.py <outdir> [kernel symbol (default: the kernel the bench line names)]
The summary carries `_key` = {config, width, height, spp, ranks, kernel} of the profiled bench run (its JSON line
in <outdir>/p1.log); bench.py uses a committed summary only for exactly that workload and kernel.
HBM traffic per dispatch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide reads, so bytes = 2 x FETCH_SIZE + WRITE_SIZE (x 1024).
"""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
key = None
try:
    line = [ln for ln in open(f"{out}/p1.log") if ln.startswith("{")][-1]
    b = json.loads(line)
    key = {"config": b["config"]["id"], "width": b["config"]["width"], "height": b["config"]["height"],
           "spp": b["config"]["spp"], "ranks": b["n_gpus"], "kernel": b["roofline"]["kernel"]}
except (OSError, IndexError, KeyError, ValueError):
    pass
kernel = sys.argv[2] if len(sys.argv) > 2 else (key["kernel"] if key else "k_trace")


def symbol(name: str) -> str:
    """rocprofv3's 'void k_trace_split<true>(hrt_dev::KParams)' -> 'k_trace_split<true>'."""
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    return name.split("(", 1)[0]

per = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in sorted(glob.glob(f"{out}/**/p*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if symbol(r["Kernel_Name"]) != kernel:
            continue
        dk = (f, r["Dispatch_Id"])
        per[dk][r["Counter_Name"]] += float(r["Counter_Value"])
        names[dk] = r["Kernel_Name"]
agg = collections.defaultdict(list)
for dk, cs in per.items():
    for c, v in cs.items():
        agg[c].append(v)
summary = {c: sum(v) / len(v) for c, v in agg.items()}
summary["_dispatches_per_pass"] = {c: len(v) for c, v in agg.items()}
summary["_kernels"] = sorted(set(names.values()))
if "FETCH_SIZE" in summary and "WRITE_SIZE" in summary:
    summary["hbm_read_bytes_per_launch"] = 2.0 * summary["FETCH_SIZE"] * 1024.0
    summary["hbm_write_bytes_per_launch"] = summary["WRITE_SIZE"] * 1024.0
    summary["hbm_bytes_per_launch"] = summary["hbm_read_bytes_per_launch"] + summary["hbm_write_bytes_per_launch"]
summary["_key"] = key
summary["_note"] = "per-dispatch averages; hbm bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE halving)"
json.dump(summary, open(f"{out}/pmc_summary.json", "w"), indent=1, sort_keys=True)
print(json.dumps(summary, indent=1, sort_keys=True))
