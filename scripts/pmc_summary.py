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
line_json = None
try:
    line = [ln for ln in open(f"{out}/p1.log") if ln.startswith("{")][-1]
    b = json.loads(line)
    line_json = b
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
# The timed launches only (round 6): a bench run's warmup step learns the tiles' cost order, and its learning launch also
# writes every sample's query count to a per-pixel counter — C4: 19.5 GB of writes against the timed launch's 13.5 GB
# (profiles/r06/c4_learning_vs_timed.txt). Averaging it in made round 5's C4 summary read 15.0 GB. PMC_DISPATCH=timed
# (the default) keeps each pass's last `launches_per_step` x `steps` dispatches of the kernel (the bench line's timed
# steps; run the passes with --emulate-ranks 0); PMC_DISPATCH=all averages every dispatch.
import os  # noqa: E402
if os.environ.get("PMC_DISPATCH", "timed") == "timed" and line_json is not None:
    keep = int(round(line_json["roofline"].get("launches_per_step", 1) * line_json.get("steps", 1)))
    by_file = collections.defaultdict(list)
    for f, d in per:
        by_file[f].append(int(d))
    last = {f: set(sorted(ds)[-keep:]) for f, ds in by_file.items()}
    per = {dk: cs for dk, cs in per.items() if int(dk[1]) in last[dk[0]]}
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
