#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace (`--kernel-trace --output-format csv`): per dispatch its start / end
relative to the first dispatch of the timed step, duration, and overlap with the previous trace launch; the
union of the trace-kernel intervals (the step's trace wall time) against the sum of their durations.

usage: python scripts/trace_overlap.py gpurun_out/bandtrace/b8g_c4 [--last-step]
The directory is searched for *kernel_trace.csv. With --last-step only the dispatches after the last
k_accumulate gap of more than 20 ms before the final burst are shown (the bench's timed step)."""
from __future__ import annotations

import argparse
import csv
import sys
from pathlib import Path


def load(d: Path):
    files = sorted(d.rglob("*kernel_trace.csv"))
    if not files:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name") or r.get("KernelName") or ""
                s = int(r.get("Start_Timestamp") or r.get("BeginNs"))
                e = int(r.get("End_Timestamp") or r.get("EndNs"))
                rows.append((s, e, name.split("(")[0].replace("void ", ""), r.get("Queue_Id") or r.get("Stream_Id") or ""))
    rows.sort()
    return rows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=1, help="timed steps at the end of the trace (bench --steps)")
    a = ap.parse_args()
    rows = [r for r in load(Path(a.dir)) if r[2].startswith(("k_trace", "k_accumulate", "k_render"))]
    # split into draws: a draw starts with a trace launch after a gap (> 5 ms) with no dispatch in flight
    draws, cur, end = [], [], 0
    for r in rows:
        if cur and r[0] > end + 5_000_000:
            draws.append(cur)
            cur = []
        cur.append(r)
        end = max(end, r[1])
    if cur:
        draws.append(cur)
    for draw in draws[-a.steps:]:
        t0 = draw[0][0]
        print(f"{'kernel':<42} {'queue':>5} {'start ms':>9} {'end ms':>9} {'dur ms':>8} {'overlap prev ms':>15}")
        prev_end = None
        union, dur_sum, iv = 0, 0, []
        for s, e, n, q in draw:
            ov = "" if prev_end is None or not n.startswith("k_trace") else f"{max(0, prev_end - s) / 1e6:.2f}"
            print(f"{n[:42]:<42} {q:>5} {(s - t0) / 1e6:9.2f} {(e - t0) / 1e6:9.2f} {(e - s) / 1e6:8.2f} {ov:>15}")
            if n.startswith("k_trace"):
                prev_end = e
                dur_sum += e - s
                iv.append((s, e))
        iv.sort()
        cs, ce = None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    union += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        if cs is not None:
            union += ce - cs
        wall = max(e for _, e, _, _ in draw) - t0
        print(f"draw wall {wall / 1e6:.2f} ms; trace launches {len(iv)}: union {union / 1e6:.2f} ms, sum of durations "
              f"{dur_sum / 1e6:.2f} ms")
    return 0


if __name__ == "__main__":
    sys.exit(main())
