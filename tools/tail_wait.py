"""What the main stream waits for at the end of a train step: for each sumsq_part_kernel launch (the gradient-norm
reduction before AdamW, main stream) in a rocprofv3 kernel trace, the main queue's idle gap before it and the kernels
of the other queues that run inside that gap. usage: python tools/tail_wait.py <kernel_trace.csv> [main_queue]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["q"] = r.get("Queue_Id") or r.get("Stream_Id")
    r["k"] = r["Kernel_Name"].split("(")[0][:48]
rows.sort(key=lambda r: r["s"])
mainq = sys.argv[2] if len(sys.argv) > 2 else "1"
for i, r in enumerate(rows):
    if r["q"] != mainq or "sumsq_part" not in r["k"]:
        continue
    prev = max((x for x in rows[:i] if x["q"] == mainq and x["e"] <= r["s"]), key=lambda x: x["e"], default=None)
    if prev is None:
        continue
    g0, g1 = prev["e"], r["s"]
    print(f"main idle {(g1 - g0) / 1e3:8.1f} us before sumsq (after {prev['k']})")
    inside = [x for x in rows if x["q"] != mainq and x["e"] > g0 and x["s"] < g1]
    for x in inside[-12:]:
        print(f"   q{x['q']} {(min(x['e'], g1) - max(x['s'], g0)) / 1e3:8.1f} us of {(x['e'] - x['s']) / 1e3:8.1f}  {x['k']}")
