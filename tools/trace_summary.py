"""Per-step kernel time from a rocprofv3 kernel_trace.csv: sum of durations by kernel name, divided by the number of
adamw launches (one per train step). usage: python tools/trace_summary.py run_kernel_trace.csv [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("vcg::", "")
    n = n.split("(")[0].split("<")[0][:60]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
steps = max(agg["adamw_kernel"][0], 1)
print(f"steps {steps}, total kernel time {sum(v[1] for v in agg.values()) / steps / 1e3:.2f} ms/step")
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{t / steps / 1e3:7.2f} ms/step {c / steps:6.1f} calls avg {t / c:8.1f} us  {n}")
