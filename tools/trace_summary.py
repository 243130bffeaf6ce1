"""Per-step kernel time from a rocprofv3 kernel_trace.csv: sum of durations by kernel name over the kernels that start
between the end of the first adamw launch and the end of the last one (one adamw per train step), divided by the
number of steps in that window -- the model's set-up (weight synthesis, flat-buffer copies) and the first step stay
outside. usage: python tools/trace_summary.py run_kernel_trace.csv [top]"""
import collections
import csv
import sys


def name_of(r):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("vcg::", "")
    return n.split("(")[0].split("<")[0][:60]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ad = [int(r["End_Timestamp"]) for r in rows if name_of(r) == "adamw_kernel"]
if len(ad) >= 2:
    lo, hi, steps = ad[0], ad[-1], len(ad) - 1
else:  # (no complete step: everything, one step)
    lo, hi, steps = -1, 1 << 62, 1
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    if not lo < int(r["Start_Timestamp"]) <= hi:
        continue
    n = name_of(r)
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(f"steps {steps} (kernels after the first step's adamw through the last adamw), "
      f"total kernel time {sum(v[1] for v in agg.values()) / steps / 1e3:.2f} ms/step")
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{t / steps / 1e3:7.2f} ms/step {c / steps:6.1f} calls avg {t / c:8.1f} us  {n}")
