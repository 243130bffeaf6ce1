"""rocprofv3 --stats layout (Name, Calls, TotalDurationNs, AverageNs, Percentage) from a kernel_trace.csv, for runs
traced without --stats (tools/gpu_profile.sh's one-stream pass). usage: trace_to_stats.py TRACE_CSV OUT_CSV"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: [0, 0])
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("vcg::", "")
    n = n.split("(")[0].split("<")[0]
    agg[n][0] += 1
    agg[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = sum(v[1] for v in agg.values())
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([n, c, t, t / c, round(100.0 * t / tot, 4)])
