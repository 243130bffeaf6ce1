"""Side-by-side per-kernel totals of two rocprofv3 kernel-stats CSVs (A, B): ms per run, calls, delta.
usage: python tools/prof_diff.py A.csv B.csv"""
import csv
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        out[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6)
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
names = sorted(set(a) | set(b), key=lambda n: -max(a.get(n, (0, 0))[1], b.get(n, (0, 0))[1]))
ta, tb = sum(v[1] for v in a.values()), sum(v[1] for v in b.values())
print(f"{'kernel':44s} {'A ms':>9s} {'B ms':>9s} {'B-A':>8s}  calls A/B   (total A {ta:.1f} B {tb:.1f} ms)")
for n in names[:45]:
    ca, ma = a.get(n, (0, 0.0))
    cb, mb = b.get(n, (0, 0.0))
    print(f"{n[:44]:44s} {ma:9.2f} {mb:9.2f} {mb - ma:8.2f}  {ca}/{cb}")
