"""Join a VCG_GEMM_LOG dispatch log with a rocprofv3 kernel_trace.csv (igemm launches pair up in
order; "wide ..." lines are the wide-tile engine's gemm_wide_kernel launches) and print time per GEMM shape.
usage: gemm_breakdown.py LOG TRACE_CSV [n_steps]"""
import collections
import csv
import sys

log = [l.strip() for l in open(sys.argv[1]) if l.strip()]
rows = [r for r in csv.DictReader(open(sys.argv[2])) if any(k in r["Kernel_Name"] for k in ("igemm", "gemm256", "wgrad_fast", "wgrad3x3_patch", "conv3x3_patch", "stem_patch", "rs1x1", "gemm_wide"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
if len(log) != len(rows):
    print(f"warning: {len(log)} log lines vs {len(rows)} igemm launches; pairing the tail")
    n = min(len(log), len(rows))
    log, rows = log[-n:], rows[-n:]
agg = collections.defaultdict(lambda: [0, 0.0])
for l, r in zip(log, rows):
    agg[l][0] += 1
    agg[l][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"igemm total {tot / steps / 1e3:.2f} ms/step")
for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[4]) if len(sys.argv) > 4 else 40]:
    f = dict(x.split("=") for x in k.split() if "=" in x)
    M, N, K = int(f["M"]), int(f["N"]), int(f["K"])
    z = int(f.get("z", 1))
    fl = 2.0 * M * N * K * (z if f.get("epi") != "2" else 1)
    print(f"{us / steps / 1e3:7.2f} ms/step  n={n / steps:4.1f} avg={us / n:8.1f}us  {fl / (us / n) / 1e6:6.1f}TF/s  {k}")
