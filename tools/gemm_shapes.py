"""Per-shape breakdown of igemm dispatches from a rocprofv3 kernel_trace.csv (grid in workgroups)."""
import collections
import csv
import sys

def load(path, steps):
    g = collections.defaultdict(lambda: [0, 0.0, ""])
    for r in csv.DictReader(open(path)):
        if "igemm" not in r["Kernel_Name"]:
            continue
        key = (int(r["Grid_Size_X"]) // 256, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        g[key][0] += 1
        g[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        g[key][2] = f"lds={r['LDS_Block_Size']} vgpr={r['VGPR_Count']}"
    return {k: (v[0] / steps, v[1] / v[0] / 1e3, v[2]) for k, v in g.items()}

a = load(sys.argv[1], 3)
b = load(sys.argv[2], 3) if len(sys.argv) > 2 else None
for k, (n, us, info) in sorted(a.items(), key=lambda kv: -kv[1][0] * kv[1][1])[:25]:
    extra = f" | before {b[k][1]:8.1f}us" if b and k in b else ""
    print(f"grid={k[0]}x{k[1]}x{k[2]:<4} n/step={n:5.1f} avg={us:8.1f}us tot={n*us/1e3:6.2f}ms {info}{extra}")
