"""Average PMC counter value per dispatch of the kernels matching a name filter, from a rocprofv3 --pmc output dir
(counter_collection.csv). usage: python tools/pmc_kernel.py <dir> [name-substring] [min-dispatch-index]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "igemm_fast_kernel"
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
vals = defaultdict(lambda: defaultdict(float))  # (kernel, counter) -> dispatch -> value
for f in files:
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if sub not in k:
            continue
        vals[(k[:90], row["Counter_Name"])][row["Dispatch_Id"]] += float(row["Counter_Value"])
for (k, c), per in sorted(vals.items()):
    v = list(per.values())
    print(f"{c:14s} n={len(v):3d} avg={sum(v) / len(v) / 1e6:10.2f} M  {k}")
