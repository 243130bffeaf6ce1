"""Reduce two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --steps 1 --warmup 1`
to HBM bytes per step and per igemm_fast_kernel launch -> profiles/traffic_train_bf16_b64.json.
FETCH_SIZE / WRITE_SIZE are reported in KiB (x1024). gfx950 correction (MI355X_MICROARCH.md § HBM):
FETCH_SIZE counts half the bytes of 16-B/lane streaming reads -> x2; WRITE_SIZE is exact for 16-B/lane
stores. Both are L2 memory-side request
bytes (Infinity-Cache hits included), i.e. an upper bound on HBM bytes.
usage: traffic.py FETCH_DIR WRITE_DIR STEPS_IN_RUN [MODE]"""
import collections
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per_kernel = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(f[0])):
        name = r.get("Kernel_Name", "")
        val = float(r.get("Counter_Value", 0) or 0) * 1024.0  # KiB -> bytes
        m = re.search(r"\b(\w*(?:_kernel|Kernel|Functor|copyBuffer)\w*)", name)
        key = m.group(1) if m else name[:60]
        per_kernel[key][0] += val
        per_kernel[key][1] += 1
    return per_kernel


def main():
    fetch, write, steps = load(sys.argv[1]), load(sys.argv[2]), float(sys.argv[3])
    mode = sys.argv[4] if len(sys.argv) > 4 else "train"
    tot = sum(2 * v[0] for v in fetch.values()) + sum(v[0] for v in write.values())
    g_f, g_w = fetch.get("igemm_fast_kernel", [0, 0]), write.get("igemm_fast_kernel", [0, 0])
    launches = max(g_f[1], 1)
    out = {
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --mode {mode} --steps 1 --warmup 1 "
                  "(3 steps incl. the instrumented one); FETCH x2 (gfx950 correction)",
        "hbm_bytes_per_step": tot / steps,
        "igemm_fast_kernel": {"hbm_bytes_per_launch": (2 * g_f[0] + g_w[0]) / launches,
                              "launches_per_step": launches / steps,
                              "fetch_bytes_per_step": 2 * g_f[0] / steps, "write_bytes_per_step": g_w[0] / steps},
        "top_kernels_bytes_per_step": dict(sorted(
            ((k, (2 * fetch[k][0] + write.get(k, [0, 0])[0]) / steps) for k in fetch), key=lambda kv: -kv[1])[:15]),
    }
    path = os.path.join(REPO, "profiles", f"traffic_{mode}_bf16_b64.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_step", "igemm_fast_kernel")}))


if __name__ == "__main__":
    main()
