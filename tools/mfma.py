"""Reduce one rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE) of
`bench.py --steps 1 --warmup 1` to the matrix-core utilisation of each kernel -> profiles/mfma_<mode>_bf16_b64.json.

mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the share of SIMD-cycles in
which the matrix pipe was busy while the kernel ran (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is summed over the 8
XCDs; SQ_VALU_MFMA_BUSY_CYCLES counts pipe cycles per MFMA, e.g. 16 per v_mfma_f32_16x16x32_bf16).
Cross-check: `flop_implied_busy` = the kernel's algorithmic FLOPs / 1024 (16x16x32 bf16: 16 384 FLOP per 16-cycle
MFMA) when bench.py's GEMM timing records are available.
usage: mfma.py PMC_DIR STEPS_IN_RUN MODE"""
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
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        name = r.get("Kernel_Name", "")
        m = re.search(r"\b(\w*(?:_kernel|Kernel|Functor|copyBuffer)\w*)", name)
        key = m.group(1) if m else name[:60]
        per[key][r.get("Counter_Name", "")] += float(r.get("Counter_Value", 0) or 0)
        disp[key].add(r.get("Dispatch_Id", ""))
    return per, {k: len(v) for k, v in disp.items()}


def main():
    per, ndisp = load(sys.argv[1])
    steps, mode = float(sys.argv[2]), sys.argv[3]
    out = {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (one pass), "
                     f"bench.py --mode {mode} --steps 1 --warmup 1 ({int(steps)} steps incl. the instrumented one)",
           "formula": "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)"}
    tot_busy = tot_cyc = 0.0
    kern = {}
    for k, c in per.items():
        busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), c.get("GRBM_GUI_ACTIVE", 0.0)
        simd_cycles = gui / 8.0 * 1024.0
        tot_busy += busy
        tot_cyc += simd_cycles
        kern[k] = {"mfma_busy_frac": round(busy / simd_cycles, 4) if simd_cycles else None,
                   "mfma_busy_cycles_per_step": busy / steps, "gpu_cycles_per_step": gui / 8.0 / steps,
                   "dispatches": ndisp.get(k, 0)}
    out["whole_step"] = {"mfma_busy_frac": round(tot_busy / tot_cyc, 4) if tot_cyc else None}
    top = sorted(kern.items(), key=lambda kv: -kv[1]["gpu_cycles_per_step"])[:15]
    out["kernels"] = dict(top)
    if "igemm_fast_kernel" in kern:
        out["igemm_fast_kernel"] = kern["igemm_fast_kernel"]
    path = os.path.join(REPO, "profiles", f"mfma_{mode}_bf16_b64.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"whole_step": out["whole_step"], "igemm_fast_kernel": out.get("igemm_fast_kernel")}))


if __name__ == "__main__":
    main()
