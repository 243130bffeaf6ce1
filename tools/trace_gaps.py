"""GPU idle time inside a window of a rocprofv3 kernel trace (--kernel-trace --output-format csv):
busy = union of all kernel intervals (any queue), idle = span - busy; plus the gap histogram between consecutive
kernels of the busiest queue. Used to size what launch-side changes (fewer launches, graphs) could recover.

usage: python tools/trace_gaps.py <kernel_trace.csv> [--last-ms 200] [--skip-ms 0]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-ms", type=float, default=0.0, help="only the last N ms of the trace (0: all)")
    ap.add_argument("--skip-ms", type=float, default=0.0, help="drop the first N ms of the trace")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id") or r.get("Stream_Id") or "0",
           r["Kernel_Name"]) for r in rows]
    ks.sort()
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    lo = t0 + int(a.skip_ms * 1e6)
    if a.last_ms:
        lo = max(lo, t1 - int(a.last_ms * 1e6))
    ks = [k for k in ks if k[0] >= lo]
    span = max(k[1] for k in ks) - ks[0][0]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    by_q = {}
    for k in ks:
        by_q.setdefault(k[2], []).append(k)
    q, qk = max(by_q.items(), key=lambda kv: len(kv[1]))
    gaps = [b[0] - a_[1] for a_, b in zip(qk, qk[1:]) if b[0] >= a_[1]]
    gaps.sort()
    med = gaps[len(gaps) // 2] if gaps else 0
    print(f"window {span / 1e6:.2f} ms, {len(ks)} kernels on {len(by_q)} queues; GPU busy {busy / 1e6:.2f} ms, idle "
          f"{(span - busy) / 1e6:.2f} ms ({100 * (span - busy) / span:.1f} %)")
    print(f"busiest queue {q}: {len(qk)} kernels, gaps between consecutive kernels: median {med / 1e3:.1f} us, "
          f"sum {sum(gaps) / 1e6:.2f} ms, > 20 us: {sum(1 for g in gaps if g > 20000)} (sum "
          f"{sum(g for g in gaps if g > 20000) / 1e6:.2f} ms)")


if __name__ == "__main__":
    main()
