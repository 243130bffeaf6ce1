"""Per-queue kernel busy time in the last window of a rocprofv3 kernel trace (--kernel-trace --output-format csv):
sum of kernel durations per queue (ms per step) and the top kernels of each queue. The trunk's main stream, the
BERT stream and the weight-gradient stream are separate HIP streams (queues), so the busiest queue is the critical
path when the GPU is never idle. usage: python tools/queue_busy.py <kernel_trace.csv> [--last-ms 250] [--steps 3]
[--top 10]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-ms", type=float, default=250.0)
    ap.add_argument("--steps", type=float, default=3.0)
    ap.add_argument("--top", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    lo = end - a.last_ms * 1e6
    busy = collections.defaultdict(float)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    spans = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e <= lo:
            continue
        d = (e - max(s, lo)) / 1e6
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        busy[q] += d
        per[q][r["Kernel_Name"].split("(")[0][:60]] += d
        spans[q].append((max(s, lo), e, r["Kernel_Name"].split("(")[0][:40]))
    for q in sorted(busy, key=lambda k: -busy[k]):
        sp = sorted(spans[q])
        gaps = collections.defaultdict(float)  # idle time of this queue, by the kernel that ends the gap
        for (s0, e0, _), (s1, e1, k1) in zip(sp, sp[1:]):
            if s1 > e0 + 5000:  # > 5 us: a wait, not launch spacing
                gaps[k1] += (s1 - e0) / 1e6
        gsum = sum(gaps.values())
        print(f"queue {q}: busy-sum {busy[q] / a.steps:.2f} ms/step, waits > 5 us {gsum / a.steps:.2f} ms/step")
        for k, v in sorted(gaps.items(), key=lambda kv: -kv[1])[:4]:
            print(f"    wait {v / a.steps:7.2f} ms/step before {k}")
        for k, v in sorted(per[q].items(), key=lambda kv: -kv[1])[: a.top]:
            print(f"  {v / a.steps:9.2f} ms/step  {k}")


if __name__ == "__main__":
    main()
