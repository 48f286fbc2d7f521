"""Idle-GPU breakdown of a rocprofv3 kernel trace (run_kernel_trace.csv): splits the trace into calls at
host gaps longer than --split-us, and for the last call prints the span, the kernel-busy time, and the idle
time grouped by the (previous kernel -> next kernel) pair, largest first.

    python tools/trace_gaps.py gpurun_out/<out>/profpy<i>/run_kernel_trace.csv [--split-us 2000]
"""
import argparse
import csv
import collections
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("mq::", "")
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split-us", type=float, default=2000.0)
    ap.add_argument("--call", type=int, default=-1, help="which call (index after splitting), default the last")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    calls, cur = [], [ks[0]]
    for k in ks[1:]:
        if (k[0] - cur[-1][1]) / 1e3 > a.split_us:
            calls.append(cur)
            cur = []
        cur.append(k)
    calls.append(cur)
    print(f"{len(calls)} calls: " + ", ".join(f"{(c[-1][1] - c[0][0]) / 1e6:.2f} ms/{len(c)}" for c in calls))
    c = calls[a.call]
    span = (c[-1][1] - c[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in c) / 1e3
    gaps = collections.defaultdict(lambda: [0, 0.0])
    kern = collections.defaultdict(lambda: [0, 0.0])
    for (s0, e0, n0), (s1, e1, n1) in zip(c, c[1:]):
        g = max(0, s1 - e0) / 1e3
        gaps[(n0, n1)][0] += 1
        gaps[(n0, n1)][1] += g
    for s, e, n in c:
        kern[n][0] += 1
        kern[n][1] += (e - s) / 1e3
    print(f"call {a.call}: span {span:.1f} us, kernels {len(c)}, busy {busy:.1f} us, idle {span - busy:.1f} us")
    print("kernels (count, total us, avg us):")
    for n, (cnt, t) in sorted(kern.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {cnt:6d} {t:10.1f} {t / cnt:8.2f}  {n}")
    print("idle between (count, total us, avg us):")
    for (n0, n1), (cnt, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {cnt:6d} {t:10.1f} {t / cnt:8.2f}  {n0} -> {n1}")


if __name__ == "__main__":
    main()
