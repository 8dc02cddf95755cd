#!/usr/bin/env python3
"""Kernel concurrency in a rocprofv3 kernel trace: for each kernel name, the
fraction of its dispatches' time during which a dispatch of another kernel
was also running (on any queue), and the timeline's busy time vs the sum of
the kernel times.  usage: python tools/overlap.py <kernel_trace.csv> [substr]"""
import csv
import re
import sys


def main(path, only=None):
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:30]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "")))
    ev.sort()
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    # busy time of the union of intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    total = sum(e - s for s, e, _, _ in ev)
    print(f"span {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, sum of kernels {total / 1e6:.3f} ms, "
          f"queues {sorted(set(q for *_, q in ev))}")
    stats = {}
    for i, (s, e, n, q) in enumerate(ev):
        if only and only not in n:
            continue
        ov = 0
        for j, (s2, e2, n2, q2) in enumerate(ev):
            if j != i and s2 < e and e2 > s:
                ov = max(ov, min(e, e2) - max(s, s2))
        d = stats.setdefault(n, [0, 0, 0])
        d[0] += e - s
        d[1] += ov
        d[2] += 1
    for n, (t, ov, c) in sorted(stats.items(), key=lambda x: -x[1][0]):
        print(f"{n:28s} calls {c:4d}  time {t / 1e6:8.3f} ms  overlapped {ov / max(t, 1):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
