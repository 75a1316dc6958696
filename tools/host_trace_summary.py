#!/usr/bin/env python3
"""Copy-engine timeline of the host-resident pipeline (tools/host_bench --host-path-trace under rocprofv3
--memory-copy-trace --kernel-trace): the trace's copies and kernels grouped into calls (host_bench leaves 20 ms
of idle between calls), and per call its span (first host-to-device copy start -> last copy end), the time the
host-to-device copies are busy (union of their intervals), the idle gaps between them, the device-to-host and
kernel busy times. Usage: host_trace_summary.py <rocprofv3 output dir> [<prefix>]"""
import csv
import glob
import json
import os
import sys


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main():
    d = sys.argv[1]
    pre = sys.argv[2] if len(sys.argv) > 2 else ""
    copies = list(csv.DictReader(open(glob.glob(os.path.join(d, f"{pre}*memory_copy_trace.csv"))[0])))
    kernels = list(csv.DictReader(open(glob.glob(os.path.join(d, f"{pre}*kernel_trace.csv"))[0])))
    ev = [("h2d" if "HOST_TO_DEVICE" in c["Direction"] else "d2h", int(c["Start_Timestamp"]), int(c["End_Timestamp"]))
          for c in copies]
    ev += [("kernel", int(k["Start_Timestamp"]), int(k["End_Timestamp"])) for k in kernels]
    ev.sort(key=lambda x: x[1])
    calls, cur = [], []
    for e in ev:  # a new call after 5 ms of nothing
        if cur and e[1] - max(x[2] for x in cur) > 5_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
    if cur:
        calls.append(cur)
    for i, c in enumerate(calls):
        h2d = [(s, e) for k, s, e in c if k == "h2d"]
        if len(h2d) < 4:
            continue  # warm-up / build traffic
        span = max(e for _, _, e in c) - min(s for s, _ in h2d)
        hs = sorted(h2d)
        gaps = [b[0] - a[1] for a, b in zip(hs, hs[1:]) if b[0] > a[1]]
        out = {
            "call": i, "h2d_copies": len(h2d), "span_ms": span / 1e6,
            "h2d_busy_ms": union(h2d) / 1e6, "h2d_busy_frac": union(h2d) / span,
            "h2d_copy_ms_mean": sum(e - s for s, e in h2d) / len(h2d) / 1e6,
            "h2d_idle_gap_ms_mean": (sum(gaps) / len(gaps) / 1e6) if gaps else 0.0,
            "d2h_busy_ms": union([(s, e) for k, s, e in c if k == "d2h"]) / 1e6,
            "kernel_busy_ms": union([(s, e) for k, s, e in c if k == "kernel"]) / 1e6,
        }
        print(json.dumps(out))


if __name__ == "__main__":
    main()
