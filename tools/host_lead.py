"""Host lead per kernel from a rocprofv3 --kernel-trace --hip-runtime-trace of bench.py.

    python tools/host_lead.py <dir with run_kernel_trace.csv + run_hip_api_trace.csv> [--steps N]

For every kernel of the last N steps (delimited by the adam_dev_kernel launches, two per step):
lead = GPU start - end of the host API call that enqueued it.  A main-stream gap with a lead
near zero is the host arriving late (launch-bound); a gap with a large lead is a dependency
wait on the device.  Also prints the host time of the API calls by function per step.
"""
import argparse
import csv
import os
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--dump", action="store_true", help="print every main-stream kernel")
    a = ap.parse_args()
    api = {}
    calls = []
    for r in csv.DictReader(open(os.path.join(a.dir, "run_hip_api_trace.csv"))):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        api[int(r["Correlation_Id"])] = (s, e, r["Function"])
        calls.append((s, e, r["Function"]))
    ev = []
    for r in csv.DictReader(open(os.path.join(a.dir, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                   int(r["Correlation_Id"]), short(r["Kernel_Name"])))
    ev.sort()
    ad = [i for i, e in enumerate(ev) if "adam_dev_kernel" in e[4]]
    w = ev[ad[-1 - 2 * a.steps] + 1:ad[-1] + 1]
    t0, t1 = w[0][0], w[-1][1]
    nq = defaultdict(int)
    for e in w:
        nq[e[2]] += 1
    main = max(nq, key=nq.get)
    prev = None
    late = wait = 0.0
    nlate = 0
    for s, e, q, cid, n in w:
        if q != main:
            continue
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        prev = e
        h = api.get(cid)
        lead = (s - h[1]) / 1e3 if h else float("nan")
        if gap > 2.0:
            if lead < 15.0:
                late += gap
                nlate += 1
            else:
                wait += gap
        if a.dump:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {gap:7.1f} lead {lead:9.1f} {n}")
    span = (t1 - t0) / 1e6 / a.steps
    print(f"window {span:.3f} ms/step; main-stream gaps > 2 us: host-late (lead < 15 us) "
          f"{late / 1e3 / a.steps:.3f} ms/step in {nlate / a.steps:.0f} gaps, device waits "
          f"{wait / 1e3 / a.steps:.3f} ms/step")
    per = defaultdict(lambda: [0, 0.0])
    for s, e, f in calls:
        if t0 <= s <= t1:
            per[f][0] += 1
            per[f][1] += (e - s) / 1e3
    tot = sum(v[1] for v in per.values())
    print(f"host API time in the window: {tot / 1e3 / a.steps:.3f} ms/step")
    for f, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:12]:
        print(f"  {f:40s} {c / a.steps:7.1f}/step {t / 1e3 / a.steps:7.3f} ms/step {t / c:6.1f} us")


if __name__ == "__main__":
    main()
