"""Per-stream view of a rocprofv3 kernel trace of bench.py (one steady-state step).

    python tools/trace_streams.py <run_kernel_trace.csv> [--steps N] [--top K]

Splits the trace into steps at the largest idle gaps... simpler: takes the last `--span`
fraction; reports per Queue_Id / Stream_Id the busy time, kernel count, and the top kernels
of each stream, plus the union busy time (any stream running) over the window.
"""
import argparse
import csv
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3, help="timed steps in the profiled run")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    ev = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                       r["Stream_Id"], r["Kernel_Name"]))
    ev.sort()
    # steady state: the adam_dev_kernel launches mark the end of each half-step (2 per step)
    ad = [i for i, e in enumerate(ev) if "adam_dev_kernel" in e[4]]
    # window = between the end of the 2*(k+1)-th-from-last adam of G and the last one
    i1 = ad[-1]
    i0 = ad[-1 - 2 * a.steps]
    w = ev[i0 + 1:i1 + 1]
    t0, t1 = w[0][0], w[-1][1]
    span = (t1 - t0) / 1e6
    print(f"window: {len(w)} kernels, {span:.3f} ms over {a.steps} steps = {span / a.steps:.3f} ms/step")
    per = defaultdict(lambda: [0, 0, defaultdict(lambda: [0, 0])])
    for s, e, q, st, n in w:
        k = f"q{q}/s{st}"
        per[k][0] += e - s
        per[k][1] += 1
        per[k][2][short(n)][0] += e - s
        per[k][2][short(n)][1] += 1
    # union busy
    busy, cur_s, cur_e = 0, None, None
    for s, e, *_ in w:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"union busy {busy / 1e6 / a.steps:.3f} ms/step, idle {(span * 1e6 - busy) / 1e6 / a.steps:.3f}")
    for k, (ns, c, kk) in sorted(per.items(), key=lambda kv: -kv[1][0]):
        print(f"\n== {k}: {ns / 1e6 / a.steps:.3f} ms/step busy, {c / a.steps:.1f} kernels/step")
        for n, (t, cc) in sorted(kk.items(), key=lambda kv: -kv[1][0])[:a.top]:
            print(f"   {t / 1e6 / a.steps:7.3f} ms  {cc / a.steps:5.1f}x  {t / cc / 1e3:7.1f} us  {n}")


if __name__ == "__main__":
    main()
