"""Per-spec median GPU durations from tools/kprof_ab.sh traces: the kernels of one kbench
spec are the launches between its first and last call; kbench runs 3 warm-up + --iters timed
calls per spec in order, so consecutive dispatches are grouped by spec in launch order.

    python tools/kprof_table.py SPEC... -- DIR [DIR ...]
"""
import csv
import glob
import os
import sys


def segments(d):
    """The spec segments of a trace: runs of conv / wgrad launches between kbench's set-up
    kernels (randn, fills), in launch order."""
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    segs, cur = [], []
    for r in rows:
        n = r["Kernel_Name"]
        if "elementwise" in n or "distribution" in n or "fill" in n.lower():
            if cur:
                segs.append(cur)
                cur = []
            continue
        cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if cur:
        segs.append(cur)
    return segs


def main():
    argv = sys.argv[1:]
    cut = argv.index("--")
    specs, dirs = argv[:cut], argv[cut + 1:]
    calls = int(os.environ.get("KPROF_CALLS", 13))   # 3 warm-up + --iters 10 (kprof_ab.sh)
    for d in dirs:
        segs = segments(d)
        print(f"== {d}: {len(segs)} segments for {len(specs)} specs")
        for s, seg in zip(specs, segs):
            per = len(seg) // calls
            seg = seg[3 * per:]
            # one call = `per` dispatches: its span from the first start to the last end
            spans = sorted((seg[j + per - 1][2] - seg[j][1]) / 1000 for j in range(0, len(seg), per))
            names = sorted({n.replace("(anonymous namespace)::", "").replace("void ", "")
                            .split("((")[0].split("(")[0][:60] for n, *_ in seg})
            print(f"  {s:24s} x{per} span med {spans[len(spans) // 2]:7.2f} us  min {spans[0]:7.2f}  {names}")

if __name__ == "__main__":
    main()
