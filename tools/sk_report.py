"""Per-call GPU time of each tools/sk_probe.py spec from its rocprofv3 kernel trace: the calls
of one spec are the conv launches between two set-up phases (randn / elementwise kernels);
per call = the sum of its launches' durations / 10 (a split-K epilogue launch included).

    python tools/sk_report.py TRACE.csv PROBE_STDOUT.txt"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    labels = [l.strip() for l in open(sys.argv[2]) if l.startswith(("sk ", "old"))]
    segs, cur = [], []
    for r in rows:
        n = r["Kernel_Name"]
        if "elementwise" in n or "distribution" in n or "fill" in n.lower() or "copy" in n.lower():
            if cur:
                segs.append(cur)
                cur = []
            continue
        cur.append((n.replace("void ", "").split("(")[0].replace("(anonymous namespace)::", ""),
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    if cur:
        segs.append(cur)
    for lab, seg in zip(labels, segs):
        names = sorted(set(n.split("<")[0] for n, _ in seg))
        print(f"{lab:36s} {sum(t for _, t in seg) / 10 / 1e3:7.1f} us/call  {len(seg) // 10} launch(es)  {' + '.join(names)}")


if __name__ == "__main__":
    main()
