"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (tools/gpu_check.sh pmcq)."""
import collections
import csv
import glob
import sys


def main():
    for d in sys.argv[1:]:
        f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
        if not f:
            print(d, "no counters")
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        cnt = collections.Counter()
        for r in csv.DictReader(open(f[0])):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            k = k.replace("void ", "")
            if not any(s in k for s in ("conv", "wgrad", "pack", "unpool", "pixnorm", "rgb")):
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[(k, r["Counter_Name"])] += 1
        print(d)
        for k, c in agg.items():
            n = max(cnt[(k, name)] for name in c)
            print(f"  {k[:90]}  dispatches={n}")
            print("    " + "  ".join(f"{name.replace('SQ_', '')}={v / n:.4g}" for name, v in c.items()))
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                print("    fractions of wave cycles: " + "  ".join(
                    f"{name.replace('SQ_', '')}={c[name] / wc:.2f}"
                    for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                 "SQ_WAIT_INST_LDS") if name in c))
            if c.get("SQ_INSTS_LDS"):
                print(f"    LDS bank conflict cycles per LDS instr: "
                      f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_INSTS_LDS']:.2f}")


if __name__ == "__main__":
    main()
