"""Static instruction mix of kernels in a gfx950 assembly file.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S conv.hip -o /tmp/conv.s
    python tools/isa_stats.py /tmp/conv.s <kernel-name substring> [...]
"""
import re
import sys
from collections import Counter


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur and line.startswith("\t") and not line.startswith(("\t.", "\t;")):
            body.append(line.split()[0])
        elif cur and line.startswith(".Lfunc_end"):
            yield cur, body
            cur = None
    if cur:
        yield cur, body


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    for name, ops in kernels(path):
        if pats and not any(p in name for p in pats):
            continue
        c = Counter()
        for op in ops:
            if "mfma" in op:
                c["mfma"] += 1
            elif op.startswith("ds_"):
                c["ds"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["vmem"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            elif op.startswith("v_"):
                c["valu"] += 1
            else:
                c["other"] += 1
        print(f"{name[:100]}\n   total {len(ops)}  " + "  ".join(f"{k} {v}" for k, v in c.most_common()))


if __name__ == "__main__":
    main()
