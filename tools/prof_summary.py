"""Summarise rocprofv3 output of a bench.py run into the kernel families bench.py reports.

    python tools/prof_summary.py <kernel_trace.csv> [--fetch counter_collection.csv]
                                 [--write counter_collection.csv] [--steps-total N]
                                 [-o out.json]

Families (same bracketing as bench.py's HIP events):
  conv3x3  = conv3x3_kernel / conv_hr_kernel / conv_lr_kernel / conv_kg_kernel dispatches + their
             split-K epilogue dispatches, per conv call
  wgrad3x3 = wgrad3x3_kernel / wgrad_bf16_kernel / wgrad_dma_kernel dispatches (bias grad fused), per call
Traffic per call = 2 * FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md "HBM [CDNA4]": gfx950
FETCH_SIZE reports half of the bytes of wide coalesced reads; WRITE_SIZE is exact for
16-B stores and float atomics), summed over the family's dispatches / calls.
"""
import argparse
import csv
import glob
import os
import json
from collections import defaultdict


def family(name):
    if ("conv3x3_kernel" in name or "conv_hr_kernel" in name or "conv_lr_kernel" in name or
            "conv_kg_kernel" in name):
        return "conv3x3", True
    if "conv_splitk_epilogue" in name:
        return "conv3x3", False
    if "wgrad3x3_kernel" in name or "wgrad_bf16_kernel" in name or "wgrad_dma_kernel" in name:
        return "wgrad3x3", True
    if "wgrad_slab_reduce" in name:
        return "wgrad3x3", False
    return None, False


def group_traffic(path_fetch, path_write, launches_json):
    """HBM bytes per call of each (family, bound) roofline group of bench.py: the last N
    conv / wgrad calls of each --pmc pass (N = the instrumented step's calls, every step
    launches the same sequence) aligned one to one with bench.py's launch list; a call =
    its main kernel + the split epilogue / slab reduction that follows it."""
    launches = json.load(open(launches_json))
    n = len(launches)
    # the --pmc pass's last dispatches are bench.py's one-stream (isolated) step: its calls in
    # its own order (launches_json + ".iso"); the result is re-ordered to the timed step's calls
    # (the kernel trace's order) by matching identical calls in sequence
    order = launches
    if os.path.exists(launches_json + ".iso"):
        order = json.load(open(launches_json + ".iso"))
        assert len(order) == n, (len(order), n)

    def calls(path, counter):
        path = _resolve(path, "counter_collection.csv")
        rows = []
        with open(path) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                fm, is_call = family(r["Kernel_Name"])
                if fm:
                    rows.append((int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0),
                                 fm, is_call, float(r["Counter_Value"])))
        rows.sort()
        out = []
        for _, fm, is_call, v in rows:
            if is_call or not out:
                out.append([fm, 0.0])
            out[-1][1] += v
        return out[-n:]

    fe, wr = calls(path_fetch, "FETCH_SIZE"), calls(path_write, "WRITE_SIZE")
    assert len(fe) == n and len(wr) == n, (len(fe), len(wr), n)
    groups = defaultdict(lambda: dict(calls=0, hbm_bytes=0.0, alg_bytes=0.0))
    for L, (f1, fv), (f2, wv) in zip(order, fe, wr):
        assert L["group"].split("/")[0] == f1 == f2, (L["group"], f1, f2)
        g = groups[L["group"]]
        g["calls"] += 1
        g["hbm_bytes"] += (2.0 * fv + wv) * 1024.0
        g["alg_bytes"] += L["bytes"]
    out = {k: dict(calls=v["calls"], hbm_bytes_per_call=v["hbm_bytes"] / v["calls"],
                   alg_bytes_per_call=v["alg_bytes"] / v["calls"],
                   traffic_over_alg=v["hbm_bytes"] / max(v["alg_bytes"], 1.0))
           for k, v in groups.items()}
    per_iso = [(L, (2.0 * fv + wv) * 1024.0) for L, (_, fv), (_, wv) in zip(order, fe, wr)]
    if order is launches:
        return out, per_iso
    # (family, resolution, FLOPs): the one-stream step runs a few calls in another form (the
    # final pass's fromRGB weight gradient outside the conv epilogue), same shape, other bytes
    key = lambda L: (L["group"].split("/")[0], L["H"], L["flops"])
    pool = defaultdict(list)
    for L, b in per_iso:
        pool[key(L)].append(b)
    per_call = [(L, pool[key(L)].pop(0)) for L in launches]
    return out, per_call


def trace_calls(path, n):
    """Durations (ns) of the last n conv / wgrad calls of a kernel trace in dispatch (= host
    issue) order, a call = its main kernel + the split epilogue / slab reduction after it."""
    path = _resolve(path, "kernel_trace.csv")
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            fm, is_call = family(r["Kernel_Name"])
            if fm:
                rows.append((int(r["Dispatch_Id"]), is_call,
                             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    out = []
    for _, is_call, d in rows:
        if is_call or not out:
            out.append(0)
        out[-1] += d
    return out[-n:]


def per_resolution(per_call, durations):
    """North star's HBM view per resolution (conv + weight-gradient launches): PMC-measured
    HBM bytes (FETCH x2 + WRITE) over the kernel-trace durations of the same calls, next to
    the algorithmic bytes."""
    rows = defaultdict(lambda: dict(calls=0, hbm_bytes=0.0, alg_bytes=0.0, ns=0))
    for (L, hb), ns in zip(per_call, durations):
        r = rows[L["H"]]
        r["calls"] += 1
        r["hbm_bytes"] += hb
        r["alg_bytes"] += L["bytes"]
        r["ns"] += ns
    return [dict(res=H, calls=r["calls"], ms=round(r["ns"] / 1e6, 4),
                 hbm_mb=round(r["hbm_bytes"] / 1e6, 2), alg_mb=round(r["alg_bytes"] / 1e6, 2),
                 hbm_gbps=round(r["hbm_bytes"] / max(r["ns"], 1), 1),
                 hbm_frac=round(r["hbm_bytes"] / max(r["ns"], 1) / 8000.0, 4))
            for H, r in sorted(rows.items())]


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def gap_stats(path):
    """Idle time of the GPU between consecutive kernels (same queue order, by start time):
    sum of positive gaps and the number of kernels, over the whole trace."""
    path = _resolve(path, "kernel_trace.csv")
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    ev.sort()
    gaps, last_end, small = 0, None, 0
    for a, b in ev:
        if last_end is not None and a > last_end:
            g = a - last_end
            if g < 1_000_000:      # ignore host-side pauses (> 1 ms) between phases
                gaps += g
                small += 1
        last_end = b if last_end is None else max(last_end, b)
    return dict(kernels=len(ev), gap_ms=gaps / 1e6, gaps_counted=small,
                avg_gap_us=gaps / 1e3 / max(small, 1))


def steady_state(path, steps=3):
    """Launches and kernel time per step over the last `steps` steps of the trace (delimited
    by the adam_dev_kernel launches, two per step): the whole-trace stats include the setup
    (buffer allocation fills, copies) and the warm-up, which a per-step count must not."""
    path = _resolve(path, "kernel_trace.csv")
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                       short(r["Kernel_Name"]).split("<")[0]))
    ev.sort()
    ad = [i for i, e in enumerate(ev) if e[3] == "adam_dev_kernel"]
    if len(ad) < 2 * steps + 1:
        return None
    w = ev[ad[-1 - 2 * steps] + 1:ad[-1] + 1]
    per = defaultdict(lambda: [0, 0.0])
    queues = defaultdict(int)
    for s, e, q, n in w:
        per[n][0] += 1
        per[n][1] += (e - s) / 1e3
        queues[q] += 1
    return dict(steps=steps, ms_per_step=(w[-1][1] - w[0][0]) / 1e6 / steps,
                launches_per_step=len(w) / steps,
                launches_per_step_by_queue={q: c / steps for q, c in sorted(queues.items())},
                kernels={n: dict(per_step=c / steps, us_per_step=round(t / steps, 1))
                         for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][0])})


def read_trace(path):
    path = _resolve(path, "kernel_trace.csv")
    fam = defaultdict(lambda: dict(ns=0, calls=0, dispatches=0))
    per_kernel = defaultdict(lambda: [0, 0])
    total = 0
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            total += d
            k = per_kernel[short(n)]
            k[0] += d
            k[1] += 1
            fm, is_call = family(n)
            if fm:
                fam[fm]["ns"] += d
                fam[fm]["dispatches"] += 1
                fam[fm]["calls"] += int(is_call)
    return fam, per_kernel, total


def _resolve(path, suffix):
    if os.path.isdir(path):
        hits = sorted(glob.glob(os.path.join(path, "**", "*" + suffix), recursive=True))
        if not hits:
            raise SystemExit(f"no *{suffix} under {path}")
        return hits[0]
    return path


def read_counter(path, counter):
    path = _resolve(path, "counter_collection.csv")
    """-> ({family: summed value}, {family: calls}, {short kernel name: [sum, dispatches]})"""
    out, calls = defaultdict(float), defaultdict(int)
    per = defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            fm, is_call = family(r["Kernel_Name"])
            v = float(r["Counter_Value"])
            out[fm or "other"] += v
            calls[fm or "other"] += int(is_call)
            k = per[short(r["Kernel_Name"])]
            k[0] += v
            k[1] += 1
    return out, calls, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("-o", "--out")
    ap.add_argument("--launches", help="bench.py PG_BENCH_LAUNCHES dump of the PMC runs")
    ap.add_argument("--config", default="stage8_b4_bf16",
                    help="bench.py workload key the profiled run used (bench.py matches it)")
    a = ap.parse_args()
    fam, per_kernel, total = read_trace(a.trace)
    res = {"config": a.config, "total_kernel_ms": total / 1e6, "families": {},
           "top_kernels": [], "gaps": gap_stats(a.trace), "steady_state": steady_state(a.trace)}
    for k, v in fam.items():
        res["families"][k] = dict(total_ms=v["ns"] / 1e6, calls=v["calls"],
                                  dispatches=v["dispatches"],
                                  avg_us_per_call=v["ns"] / 1e3 / max(v["calls"], 1))
    if a.fetch and a.write:
        fe, fcalls, fper = read_counter(a.fetch, "FETCH_SIZE")
        wr, _, wper = read_counter(a.write, "WRITE_SIZE")
        for k, v in res["families"].items():
            # FETCH_SIZE / WRITE_SIZE are reported in KiB
            by = (2.0 * fe.get(k, 0.0) + wr.get(k, 0.0)) * 1024.0
            v["pmc_calls"] = fcalls.get(k, 0)
            v["hbm_bytes_per_call"] = by / max(fcalls.get(k, 0), 1)
        res["pmc_per_kernel_kib"] = {n: dict(fetch_x2=2 * f[0] / f[1],
                                             write=wper.get(n, [0, 1])[0] / max(wper.get(n, [0, 1])[1], 1),
                                             dispatches=f[1])
                                     for n, f in sorted(fper.items(), key=lambda kv: -kv[1][0])[:25]}
        if a.launches:
            res["groups"], per_call = group_traffic(a.fetch, a.write, a.launches)
            try:
                res["per_resolution"] = per_resolution(per_call, trace_calls(a.trace, len(per_call)))
                res["per_resolution_note"] = (
                    "conv + weight-gradient calls of one step: hbm_mb = PMC FETCH_SIZE x2 + "
                    "WRITE_SIZE (separate --pmc passes), ms = the same calls' kernel-trace "
                    "durations (two streams: calls overlap, so a row's GB/s is per call time)")
            except (AssertionError, KeyError, ValueError) as e:
                res["per_resolution_error"] = str(e)
        res["pmc_note"] = ("bytes/call = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 summed over the "
                           "family's dispatches of the PMC passes / the family's calls; "
                           "calibrate with adam_kernel: 28 B per parameter (4 fp32 reads, 3 writes)")
    for n, (ns, c) in sorted(per_kernel.items(), key=lambda kv: -kv[1][0])[:25]:
        res["top_kernels"].append(dict(kernel=n, total_ms=ns / 1e6, calls=c,
                                       avg_us=ns / 1e3 / c, pct=100.0 * ns / total))
    s = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
