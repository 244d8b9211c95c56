#!/usr/bin/env python3
"""Attribute rocprofv3 output of bench.py to the named ops of the step plan.

Every batched step is one hipGraph launch whose dispatches run back to back, in plan order, on
the engine stream and end with the `commit` kernel. A window of len(plan) dispatches ending at a
k_commit dispatch whose kernel-name sequence equals the most common such window is one step.

  prof_ops.py trace    <run_kernel_trace.csv> <bench_ops.json> <out.csv>
      per-op kernel durations next to the bench's own HIP-event timings (the cross-check of
      the bench's roofline kernel duration)
  prof_ops.py counters <run_counter_collection.csv> <bench_ops.json> <COUNTER> <out.json>
      per-op average of one PMC counter per launch
  prof_ops.py traffic  <fetch.json> <write.json> <out.json>
      HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB units -> bytes), the gfx950
      correction of MI355X_MICROARCH.md (FETCH_SIZE counts half of a 16 B/lane streaming read)
"""

import collections
import csv
import json
import sys


def is_engine(name):
    """Engine kernels live in namespace ptts; the runtime's copy kernels of the graphs' D2H nodes
    (frame to pinned host memory) are not ops of the plan."""
    return "ptts::" in name


def step_windows(names, n):
    windows = [i + 1 - n for i, nm in enumerate(names) if "k_commit" in nm and i + 1 >= n]
    seqs = collections.Counter(tuple(names[w:w + n]) for w in windows)
    if not seqs:
        raise SystemExit("no step windows found")
    ref_seq, _ = seqs.most_common(1)[0]
    return ref_seq, [w for w in windows if tuple(names[w:w + n]) == ref_seq]


def cmd_trace(trace_path, ops_path, out_path):
    ops = json.load(open(ops_path))
    plan = ops["plan"]
    event_us = {o["op"]: o for o in ops["ops"]}
    rows = [r for r in csv.DictReader(open(trace_path)) if is_engine(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(plan)
    ref_seq, steps = step_windows([r["Kernel_Name"] for r in rows], n)

    def dur(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0

    per = collections.defaultdict(list)
    for w in steps:
        for j in range(n):
            per[plan[j]].append(dur(rows[w + j]))
    with open(out_path, "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(["op", "kernel", "calls", "rocprof_avg_us", "bench_event_avg_us", "flops", "bytes"])
        seen = set()
        for j, op in enumerate(plan):
            if op in seen:
                continue
            seen.add(op)
            d = per[op]
            e = event_us.get(op, {})
            wr.writerow([op, ref_seq[j].split("(")[0], len(d), round(sum(d) / len(d), 3),
                         round(e.get("avg_us", float("nan")), 3), e.get("flops", 0), e.get("bytes", 0)])
    busy = [sum(dur(rows[w + j]) for j in range(n)) for w in steps]
    span = [(int(rows[w + n - 1]["End_Timestamp"]) - int(rows[w]["Start_Timestamp"])) / 1000.0 for w in steps]
    print(f"{len(steps)} steps of {n} ops; kernels busy {sum(busy) / len(busy):.1f} us/step, "
          f"first-start to last-end {sum(span) / len(span):.1f} us/step")


def cmd_counters(cc_path, ops_path, counter, out_path):
    plan = json.load(open(ops_path))["plan"]
    disp = {}
    for r in csv.DictReader(open(cc_path)):
        if r["Counter_Name"] != counter or not is_engine(r["Kernel_Name"]):
            continue
        d = disp.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], 0.0])
        d[1] += float(r["Counter_Value"])
    order = sorted(disp)
    names = [disp[i][0] for i in order]
    vals = [disp[i][1] for i in order]
    n = len(plan)
    _, steps = step_windows(names, n)
    per = collections.defaultdict(list)
    for w in steps:
        for j in range(n):
            per[plan[j]].append(vals[w + j])
    out = {"counter": counter, "steps": len(steps),
           "ops": {op: sum(v) / len(v) for op, v in per.items()}}
    json.dump(out, open(out_path, "w"), indent=1)
    print(f"{counter}: {len(steps)} steps attributed")


def cmd_traffic(fetch_path, write_path, out_path):
    fe = json.load(open(fetch_path))["ops"]
    wr = json.load(open(write_path))["ops"]
    ops = {}
    for op in fe:
        fb = 2.0 * fe[op] * 1024.0
        wb = wr.get(op, 0.0) * 1024.0
        ops[op] = {"fetch_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py (KB units, FETCH x2 "
                         "gfx950 correction), attributed per op by tools/prof_ops.py",
               "ops": ops}, open(out_path, "w"), indent=1)
    print(f"traffic for {len(ops)} ops")


def cmd_mfma(busy_path, gui_path, op_stats_path, out_path):
    """Per-op MFMA utilisation from one --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass:
    busy = SIMD cycles the matrix core was busy, summed over the 1,024 SIMDs (MI355X_MICROARCH.md:
    32 per v_mfma_f32_32x32x16_bf16, 64 per v_mfma_f32_32x32x2_f32, so flops/64 for f32 32x32x2);
    util_peak_clock = busy / (1024 SIMDs x 2.4 GHz x duration) (the 157.3 TF fp32 peak's clock);
    util_eff_clock uses the dispatch's own clock GRBM_GUI_ACTIVE / 8 XCDs (reads high on short
    dispatches). Durations are the rocprofv3 per-dispatch averages of op_stats.csv."""
    busy = json.load(open(busy_path))["ops"]
    gui = json.load(open(gui_path))["ops"]
    stats = {r["op"]: r for r in csv.DictReader(open(op_stats_path))}
    ops = {}
    for op, b in busy.items():
        if op not in stats or b <= 0:
            continue
        us = float(stats[op]["rocprof_avg_us"])
        fl = float(stats[op]["flops"] or 0)
        cyc_eff = gui.get(op, 0.0) / 8.0
        ops[op] = {"mfma_busy_cycles": b, "flops_over_64": fl / 64.0, "rocprof_avg_us": us,
                   "util_peak_clock": round(b / (1024 * 2.4e9 * us * 1e-6), 4),
                   "util_eff_clock": round(b / (1024 * cyc_eff), 4) if cyc_eff > 0 else None,
                   "eff_clock_ghz": round(cyc_eff / (us * 1e3), 3)}
    json.dump({"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass of bench.py, attributed "
                         "per op by tools/prof_ops.py", "ops": ops}, open(out_path, "w"), indent=1)
    print(f"mfma utilisation for {len(ops)} ops")


if __name__ == "__main__":
    cmd, args = sys.argv[1], sys.argv[2:]
    {"trace": cmd_trace, "counters": cmd_counters, "traffic": cmd_traffic, "mfma": cmd_mfma}[cmd](*args)
