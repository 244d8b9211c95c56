#!/usr/bin/env python3
"""Attribute rocprofv3 output of bench.py to the named ops of the step plan.

Every batched step is one hipGraph launch whose dispatches run back to back, in plan order, on
the engine stream and end with the `commit` kernel. A window of len(plan) dispatches ending at a
k_commit dispatch whose kernel-name sequence equals the most common such window is one step.

  prof_ops.py trace    <run_kernel_trace.csv> <bench_ops.json> <out.csv>
      per-op kernel durations next to the bench's own HIP-event timings (the cross-check of
      the bench's roofline kernel duration)
  prof_ops.py piped    <run_kernel_trace.csv> <bench_ops.json> <out.csv> [<out_steps.json>]
      the same for a PIPELINED run (the bench's own configuration): the front graph (FlowLM + flow
      head, ending in k_front_commit) and the back graph (Mimi decode, ending in k_commit) run on
      two streams (two hardware queues), so their dispatches interleave in time. Each queue's
      dispatches are matched against its part of the plan; per step the front span, the back
      span, their overlap and the interval between consecutive back ends (the steady step)
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


def part_windows(names, part, closer):
    """Windows of len(part) dispatches ending at `closer` whose kernel names match the most common
    such window (one per replay of that part's graph)."""
    n = len(part)
    ends = [i for i, nm in enumerate(names) if closer in nm and i + 1 >= n]
    seqs = collections.Counter(tuple(names[i + 1 - n:i + 1]) for i in ends)
    if not seqs:
        return None, []
    ref, _ = seqs.most_common(1)[0]
    return ref, [i + 1 - n for i in ends if tuple(names[i + 1 - n:i + 1]) == ref]


def split_plan(plan):
    cut = plan.index("mimi.quant_upsample")
    return plan[:cut], plan[cut:]


def piped_attribution(rows, plan, queue_key):
    """{op: [row, ...]} over every replay of the front and back graphs, grouped by hardware queue;
    plus the per-part window lists [(part, [rows of one replay]), ...]."""
    front, back = split_plan(plan)
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r[queue_key]].append(r)
    per = collections.defaultdict(list)
    reps = {"front": [], "back": []}
    for q, rs in byq.items():
        names = [r["Kernel_Name"] for r in rs]
        for label, part, closer in (("front", front, "k_front_commit"), ("back", back, "k_commit")):
            _, wins = part_windows(names, part, closer)
            for w in wins:
                win = rs[w:w + len(part)]
                reps[label].append(win)
                for j, op in enumerate(part):
                    per[op].append(win[j])
    return per, reps


def cmd_piped(trace_path, ops_path, out_path, steps_path=None):
    ops = json.load(open(ops_path))
    plan = ops["plan"]
    event_us = {o["op"]: o for o in ops["ops"]}
    rows = [r for r in csv.DictReader(open(trace_path)) if is_engine(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per, reps = piped_attribution(rows, plan, "Queue_Id")
    if not reps["front"] or not reps["back"]:
        raise SystemExit("no front/back windows found")

    def dur(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0

    with open(out_path, "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(["op", "kernel", "calls", "rocprof_avg_us", "bench_event_avg_us", "flops", "bytes"])
        seen = set()
        for op in plan:
            if op in seen or op not in per:
                continue
            seen.add(op)
            d = [dur(r) for r in per[op]]
            e = event_us.get(op, {})
            wr.writerow([op, per[op][0]["Kernel_Name"].split("(")[0], len(d), round(sum(d) / len(d), 3),
                         round(e.get("avg_us", float("nan")), 3), e.get("flops", 0), e.get("bytes", 0)])

    def span(win):
        return int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])

    fr = sorted(span(w) for w in reps["front"])
    bk = sorted(span(w) for w in reps["back"])
    med = lambda v: sorted(v)[len(v) // 2] if v else None
    f_us = [(b - a) / 1000.0 for a, b in fr]
    b_us = [(b - a) / 1000.0 for a, b in bk]
    step = [(bk[i + 1][1] - bk[i][1]) / 1000.0 for i in range(len(bk) - 1)]
    ov = []
    for a, b in bk:  # overlap of each back replay with the front replays
        ov.append(sum(max(0, min(b, fb) - max(a, fa)) for fa, fb in fr) / 1000.0)
    busy_f = [sum(dur(r) for r in w) for w in reps["front"]]
    busy_b = [sum(dur(r) for r in w) for w in reps["back"]]
    out = {"front_replays": len(fr), "back_replays": len(bk),
           "front_span_us_median": med(f_us), "back_span_us_median": med(b_us),
           "front_kernel_busy_us_median": med(busy_f), "back_kernel_busy_us_median": med(busy_b),
           "back_overlapped_by_front_us_median": med(ov),
           "steady_step_us_median (back end to back end)": med(step)}
    print(json.dumps(out))
    if steps_path:
        json.dump(out, open(steps_path, "w"), indent=1)


def cmd_counters(cc_path, ops_path, counter, out_path):
    plan = json.load(open(ops_path))["plan"]
    disp = {}
    for r in csv.DictReader(open(cc_path)):
        if r["Counter_Name"] != counter or not is_engine(r["Kernel_Name"]):
            continue
        d = disp.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], 0.0, r.get("Queue_Id", "0")])
        d[1] += float(r["Counter_Value"])
    order = sorted(disp)
    names = [disp[i][0] for i in order]
    vals = [disp[i][1] for i in order]
    n = len(plan)
    per = collections.defaultdict(list)
    try:
        _, steps = step_windows(names, n)  # sequential engine: one stream, plan order
        for w in steps:
            for j in range(n):
                per[plan[j]].append(vals[w + j])
        nsteps = len(steps)
    except SystemExit:  # pipelined engine: front and back parts interleave; match each part alone
        rows = [{"Kernel_Name": disp[i][0], "v": disp[i][1], "q": disp[i][2]} for i in order]
        pr, reps = piped_attribution(rows, plan, "q")
        per = {op: [r["v"] for r in rs] for op, rs in pr.items()}
        nsteps = min(len(reps["front"]), len(reps["back"]))
    out = {"counter": counter, "steps": nsteps,
           "ops": {op: sum(v) / len(v) for op, v in per.items()}}
    json.dump(out, open(out_path, "w"), indent=1)
    print(f"{counter}: {nsteps} steps attributed")


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
    {"trace": cmd_trace, "piped": cmd_piped, "counters": cmd_counters, "traffic": cmd_traffic,
     "mfma": cmd_mfma}[cmd](*args)
