#!/usr/bin/env python3
"""Per-launch start delays of one steady pipelined step, from a rocprofv3 --kernel-trace of
bench.py (the front graph on the engine stream, the back graph on the second stream).

  launch_delay.py <run_kernel_trace.csv> <bench_ops.json> <out.json>

Steps are found as in pipe_trace.py (per queue, windows of the part's plan length ending in the
part's last kernel, most common name sequence). For every launch position of each part, over the
steady windows (medians):
  gap_us   its start minus the end of the launch before it on the same queue (the first launch of
           a window: minus the end of the previous window's last launch) = dispatch latency +
           any wait for room on the CUs;
  dur_us   its duration;
  back_busy  (front launches) the fraction of windows in which a back-part kernel was running when
           the launch started.
The table says where the step's critical path (the front chain, in frame-pair mode) loses time:
launches that start late beside the back part's workgroups, or that run long."""

import bisect
import collections
import csv
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pipe_trace import windows  # noqa: E402


def main(trace, ops_path, out):
    plan = json.load(open(ops_path))["plan"]
    nf = plan.index("mimi.quant_upsample")
    fend = "k_front_commit" if plan[nf - 1] == "front_commit" else "k_flow_head"
    parts = {"front": (plan[:nf], fend), "back": (plan[nf:], "k_commit")}
    rows = list(csv.DictReader(open(trace)))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    byq = collections.defaultdict(list)
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        byq[r[qkey]].append(r)
    for rs in byq.values():
        rs.sort(key=lambda r: r["s"])
    found = {}
    for part, (names, last) in parts.items():
        best = None
        for q, rs in byq.items():
            ws = windows(rs, len(names), last)
            if ws and (best is None or len(ws) > len(best[2])):
                best = (q, rs, ws)
        found[part] = best
    # back-part kernel intervals (for "was the back part running when this front launch started")
    back_iv = []
    if found["back"]:
        _, rs, ws = found["back"]
        for w in ws:
            back_iv += [(r["s"], r["e"]) for r in rs[w:w + len(parts["back"][0])]]
    back_iv.sort()
    starts = [s for s, _ in back_iv]

    def back_running(t):
        i = bisect.bisect_right(starts, t)
        return any(s <= t < e for s, e in back_iv[max(0, i - 64):i])

    res = {}
    for part, (names, _) in parts.items():
        if not found[part]:
            res[part] = None
            continue
        _, rs, ws = found[part]
        ws = ws[2:-1] if len(ws) > 4 else ws
        gaps, durs, busy = (collections.defaultdict(list) for _ in range(3))
        spans = []
        for w in ws:
            seg = rs[w:w + len(names)]
            prev_end = rs[w - 1]["e"] if w > 0 else seg[0]["s"]
            spans.append((seg[-1]["e"] - seg[0]["s"]) / 1e3)
            for i, r in enumerate(seg):
                gaps[i].append((r["s"] - prev_end) / 1e3)
                durs[i].append((r["e"] - r["s"]) / 1e3)
                if part == "front":
                    busy[i].append(1.0 if back_running(r["s"]) else 0.0)
                prev_end = r["e"]
        med = statistics.median
        table = []
        for i, nm in enumerate(names):
            row = {"i": i, "op": nm, "gap_us": round(med(gaps[i]), 2), "gap_max_us": round(max(gaps[i]), 2),
                   "dur_us": round(med(durs[i]), 2)}
            if part == "front":
                row["back_busy"] = round(sum(busy[i]) / len(busy[i]), 2)
            table.append(row)
        res[part] = {"windows": len(ws), "span_us_median": round(med(spans), 1),
                     "sum_gap_us": round(sum(r["gap_us"] for r in table), 1),
                     "sum_dur_us": round(sum(r["dur_us"] for r in table), 1), "launches": table}
    json.dump(res, open(out, "w"), indent=1)
    for part in ("front", "back"):
        p = res[part]
        if not p:
            continue
        print(f"{part}: {p['windows']} windows, span {p['span_us_median']} us = launches {p['sum_dur_us']} "
              f"+ gaps {p['sum_gap_us']}")
        for r in sorted(p["launches"], key=lambda r: -r["gap_us"])[:10]:
            print("   late:", r)


if __name__ == "__main__":
    main(*sys.argv[1:4])
