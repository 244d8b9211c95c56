#!/usr/bin/env python3
"""Front/back interference in pipelined stepping, from a rocprofv3 kernel trace of bench.py
(pipelined: the front graph on the engine stream, the back graph on the second stream).

  pipe_trace.py <run_kernel_trace.csv> <bench_ops.json> <out.json>

Dispatches are split by queue; on each queue a window of the part's plan length ending at that
part's last kernel (k_front_commit / k_commit) whose name sequence is the most common one is one
step of that part. Per op: mean duration in the pipelined run next to the op timed alone
(bench_ops.json), and per part: mean span (first start to last end), summed kernel time and
summed gaps, so stretched kernels (shared CUs / memory) and stretched gaps (dispatch) separate."""

import collections
import csv
import json
import sys


def windows(rows, n, last):
    names = [r["Kernel_Name"] for r in rows]
    ends = [i + 1 - n for i, nm in enumerate(names) if last in nm and i + 1 >= n]
    seqs = collections.Counter(tuple(names[w:w + n]) for w in ends)
    if not seqs:
        return []
    ref, _ = seqs.most_common(1)[0]
    return [w for w in ends if tuple(names[w:w + n]) == ref]


def main(trace, ops_path, out):
    ops = json.load(open(ops_path))
    plan = ops["plan"]
    alone = {o["op"]: o["avg_us"] for o in ops["ops"]}
    nf = plan.index("mimi.quant_upsample")  # the front part ends in front_commit or in the chain
    fend = "k_front_commit" if plan[nf - 1] == "front_commit" else "k_flow_head"
    parts = {"front": (plan[:nf], fend), "back": (plan[nf:], "k_commit")}
    rows = list(csv.DictReader(open(trace)))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r[qkey]].append(r)
    res = {"queues": {q: len(v) for q, v in byq.items()}}
    for part, (names, last) in parts.items():
        best = None
        for q, rs in byq.items():
            rs.sort(key=lambda r: int(r["Start_Timestamp"]))
            ws = windows(rs, len(names), last)
            if ws and (best is None or len(ws) > len(best[1])):
                best = (rs, ws)
        if best is None:
            res[part] = None
            continue
        rs, ws = best
        ws = ws[2:]  # skip warmup-ish first windows
        dur = collections.defaultdict(list)
        spans, busy, gaps = [], [], []
        for w in ws:
            seg = rs[w:w + len(names)]
            s0, e1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
            spans.append((e1 - s0) / 1e3)
            b = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
            busy.append(b)
            gaps.append(spans[-1] - b)
            for nm, r in zip(names, seg):
                dur[nm].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        mean = lambda v: sum(v) / len(v)
        per = [{"op": nm, "pipelined_us": round(mean(dur[nm]), 2), "alone_us": round(alone.get(nm, 0.0), 2)}
               for nm in dict.fromkeys(names)]
        res[part] = {"steps": len(ws), "span_us": round(mean(spans), 1), "kernel_us": round(mean(busy), 1),
                     "gap_us": round(mean(gaps), 1), "alone_sum_us": round(sum(alone.get(n, 0.0) for n in names), 1),
                     "ops": per}
    json.dump(res, open(out, "w"), indent=1)
    for part in ("front", "back"):
        p = res[part]
        if p:
            print(part, {k: p[k] for k in ("steps", "span_us", "kernel_us", "gap_us", "alone_sum_us")})
            worst = sorted(p["ops"], key=lambda o: o["alone_us"] - o["pipelined_us"])[:6]
            print("  most stretched:", [(o["op"], o["alone_us"], o["pipelined_us"]) for o in worst])


if __name__ == "__main__":
    main(*sys.argv[1:4])
