#!/usr/bin/env python3
"""Pipelined-step timeline from a rocprofv3 --kernel-trace of bench.py (pipelined engine).

Splits the engine kernels by queue (front graph on the engine stream, back graph on the second
stream), finds the steady-state steps (front windows ending at k_front_commit (or k_flow_head when the commit runs inside it), back windows
ending at k_commit), and reports per-part spans and per-op durations overlapped, next to the
isolated HIP-event times of bench_ops.json. Usage:
  overlap_trace.py <run_kernel_trace.csv> <bench_ops.json>"""

import collections
import csv
import json
import sys


def main(trace, ops_path):
    ops = json.load(open(ops_path))
    plan = ops["plan"]
    iso = {o["op"]: o["avg_us"] for o in ops.get("ops", [])}
    cut = plan.index("mimi.quant_upsample")
    front, back = plan[:cut], plan[cut:]
    rows = [r for r in csv.DictReader(open(trace)) if "ptts::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_q = collections.defaultdict(list)
    for r in rows:
        by_q[r["Queue_Id"]].append(r)
    res = {}
    for q, rs in by_q.items():
        names = [r["Kernel_Name"] for r in rs]
        fend = "k_front_commit" if front[-1] == "front_commit" else "k_flow_head"
        for part, seq, last in (("front", front, fend), ("back", back, "k_commit")):
            n = len(seq)
            wins = [i + 1 - n for i, nm in enumerate(names) if last in nm and i + 1 >= n]
            if not wins:
                continue
            per = collections.defaultdict(list)
            spans = []
            for w in wins[2:]:  # skip warmup-ish first windows
                spans.append((int(rs[w + n - 1]["End_Timestamp"]) - int(rs[w]["Start_Timestamp"])) / 1e3)
                for j in range(n):
                    per[seq[j]].append((int(rs[w + j]["End_Timestamp"]) - int(rs[w + j]["Start_Timestamp"])) / 1e3)
            if spans:
                res[part] = (q, spans, per)
    for part in ("front", "back"):
        if part not in res:
            continue
        q, spans, per = res[part]
        spans.sort()
        print(f"{part}: queue {q}, {len(spans)} steps, span median {spans[len(spans) // 2]:.1f} us")
        agg = collections.defaultdict(lambda: [0.0, 0.0])
        for op, d in per.items():
            key = ".".join(p for p in op.split(".") if not (p[0] == "l" and p[1:].isdigit()))
            mult = sum(1 for x in (front if part == "front" else back) if x == op)
            agg[key][0] += sum(d) / len(d) * mult
            agg[key][1] += iso.get(op, 0.0) * mult
        tot = [0.0, 0.0]
        for k, (ov, isol) in sorted(agg.items(), key=lambda x: -x[1][0]):
            print(f"  {k:28s} overlapped {ov:7.1f}  isolated {isol:7.1f}")
            tot[0] += ov
            tot[1] += isol
        print(f"  {'sum':28s} overlapped {tot[0]:7.1f}  isolated {tot[1]:7.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
