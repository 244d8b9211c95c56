"""Per-op intervals of the front / back graphs from the probe build's op stamps.

PTTS_STAMPS=<file> PTTS_STAMP_OPS=1 (probe build): every part graph stamps s_memrealtime (100 MHz)
at its start, twice back to back (the cost of one stamp launch), ahead of each op and at its end.
An op's interval is stamp(op i + 1) - stamp(op i): the op's kernel plus one stamp launch and the
launch gaps around it, so `net_us` = interval - the back-to-back stamp interval. Medians over the
steady graphs (the middle half of the run):  python tools/op_stamps.py <file> [json out]
"""
import json
import sys

import numpy as np


def main():
    names = {0: {}, 1: {}}
    rows = []
    for ln in open(sys.argv[1]):
        if ln.startswith("#"):
            _, p, i, name = ln.split(maxsplit=3)
            names[int(p)][int(i)] = name.strip()
        elif ln.strip():
            rows.append(tuple(int(x) for x in ln.split()))
    res = {}
    for part in (0, 1):
        graphs, cur = [], None
        for tag, t in rows:
            if tag < 0x10000:
                if tag >> 8 != part:
                    continue
                if tag & 1 == 0:
                    cur = {"start": t, "ops": {}}
                elif cur is not None:
                    cur["end"] = t
                    graphs.append(cur)
                    cur = None
            elif (tag >> 12) & 1 == part and cur is not None:
                cur["ops"][tag & 0xFFF] = t
        graphs = [g for g in graphs if len(g["ops"]) == len(names[part]) + 2]
        if not graphs:
            continue
        mid = graphs[len(graphs) // 4: 3 * len(graphs) // 4]
        n = len(names[part])
        iv = np.zeros((len(mid), n))
        cal = np.zeros(len(mid))
        for gi, g in enumerate(mid):
            o = g["ops"]
            cal[gi] = o[0xFFF] - o[0xFFE]
            for i in range(n):
                nxt = o[i + 1] if i + 1 < n else g["end"]
                iv[gi, i] = nxt - o[i]
        iv /= 100.0
        cal /= 100.0
        c = float(np.median(cal))
        med = np.median(iv, axis=0)
        dur = np.median([(g["end"] - g["start"]) / 100.0 for g in mid])
        res["front" if part == 0 else "back"] = {
            "graphs": len(mid), "graph_us": float(dur), "stamp_us": c, "sum_interval_us": float(med.sum()),
            "ops": [{"i": i, "op": names[part][i], "interval_us": round(float(med[i]), 2),
                     "net_us": round(float(med[i] - c), 2)} for i in range(n)]}
    for k, v in res.items():
        print(f"{k}: graph {v['graph_us']:.1f} us, stamp {v['stamp_us']:.2f} us, sum of intervals "
              f"{v['sum_interval_us']:.1f} us over {v['graphs']} graphs")
        for o in v["ops"]:
            print(f"  {o['i']:3d} {o['op']:32s} {o['interval_us']:7.2f} {o['net_us']:7.2f}")
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
