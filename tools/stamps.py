"""Front / back part timelines of a pipelined bench from the probe build's graph stamps.

PTTS_STAMPS=<file> (probe build) makes every part graph stamp s_memrealtime (100 MHz) at its start
and end; the engine writes `tag time` lines at destruction, tag = part << 8 | buffer << 1 | end.
This prints, over the steady calls (the middle of the run), the medians of each part's graph
duration and of the idle gap before its next graph, and how much of the front part's time the
back part overlapped:  python tools/stamps.py <file> [json out]
"""
import json
import sys

import numpy as np


def intervals(rows, part):
    out, start = [], None
    for tag, t in rows:
        if tag >> 8 != part:
            continue
        if tag & 1 == 0:
            start = t
        elif start is not None:
            out.append((start, t))
            start = None
    return np.array(out, dtype=np.float64) / 100.0  # us


def main():
    rows = [tuple(int(x) for x in ln.split()) for ln in open(sys.argv[1]) if ln.strip()]
    fr, bk = intervals(rows, 0), intervals(rows, 1)
    res = {}
    for name, iv in (("front", fr), ("back", bk)):
        n = len(iv)
        mid = iv[n // 4: 3 * n // 4]  # steady calls: drop warmup / tails
        dur = mid[:, 1] - mid[:, 0]
        gap = mid[1:, 0] - mid[:-1, 1]
        period = np.diff(mid[:, 0])
        res[name] = {"graphs": n, "dur_us_median": float(np.median(dur)), "dur_us_p10": float(np.percentile(dur, 10)),
                     "dur_us_p90": float(np.percentile(dur, 90)), "gap_us_median": float(np.median(gap)),
                     "gap_us_p90": float(np.percentile(gap, 90)), "period_us_median": float(np.median(period))}
    # overlap: per steady front graph, the fraction of its time some back graph ran
    n = len(fr)
    ov = []
    for s, e in fr[n // 4: 3 * n // 4]:
        o = np.clip(np.minimum(bk[:, 1], e) - np.maximum(bk[:, 0], s), 0, None).sum()
        ov.append(o / (e - s))
    res["front_overlapped_by_back_median"] = float(np.median(ov))
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
