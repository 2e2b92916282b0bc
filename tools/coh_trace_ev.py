#!/usr/bin/env python3
"""Walker events of a GG_COH_TRACE_EV dump: per served (packet, position)
event the shader-clock cycles of the request and of the publish, and the
hand-off latency (the packet's publish at the previous position -> its serve
decision here), over every block and over the critical (last-ending) block
of each launch.  usage: coh_trace_ev.py prefix"""
import json
import sys

import numpy as np


def main():
    pre = sys.argv[1]
    m = json.load(open(pre + ".meta"))
    WB, n, E = m["walk_blocks"], m["ev_launches"], m["ev_max"]
    ev = np.fromfile(pre + ".ev", np.uint64).reshape(n, 2, WB, E * 4 + 4)
    wk = np.fromfile(pre + ".walk", np.uint64).reshape(m["launches"], 2, WB, 8)
    req, pub, hand, idle_first, crit_rows = [], [], [], [], []
    per_stage = {0: {"req": [], "pub": [], "hand": [], "span": [], "events": [], "first_wait": []},
                 1: {"req": [], "pub": [], "hand": [], "span": [], "events": [], "first_wait": []}}
    for L in range(n):
        for s in (0, 1):
            w = wk[m["ev_first"] + L, s]
            full = (w[:, 0] > 0) & (w[:, 1] > 0)
            if not full.any():
                continue
            crit = int(np.argmax(np.where(full, w[:, 1].astype(np.float64), -1)))
            for b in range(WB):
                e = ev[L, s, b]
                k = int(min(e[0], E))
                if k == 0:
                    continue
                rec = e[4:4 + 4 * k].reshape(k, 4).astype(np.float64)
                info = e[4:4 + 4 * k].reshape(k, 4)[:, 3]
                pk = (info & 0xFFFF).astype(np.int64); pos = ((info >> 16) & 0xFF).astype(np.int64)
                r_ = rec[:, 1] - rec[:, 0]; p_ = rec[:, 2] - rec[:, 1]       # decision -> forward, forward -> queue updated
                h_ = []
                order = np.argsort(rec[:, 0])
                last_pub = {}
                for j in order:
                    if pk[j] in last_pub:
                        h_.append(rec[j, 0] - last_pub[pk[j]])
                    last_pub[pk[j]] = rec[j, 1]
                st = per_stage[s]
                if b == crit:
                    st["req"].extend(r_); st["pub"].extend(p_); st["hand"].extend(h_)
                    st["events"].append(k)
                    t0 = float(e[1])                                 # loop start (_w1)
                    st["span"].append(float(e[2]) - t0)               # loop cycles (_w2 - _w1)
                    st["first_wait"].append(rec[:, 0].min() - t0)
    out = {}
    for s in (0, 1):
        st = per_stage[s]
        f = lambda v: round(float(np.mean(v)), 1) if len(v) else None
        out["xy"[s]] = {"crit_loop_cycles": f(st["span"]), "crit_events": f(st["events"]),
                        "decision_to_forward_cycles": f(st["req"]), "forward_to_updated_cycles": f(st["pub"]),
                        "handoff_cycles(prev forward -> decision)": f(st["hand"]),
                        "handoff_p50": float(np.median(st["hand"])) if st["hand"] else None,
                        "first_serve_after_loop_start": f(st["first_wait"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
