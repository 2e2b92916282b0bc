#!/usr/bin/env python3
"""Analyse a GG_COH_TRACE dump (gg_coherent_run with GG_COH_TRACE=n and
GG_COH_TRACE_OUT=prefix): per launch index, the step kernel's and the two
walkers' spans (s_memrealtime, 10 ns ticks), the gaps between them, and the
phase breakdown of the tile / walker block that ended each kernel last
(s_memtime deltas scaled to that tile's own realtime span).
usage: coh_trace.py prefix [first_launch]"""
import json
import sys

import numpy as np

W = 32          # kTrStep


def main():
    pre = sys.argv[1]
    L0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    m = json.load(open(pre + ".meta"))
    n, T, WB = m["launches"], m["tiles"], m["walk_blocks"]
    st = np.fromfile(pre + ".step", np.uint64).reshape(n, T, W).astype(np.float64)
    wk = np.fromfile(pre + ".walk", np.uint64).reshape(n, 2, WB, 8).astype(np.float64)
    used = np.nonzero(st[:, :, 0].max(axis=1) > 0)[0]
    used = used[used >= L0]
    tick = 10.0
    phases = ["prologue", "self", "inbox", "trace", "publish", "writeback"]
    sub = {"self": ["narv", "gather", "order", "qload", "requests", "recv_store"],
           "inbox": ["in_gather_order", "in_handlers"],
           "publish": ["pub_build", "pub_order", "pub_qload", "pub_requests", "pub_seglists"]}
    keys = ["entry", "exit"] + phases + sum(sub.values(), []) + \
        ["span_step", "span_x", "span_y", "gap_sx", "gap_xy", "gap_ys", "crit_na", "crit_ni", "crit_sent",
         "dir_msg_ns", "l2_msg_ns", "crit_dir_msgs", "crit_l2_msgs",
         "h_dget", "h_sharers", "h_dram", "h_send", "h_fifo", "h_shwords", "h_pre", "h_run", "h_eopen",
         "tiles_working", "clock_ghz", "qend", "crit_has_self", "crit_has_inbox", "crit_has_pub"]
    acc = {k: [] for k in keys}
    wacc = {s: {k: [] for k in ("entry", "staging", "loop", "handoff", "exit", "events", "n", "npos", "blocks")}
            for s in (0, 1)}
    prev_end = None
    for L in used:
        s = st[L]
        live = s[:, 0] > 0
        k0, k1 = s[live, 0].min(), s[live, 1].max()
        acc["span_step"].append((k1 - k0) * tick)
        qend = bool((s[live, 2] == 0).all())
        acc["qend"].append(float(qend))
        if prev_end is not None:
            acc["gap_ys"].append((k0 - prev_end) * tick)
        c = int(np.argmax(np.where(live, s[:, 1], -1)))
        r = s[c]
        if r[2] > 0:
            v = int(r[9])
            acc["tiles_working"].append(float((s[:, 9] > 0).sum()))
            span = (r[1] - r[0]) * tick
            cyc = r[8] - r[2]
            f = span / cyc if cyc > 0 else 0.0                     # ns per memtime cycle for this tile
            if f > 0: acc["clock_ghz"].append(1.0 / f)
            acc["entry"].append((r[0] - k0) * tick)
            mt = [r[2], r[3], r[4], r[5], r[6], r[7], r[8]]
            for k, a, b in zip(phases, mt[:-1], mt[1:]):
                acc[k].append((b - a) * f)
            acc["exit"].append(0.0)
            na, ni, ns = v & 0xFFFF, (v >> 16) & 0xFFFF, v >> 32
            acc["crit_na"].append(na); acc["crit_ni"].append(ni); acc["crit_sent"].append(ns)
            acc["crit_has_self"].append(float(na > 0)); acc["crit_has_inbox"].append(float(ni + na > 0))
            acc["crit_has_pub"].append(float(r[16] > 0))
            if r[10] > 0:
                sp = [r[3], r[10], r[11], r[12], r[13], r[15], r[4]]
                for k, a, b in zip(sub["self"], sp[:-1], sp[1:]):
                    acc[k].append((b - a) * f)
            if r[14] > 0:
                acc["in_gather_order"].append((r[14] - r[4]) * f); acc["in_handlers"].append((r[5] - r[14]) * f)
                hn = int(r[22]); nd, nl = hn & 0xFFFFFFFF, hn >> 32
                acc["crit_dir_msgs"].append(nd); acc["crit_l2_msgs"].append(nl)
                if nd: acc["dir_msg_ns"].append(r[20] * f / nd)
                for i, k in enumerate(("h_dget", "h_sharers", "h_dram", "h_send", "h_fifo", "h_shwords", "h_pre", "h_run", "h_eopen")):
                    acc[k].append(r[23 + i] * f)
                if nl: acc["l2_msg_ns"].append(r[21] * f / nl)
            if r[16] > 0:
                sp = [r[6], r[16], r[17], r[18], r[19], r[7]]
                for k, a, b in zip(sub["publish"], sp[:-1], sp[1:]):
                    acc[k].append((b - a) * f)
        end = k1
        for stage in (0, 1):
            w = wk[L, stage]
            wl = w[:, 0] > 0
            if not wl.any():
                continue
            a0 = w[wl, 0].min()
            full = wl & (w[:, 1] > 0)
            (acc["gap_sx"] if stage == 0 else acc["gap_xy"]).append((a0 - end) * tick)
            e1 = w[full, 1].max() if full.any() else w[wl, 0].max()
            (acc["span_x"] if stage == 0 else acc["span_y"]).append((e1 - a0) * tick)
            wacc[stage]["blocks"].append(float(full.sum()))
            if full.any():
                b = int(np.argmax(np.where(full, w[:, 1], -1)))
                q = w[b]
                span = (q[1] - q[0]) * tick
                cyc = q[5] - q[2]
                f = span / cyc if cyc > 0 else 0.0
                wacc[stage]["entry"].append((q[0] - a0) * tick)
                wacc[stage]["staging"].append((q[3] - q[2]) * f)
                wacc[stage]["loop"].append((q[4] - q[3]) * f)
                wacc[stage]["handoff"].append((q[5] - q[4]) * f)
                wacc[stage]["exit"].append(0.0)
                wacc[stage]["n"].append(float(int(q[6]) & 0xFFFFFFFF)); wacc[stage]["npos"].append(float(int(q[6]) >> 32))
                wacc[stage]["events"].append(q[7])
            end = e1
        prev_end = end
    mean = lambda v: round(float(np.mean(v)), 1) if v else None
    out = {"launches": len(used)}
    out["step"] = {k: mean(v) for k, v in acc.items()}
    out["step_note"] = "phase ns are means over the launches where the critical tile ran that phase"
    for s in (0, 1):
        out["walk_" + "xy"[s]] = {k: mean(v) for k, v in wacc[s].items()}
    per = lambda k: (np.sum(acc[k]) / len(used)) if acc[k] else 0.0
    out["per_launch_ns"] = {k: round(per(k), 1) for k in ("span_step", "span_x", "span_y", "gap_sx", "gap_xy", "gap_ys")}
    out["per_launch_ns_total"] = round(sum(out["per_launch_ns"].values()), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
