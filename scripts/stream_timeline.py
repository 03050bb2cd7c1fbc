#!/usr/bin/env python3
"""Per-stream timeline of a rocprofv3 kernel trace (run_results.db): how often the task streams
overlap, and what the other streams do while one stream idles.

    python scripts/stream_timeline.py gpurun_out/x/run_results.db [--md out.md] [--gap-ms 2]

Reports, per HIP stream (or HW queue when the trace has no stream ids): dispatches, busy time
(union of its kernels' intervals), the longest idle gaps inside the traced window, and the
chip-level concurrency split (time with 0 / 1 / 2+ streams running a kernel).  A stream that
idles for long gaps while another stream runs a dense kernel sequence (a graph replay) is the
signature of serialised streams.
"""
import argparse
import sqlite3
from collections import defaultdict


def _cols(c, table):
    return [r[1] for r in c.execute(f"pragma table_info({table})")]


def load(db, by=None):
    c = sqlite3.connect(db)
    cols = _cols(c, "kernels")
    name = "name" if "name" in cols else "kernel_name"
    key = by if by in cols else next((k for k in ("stream_id", "queue_id") if k in cols), None)
    sel = f"select {name}, start, end, {key or 0} from kernels order by start"
    rows = [(n, s, e, q) for n, s, e, q in c.execute(sel).fetchall()]
    qmap = {}
    if "stream_id" in cols and "queue_id" in cols:
        for st, q, n in c.execute("select stream_id, queue_id, count(*) from kernels group by stream_id, queue_id"):
            qmap.setdefault(st, []).append((q, n))
    return rows, key or "none", cols, qmap


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--md", default=None)
    ap.add_argument("--gap-ms", type=float, default=2.0)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--by", default=None, help="group by this column (stream_id / queue_id)")
    ap.add_argument("--window", nargs=2, type=int, default=None, metavar=("T0_NS", "T1_NS"),
                    help="keep only kernels inside [T0, T1] (trace clock; bench.py ARB_BENCH_MARKS=1 prints "
                         "the timed region's bounds)")
    ap.add_argument("--skip-ms", type=float, default=0.0,
                    help="drop the first N ms of the trace (warm-up captures) when no --window is given")
    a = ap.parse_args()
    rows, key, cols, qmap = load(a.db, a.by)
    if a.window:
        w0, w1 = a.window
        inside = [(n, max(s, w0), min(e, w1), q) for n, s, e, q in rows if e > w0 and s < w1]
        if not inside:
            print(f"window {w0}..{w1} misses the trace ({rows[0][1]}..{rows[-1][2]}): clocks differ; "
                  "falling back to --skip-ms")
        else:
            rows = inside
    elif a.skip_ms > 0:
        cut = rows[0][1] + int(a.skip_ms * 1e6)
        rows = [(n, max(s, cut), e, q) for n, s, e, q in rows if e > cut]
    t0, t1 = min(r[1] for r in rows), max(r[2] for r in rows)
    wall = (t1 - t0) / 1e6
    per = defaultdict(list)
    names = defaultdict(list)
    for n, s, e, q in rows:
        per[q].append((s, e))
        names[q].append((s, e, n))
    lines = [f"kernel trace: {len(rows)} dispatches over {wall:.1f} ms, grouped by `{key}`", "",
             f"| stream | dispatches | busy ms | busy % | gaps > {a.gap_ms:.1f} ms | longest gaps (ms) |",
             "|---|---:|---:|---:|---:|---|"]
    unions = {}
    for q, iv in sorted(per.items(), key=lambda kv: -len(kv[1])):
        u = union(iv)
        unions[q] = u
        busy = sum(e - s for s, e in u) / 1e6
        gaps = sorted(((u[i + 1][0] - u[i][1]) / 1e6, u[i][1]) for i in range(len(u) - 1))
        big = [g for g in gaps if g[0] > a.gap_ms]
        lines.append(f"| {q} | {len(iv)} | {busy:.1f} | {100 * busy / wall:.0f} | {len(big)} | "
                     f"{', '.join(f'{g:.1f}' for g, _ in big[::-1][:a.top])} |")
    # concurrency sweep over the stream unions
    ev = []
    for q, u in unions.items():
        for s, e in u:
            ev.append((s, 1))
            ev.append((e, -1))
    ev.sort()
    acc = defaultdict(float)
    cur, last = 0, t0
    for t, d in ev:
        acc[min(cur, 2)] += (t - last) / 1e6
        cur += d
        last = t
    lines += ["", "| streams running a kernel | ms | % of wall |", "|---|---:|---:|"]
    for k in (0, 1, 2):
        lines.append(f"| {k if k < 2 else '2+'} | {acc[k]:.1f} | {100 * acc[k] / wall:.0f} |")
    # what runs elsewhere during the longest idle gaps of the busiest streams
    lines += ["", "Longest idle gaps per stream and the other streams' kernels inside them:"]
    for q, u in list(unions.items())[:4]:
        gaps = sorted(((u[i + 1][0] - u[i][1]), u[i][1], u[i + 1][0]) for i in range(len(u) - 1))[::-1][:3]
        for g, gs, ge in gaps:
            inside = defaultdict(lambda: [0, 0.0])
            for q2, lst in names.items():
                if q2 == q:
                    continue
                for s, e, n in lst:
                    if s < ge and e > gs:
                        inside[(q2, n[:60])][0] += 1
                        inside[(q2, n[:60])][1] += (min(e, ge) - max(s, gs)) / 1e6
            top = sorted(inside.items(), key=lambda kv: -kv[1][1])[:3]
            desc = "; ".join(f"s{q2} {n} x{c} {ms:.2f} ms" for (q2, n), (c, ms) in top) or "nothing"
            lines.append(f"* stream {q}: gap {g / 1e6:.2f} ms at +{(gs - t0) / 1e6:.1f} ms -> {desc}")
    if qmap:
        lines += ["", "HIP stream -> HW queue (`queue_id`, dispatches), whole trace:", "",
                  "| stream | queues |", "|---|---|"]
        for st, qs in sorted(qmap.items()):
            lines.append(f"| {st} | {', '.join(f'q{q} ({n})' for q, n in sorted(qs))} |")
        shared = defaultdict(list)
        for st, qs in qmap.items():
            for q, _ in qs:
                shared[q].append(st)
        lines += ["", "HW queue -> streams: " + "; ".join(
            f"q{q}: {', '.join(f's{x}' for x in sorted(sts))}" for q, sts in sorted(shared.items()))]
    lines += ["", f"(kernels columns: {', '.join(cols)})"]
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")


if __name__ == "__main__":
    main()
