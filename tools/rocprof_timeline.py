"""Dispatch timeline of a rocprofv3 kernel trace: start / end (ms, relative to
the first selected dispatch), duration, queue and VGPR/LDS of every dispatch
whose name matches, so overlapped kernels (the PARITY fold on its side stream
next to the next chunk's walks) can be read as a schedule, not a sum.

Usage: python tools/rocprof_timeline.py RUN.db [--match SUBSTR[,SUBSTR]]
                                        [--after-ms X] [--limit N] [OUT.txt]
"""
import argparse
import sqlite3


def _short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][-56:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--match", default="")
    ap.add_argument("--after-ms", type=float, default=0.0)
    ap.add_argument("--limit", type=int, default=400)
    ap.add_argument("--min-us", type=float, default=0.0, help="drop dispatches shorter than this")
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    subs = [s for s in args.match.split(",") if s]
    rows = list(c.execute("select name, start, end, queue_id, vgpr_count, lds_size, grid_x, workgroup_x "
                          "from kernels order by start"))
    rows = [r for r in rows if not subs or any(s in r[0] for s in subs)]
    if not rows:
        print("no dispatches")
        return
    t0 = rows[0][1]
    out = ["# timeline of %s (ms from the first matching dispatch)" % args.db,
           "%10s %10s %9s %3s %4s %6s %9s  %s" % ("start", "end", "dur_us", "q", "vgpr", "lds", "grid", "kernel")]
    n = 0
    for name, s, e, q, vg, lds, gx, wx in rows:
        st = (s - t0) / 1e6
        if st < args.after_ms or (e - s) / 1e3 < args.min_us:
            continue
        out.append("%10.3f %10.3f %9.1f %3d %4d %6d %9d  %s" % (st, (e - t0) / 1e6, (e - s) / 1e3, q, vg, lds,
                                                              gx // max(wx, 1), _short(name)))
        n += 1
        if n >= args.limit:
            break
    text = "\n".join(out) + "\n"
    if args.out:
        open(args.out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
