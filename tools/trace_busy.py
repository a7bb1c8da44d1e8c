"""GPU busy fraction of a rocprofv3 kernel trace: the union of kernel
intervals over the span from the first kernel matching START to the last
kernel matching END (substrings), plus the largest idle gaps and the kernel
after each.  Usage: python tools/trace_busy.py RUN.db [START] [END]"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    if not cols:
        print("no kernels view; tables:", [r[0] for r in c.execute("select name from sqlite_master")])
        return
    s_col = "start" if "start" in cols else [x for x in cols if "start" in x][0]
    e_col = "end" if "end" in cols else [x for x in cols if x.endswith("end")][0]
    n_col = "name" if "name" in cols else [x for x in cols if "name" in x][0]
    rows = sorted(c.execute('select %s, "%s", "%s" from kernels' % (n_col, s_col, e_col)), key=lambda r: r[1])
    start = sys.argv[2] if len(sys.argv) > 2 else ""
    end = sys.argv[3] if len(sys.argv) > 3 else ""
    i0 = next(k for k, r in enumerate(rows) if start in r[0])
    i1 = max(k for k, r in enumerate(rows) if end in r[0])
    rows = rows[i0:i1 + 1]
    busy, cur_s, cur_e, gaps = 0, rows[0][1], rows[0][2], []
    for n, s, e in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][2] - rows[0][1]
    print("kernels %d span %.3f ms busy %.3f ms (%.1f %%) idle %.3f ms in %d gaps" %
          (len(rows), span / 1e6, busy / 1e6, 100.0 * busy / span, (span - busy) / 1e6, len(gaps)))
    for g, n in sorted(gaps, reverse=True)[:12]:
        print("  gap %.3f ms before %s" % (g / 1e6, n.split("(")[0][-70:]))


if __name__ == "__main__":
    main()
