"""Summarise a rocprofv3 results .db (kernel trace / PMC) into a small text
table for profiles/.  Usage: python tools/rocprof_summary.py RUN.db [OUT.txt]"""
import sqlite3
import sys


def _short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][-60:]


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    out = []
    out.append("# rocprofv3 kernel summary of %s" % db)
    out.append("%-60s %8s %14s %14s %8s" % ("kernel", "calls", "total_us", "avg_us", "pct"))
    for name, calls, tot, avg, pct in c.execute(
            "select name,total_calls,total_duration,average,percentage from top_kernels"):
        out.append("%-60s %8d %14.1f %14.1f %8.2f" % (_short(name), calls, tot, avg, pct))
    try:
        rows = list(c.execute("select * from pmc_events limit 1"))
        if rows:
            out.append("")
            out.append("# PMC per dispatch (counter, kernel, value)")
            q = "select dispatch_id, name, counter_name, counter_value from pmc_events order by dispatch_id"
            try:
                for d, kn, cn, v in c.execute(q):
                    out.append("%s\t%s\t%s\t%s" % (d, _short(kn), cn, v))
            except sqlite3.Error as ex:
                out.append("pmc join failed: %s" % ex)
    except sqlite3.Error:
        pass
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
