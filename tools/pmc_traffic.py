"""Per-launch HBM traffic of kernels from two rocprofv3 PMC passes, stamped.

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports exactly half the bytes of a wide coalesced read, so the
read side is doubled; WRITE_SIZE is taken as is.

Usage: python tools/pmc_traffic.py FETCH.db WRITE.db LEG OUTDIR KERNEL [KERNEL ...]
           [--units N | --units-total N] [--steady low2of3] [--commit SHA] [--skip K]
One summary per kernel substring, OUTDIR/<LEG>__<slug(KERNEL)>.json, stamped
with the kernel sources' sha256 (tools/pmc_stamp.py; bench.py uses a summary
only when the stamp matches the sources it runs), the library's sha256 and
the commit.  --units: work units one steady dispatch processed (a reader
scales the traffic to its own launch size).  --skip K: drop each kernel's
first K dispatches (warm-up launches of a different size).
"""
import argparse
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_stamp  # noqa: E402


def per_dispatch(db, counter, sub):
    c = sqlite3.connect(db)
    return [v for (n, cn, v) in c.execute(
        "select name, counter_name, counter_value from pmc_events order by dispatch_id")
        if cn == counter and sub in n]


def summary(fdb, wdb, sub, skip=0):
    f = per_dispatch(fdb, "FETCH_SIZE", sub)[skip:]
    w = per_dispatch(wdb, "WRITE_SIZE", sub)[skip:]
    if not f or not w:
        raise SystemExit("no dispatches of %r in the PMC databases" % sub)
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    return {"kernel_substr": sub, "fetch_size_kb_raw": fk, "write_size_kb_raw": wk,
            "dispatches": [len(f), len(w)],
            "hbm_read_bytes_per_launch": 2 * fk * 1024, "hbm_write_bytes_per_launch": wk * 1024,
            "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
            # per dispatch in launch order (a workload whose launches differ, e.g. the
            # E-step's first chunk of an epoch without the record drop, shows here)
            "read_bytes_per_dispatch": [2 * v * 1024 for v in f],
            "write_bytes_per_dispatch": [v * 1024 for v in w],
            "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_db")
    ap.add_argument("write_db")
    ap.add_argument("leg")
    ap.add_argument("outdir")
    ap.add_argument("kernels", nargs="+")
    ap.add_argument("--units", type=float)
    ap.add_argument("--units-total", type=float,
                    help="work units over all profiled dispatches: units per dispatch = this / dispatches")
    ap.add_argument("--steady")
    ap.add_argument("--commit")
    ap.add_argument("--skip", type=int, default=0)
    a = ap.parse_args()
    os.makedirs(a.outdir, exist_ok=True)
    stamp = {"src_sha": pmc_stamp.src_sha256(), "lib_sha": pmc_stamp.lib_sha256(),
             "commit": a.commit or pmc_stamp.git_head(), "leg": a.leg}
    for k in a.kernels:
        res = summary(a.fetch_db, a.write_db, k, a.skip)
        res.update(stamp)
        if a.units:
            res["units_per_dispatch"] = a.units
        elif a.units_total:
            res["units_per_dispatch"] = a.units_total / res["dispatches"][0]
        if a.steady:
            res["steady"] = a.steady
        out = os.path.join(a.outdir, "%s__%s.json" % (a.leg, pmc_stamp.slug(k)))
        json.dump(res, open(out, "w"), indent=1)
        print("%-40s %-40s %.4g B/launch (%d dispatches)" % (a.leg, k, res["hbm_bytes_per_launch"],
                                                              res["dispatches"][0]))


if __name__ == "__main__":
    main()
