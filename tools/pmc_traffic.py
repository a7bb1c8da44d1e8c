"""Per-launch HBM traffic of a kernel from two rocprofv3 PMC passes.

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports exactly half the bytes of a wide coalesced read, so the
read side is doubled; WRITE_SIZE is taken as is.
Usage: python tools/pmc_traffic.py FETCH.db WRITE.db KERNEL_SUBSTR OUT.json [UNITS_PER_DISPATCH]
(UNITS_PER_DISPATCH: the work units one steady dispatch processed, stored so
that a reader can scale the traffic to its own launch size.)
"""
import json
import sqlite3
import sys


def per_dispatch(db, counter, sub):
    c = sqlite3.connect(db)
    vals = [v for (n, cn, v) in c.execute(
        "select name, counter_name, counter_value from pmc_events order by dispatch_id")
        if cn == counter and sub in n]
    return vals


def main():
    fdb, wdb, sub, out = sys.argv[1:5]
    units = float(sys.argv[5]) if len(sys.argv) > 5 else None
    f = per_dispatch(fdb, "FETCH_SIZE", sub)
    w = per_dispatch(wdb, "WRITE_SIZE", sub)
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    res = {"kernel_substr": sub, "fetch_size_kb_raw": fk, "write_size_kb_raw": wk,
           "dispatches": [len(f), len(w)],
           "hbm_read_bytes_per_launch": 2 * fk * 1024, "hbm_write_bytes_per_launch": wk * 1024,
           "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
           # per dispatch in launch order (a workload whose launches differ, e.g. the
           # E-step's first chunk of an epoch without the record drop, shows here)
           "read_bytes_per_dispatch": [2 * v * 1024 for v in f],
           "write_bytes_per_dispatch": [v * 1024 for v in w],
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024",
           "sources": [fdb, wdb]}
    if units:
        res["units_per_dispatch"] = units
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
