"""Per-wave SQ instruction counters of a kernel from a rocprofv3 --pmc run.
Usage: python tools/sq_counters.py run_results.db KERNEL_SUBSTR"""
import collections
import sqlite3
import sys

db, sub = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
acc = collections.defaultdict(list)
for name, cn, v in c.execute("select name, counter_name, counter_value from pmc_events"):
    if sub in name:
        acc[cn].append(v)
waves = sum(acc["SQ_WAVES"]) / max(len(acc["SQ_WAVES"]), 1) if "SQ_WAVES" in acc else 0
print("rows", max((len(v) for v in acc.values()), default=0), "waves/row", waves)
for cn, vals in sorted(acc.items()):
    m = sum(vals) / len(vals)
    print("%-22s per-dispatch %.4g  per-wave %.4g" % (cn, m, m / waves if waves else 0))
