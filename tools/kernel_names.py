"""Kernel names and dispatch counts in a rocprofv3 PMC database."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cnt = collections.Counter(n for (n,) in c.execute("select name from pmc_events"))
for n, k in cnt.most_common():
    print("%6d  %s" % (k, n))
