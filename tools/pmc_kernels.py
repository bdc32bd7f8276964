#!/usr/bin/env python3
"""Mean PMC counter values per kernel from a rocprofv3 --pmc database.

    python tools/pmc_kernels.py DB [pattern ...]
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db, pats = sys.argv[1], sys.argv[2:]
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, value from counters_collection").fetchall()
    agg = defaultdict(lambda: defaultdict(list))
    for k, n, v in rows:
        if not pats or any(p in k for p in pats):
            agg[k.split("(")[0]][n].append(v)
    for k, cs in agg.items():
        print(k)
        for n, vs in sorted(cs.items()):
            print(f"   {n:32s} {sum(vs) / len(vs):16.1f}  (n={len(vs)})")


if __name__ == "__main__":
    main()
