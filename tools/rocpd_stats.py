#!/usr/bin/env python3
"""The kernel summary (rocpd `top_kernels` view: name, calls, total / average ns) of a rocprofv3
run written as a database (no --output-format csv), as CSV -- the form profiles/*_stats.csv take.
usage: tools/rocpd_stats.py <dir with *_results.db> <out.csv>"""
import csv
import glob
import os
import sqlite3
import sys

db = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*results.db"), recursive=True))[0]
cur = sqlite3.connect(db).execute("select * from top_kernels")
with open(sys.argv[2], "w") as f:
    w = csv.writer(f)
    w.writerow([d[0] for d in cur.description])
    w.writerows(cur.fetchall())
