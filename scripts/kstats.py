#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for x in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{x['Name'][:110]:110s} calls={x['Calls']:>6} avg_us={float(x['AverageNs'])/1e3:9.1f} "
          f"total_ms={float(x['TotalDurationNs'])/1e6:8.1f} {float(x['Percentage']):5.1f}%")
