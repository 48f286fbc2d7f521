"""Summarize a rocprofv3 kernel_stats.csv: per-kernel calls, average us, ms per bench step."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
rows = list(csv.DictReader(open(path)))
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 16]:
    print(f"{r['Name'][:72]:72s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f}us "
          f"{float(r['TotalDurationNs'])/steps/1e6:7.3f}ms/step {float(r['Percentage']):6.2f}%")
