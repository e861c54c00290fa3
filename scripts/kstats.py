"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, %."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:10.1f}us "
              f"pct={float(r['Percentage']):6.2f}")
