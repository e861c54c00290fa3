"""Top kernels of a rocprofv3 --stats run: python scripts/kstat_top.py DIR [N]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
    print(f"{r['Name'][:64]:64s} {r['Calls']:>6s} {float(r['TotalDurationNs']) / 1e6:9.3f} ms "
          f"{float(r['AverageNs']) / 1e3:9.1f} us")
