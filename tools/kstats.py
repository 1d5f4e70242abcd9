"""Print the top kernels of a rocprofv3 *kernel_stats.csv by total time.
usage: python tools/kstats.py <kernel_stats.csv> [top_n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print('%-72s %6s %9.1f us' % (r['Name'][:72], r['Calls'], float(r['AverageNs']) / 1e3))
