"""Print a rocprofv3 kernel_stats.csv compactly: name (shortened), calls, average and total us."""
import csv
import re
import sys

for f in sys.argv[1:]:
    print(f)
    for r in list(csv.DictReader(open(f)))[:int(sys.argv[0:1] and 24)]:
        name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
        name = re.sub(r"\(.*", "", name)[:60]
        print(f"  {name:60s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us  {float(r['TotalDurationNs']) / 1e6:8.2f} ms")
