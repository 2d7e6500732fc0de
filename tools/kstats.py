"""Print a rocprofv3 kernel_stats.csv as short name / calls / average us (diagnostics)."""
import csv
import re
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        for r in csv.DictReader(f):
            name = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
            print(f"  {name[:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1000:9.1f} us")
