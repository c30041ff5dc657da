"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, share."""
import csv
import sys

for x in list(csv.DictReader(open(sys.argv[1])))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{x['Name'][:64]:64s} {x['Calls']:>6} {float(x['AverageNs'])/1e3:9.2f}us "
          f"{float(x['Percentage']):6.2f}%")
