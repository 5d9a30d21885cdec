"""Print a rocprofv3 kernel_stats.csv as a table (diagnostic helper)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for x in rows:
    print(f"{x['Name'][:64]:64s} {x['Calls']:>5s} avg {float(x['AverageNs'])/1000:10.2f} us  min {float(x['MinNs'])/1000:9.2f}  tot% {float(x['Percentage']):6.2f}")
