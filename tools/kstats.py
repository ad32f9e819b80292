"""Print a rocprofv3 kernel_stats.csv as a compact table (dev helper)."""
import csv, sys
for path in sys.argv[1:]:
    print(path)
    for x in csv.DictReader(open(path)):
        print(f"  {x['Name'][:58]:58s} calls={x['Calls']:>5s} avg={float(x['AverageNs'])/1e3:8.2f}us "
              f"min={float(x['MinNs'])/1e3:7.2f} max={float(x['MaxNs'])/1e3:8.2f} {float(x['Percentage']):5.1f}%")
