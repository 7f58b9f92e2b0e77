"""Print the codec kernels of a rocprofv3 kernel_stats.csv: name, calls, average / min µs, share."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        name = r["Name"]
        if "anonymous namespace)::k_" not in name:
            continue
        short = name.split("::")[-1].split("(")[0] if "::k_" in name else name
        short = name[name.index("::k_") + 2:].split("((")[0]
        print(f"  {short:52s} calls={int(r['Calls']):6d} avg={float(r['AverageNs']) / 1e3:8.2f} us "
              f"min={float(r['MinNs']) / 1e3:8.2f} us  {float(r['Percentage']):6.2f} %")
