"""Print a rocprofv3 --stats kernel_stats.csv compactly: name, calls, average and total time."""
import csv
import glob
import sys

for f in sys.argv[1:] or glob.glob("gpurun_out/gprof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        n = n.split("(")[0] if "rocprim" not in n else "rocprim:" + (n.split("wrapped_")[1][:40] if "wrapped_" in n else n[:50])
        print(f"{n[:64]:64s} calls {r['Calls']:>5} avg {float(r['AverageNs']) / 1e3:9.1f} us  total {float(r['TotalDurationNs']) / 1e6:8.3f} ms")
