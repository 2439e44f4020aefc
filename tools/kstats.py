"""Print a rocprofv3 kernel_stats.csv compactly: python tools/kstats.py <dir>"""
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-58s %6s %10.3f ms %10.1f us %6.2f%%" % (r["Name"][:58], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                                 float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
