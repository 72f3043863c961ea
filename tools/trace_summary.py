"""Print the per-dispatch timeline of a rocprofv3 kernel-trace csv (class launches of one run)."""
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(path)) if "copyBuffer" not in r["Kernel_Name"]]
t0 = min(int(r["Start_Timestamp"]) for r in rows)
for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    print("%-44s q%-3s lds %6s  %8.1f -> %8.1f ms (%7.1f)" % (r["Kernel_Name"][:44], r["Queue_Id"],
          r["LDS_Block_Size"], s, e, e - s))
