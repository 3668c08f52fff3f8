"""Print the last kernels of a rocprofv3 --kernel-trace CSV as a timeline (us from the first)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
t0 = int(rows[-n]["Start_Timestamp"])
for r in rows[-n:]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print("q%s %-34s %9.1f %9.1f %7.1f" % (r["Queue_Id"], r["Kernel_Name"][:34], s, e, e - s))
