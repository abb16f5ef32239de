"""Summarise a rocprofv3 run (rocpd SQLite .db or kernel_stats.csv) into a small CSV for profiles/."""
import csv
import sqlite3
import sys


def main(src, dst):
    rows = []
    if src.endswith(".db"):
        con = sqlite3.connect(src)
        for name, calls, total, avg, pct in con.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            rows.append((name.split("(")[0], calls, total, avg, pct))   # top_kernels is in us
    else:
        for r in csv.DictReader(open(src)):
            rows.append((r["Name"].split("(")[0], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                         float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], f"{r[2]:.1f}", f"{r[3]:.1f}", f"{r[4]:.2f}"])
    print(open(dst).read()[:2000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
