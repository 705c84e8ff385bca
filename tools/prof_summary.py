"""rocprofv3 output (rocpd SQLite database) -> per-kernel stats CSV for profiles/ (tooling only)."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for name, calls, tot, avg, pct in rows:
            if name.startswith("void at::native"):
                name = name.split("<")[0] + "<torch elementwise/reduce>"
            w.writerow([name[:120], calls, "%.1f" % tot, "%.1f" % avg, "%.2f" % pct])
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
