"""Kernel-stats summary (CSV + markdown) from a rocprofv3 rocpd SQLite db (durations in ns)."""
import csv
import sqlite3
import sys


def main(db, out_prefix):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(lds_size), max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(scratch_size), "
        "max(grid_x), max(workgroup_x) from kernels group by name order by sum(duration) desc"
    ).fetchall()
    total = sum(r[2] for r in rows)
    with open(out_prefix + ".csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage",
                    "LDS", "VGPR", "AGPR", "SGPR", "Scratch", "Grid", "Workgroup"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100 * r[2] / total, 3), *r[6:]])
    with open(out_prefix + ".md", "w") as f:
        f.write(f"rocprofv3 --kernel-trace --stats summary (source: {db})\n\n")
        f.write("| kernel | calls | total (ms) | average (us) | % | LDS B | VGPR | scratch B/lane | grid |\n")
        f.write("|---|---|---|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| {r[0]} | {r[1]} | {r[2]/1e6:.3f} | {r[3]/1e3:.2f} | {100*r[2]/total:.2f} | "
                    f"{r[6]} | {r[7]} | {r[10]} | {r[11]} |\n")
    print(open(out_prefix + ".md").read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
