"""Per-kernel summary of a rocprofv3 rocpd database (the default output format):
  python scripts/rocpd_summary.py <results.db> [--by-dispatch-order N]
Prints calls / total / avg / min / max us per kernel name (+ grid), sorted by total time."""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, grid_x, grid_y, workgroup_x, duration from kernels order by start").fetchall()
    agg = {}
    for name, gx, gy, wx, dur in rows:
        k = (name[:90], f"{gx}x{gy}/{wx}")
        a = agg.setdefault(k, [0, 0.0, 1e30, 0.0])
        a[0] += 1
        a[1] += dur / 1000.0
        a[2] = min(a[2], dur / 1000.0)
        a[3] = max(a[3], dur / 1000.0)
    total = sum(a[1] for a in agg.values())
    print(f"{'kernel':90s} {'grid':>16s} {'calls':>6s} {'total us':>10s} {'avg us':>9s} {'min':>8s} {'max':>8s}   %")
    for (n, g), a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:90s} {g:>16s} {a[0]:6d} {a[1]:10.1f} {a[1] / a[0]:9.2f} {a[2]:8.2f} {a[3]:8.2f} {100 * a[1] / total:5.1f}")
    if len(sys.argv) > 3 and sys.argv[2] == "--by-dispatch-order":
        for name, gx, gy, wx, dur in rows[:int(sys.argv[3])]:
            print(f"{name[:60]:60s} {gx}x{gy}/{wx} {dur / 1000.0:.2f}")


if __name__ == "__main__":
    main()
