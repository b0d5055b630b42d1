"""Per-kernel summary of a rocprofv3 SQLite (rocpd) output: calls, total / mean us, share, grid,
LDS and VGPRs. Usage: rocpd_summary.py <results.db> [--per N] (N = divide totals by N, e.g. tokens)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=float, default=0.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), max(grid_x / workgroup_x), max(lds_size), "
                     "max(vgpr_count) from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    hdr = f"{'kernel':70s} {'calls':>6s} {'total us':>10s} {'mean us':>8s} {'%':>5s} {'wgs':>6s} {'lds':>6s} {'vgpr':>4s}"
    if a.per:
        hdr += f" {'us/unit':>8s}"
    print(hdr)
    for name, n, s, m, g, lds, v in rows[:a.top]:
        short = name.split("(")[0].replace("void ", "").replace("dl::hipk::", "")[:70]
        line = f"{short:70s} {n:6d} {s / 1e3:10.1f} {m / 1e3:8.2f} {100 * s / tot:5.1f} {g:6d} {lds:6d} {v:4d}"
        if a.per:
            line += f" {s / 1e3 / a.per:8.2f}"
        print(line)
    print(f"total {tot / 1e6:.3f} ms" + (f", {tot / 1e3 / a.per:.1f} us per unit" if a.per else ""))


if __name__ == "__main__":
    main()
