"""Summarise a rocprofv3 run (sqlite .db or kernel_stats.csv) into a per-kernel table.

usage: python scripts/prof_summary.py gpurun_out/prof/run_results.db [--last N] > profiles/x.md
`--last N` restricts to the last N dispatches of each kernel name (steady state)."""
import argparse
import collections
import csv
import glob
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("dl::hipk::", "")
    return name[:80]


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, "
                     "accum_vgpr_count, sgpr_count from kernels").fetchall()
    return [dict(name=r[0], start=r[1], end=r[2], grid=f"{r[3]}x{r[4]}x{r[5]}", wg=r[6], lds=r[7], vgpr=r[8] + r[9],
                 sgpr=r[10]) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--by-grid", action="store_true", help="separate rows per launch grid (wo vs w2, ...)")
    ap.add_argument("--skip-first", type=int, default=0, help="ignore the first N dispatches overall (warmup)")
    args = ap.parse_args()
    path = args.path
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = cands[0]
    rows = from_db(path)
    rows.sort(key=lambda r: r["start"])
    rows = rows[args.skip_first:]
    agg = collections.OrderedDict()
    for r in rows:
        k = short(r["name"]) + (f" [{r['grid']}]" if args.by_grid else "")
        a = agg.setdefault(k, dict(calls=0, ns=0, vgpr=r["vgpr"], lds=r["lds"], grid=r["grid"], wg=r["wg"]))
        a["calls"] += 1
        a["ns"] += r["end"] - r["start"]
    total = sum(a["ns"] for a in agg.values())
    span = (rows[-1]["end"] - rows[0]["start"]) if rows else 0
    print(f"dispatches: {len(rows)}  kernel time: {total / 1e6:.3f} ms  span: {span / 1e6:.3f} ms  "
          f"(busy {100.0 * total / max(span, 1):.1f}%)\n")
    print("| kernel | calls | total ms | avg us | % | vgpr | lds B | grid | wg |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        print(f"| {k} | {a['calls']} | {a['ns'] / 1e6:.3f} | {a['ns'] / a['calls'] / 1e3:.2f} | "
              f"{100.0 * a['ns'] / total:.1f} | {a['vgpr']} | {a['lds']} | {a['grid']} | {a['wg']} |")


if __name__ == "__main__":
    main()
