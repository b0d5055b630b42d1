#!/usr/bin/env python3
"""Aggregate a rocprofv3 `--pmc ... --output-format csv` run per kernel: sum of every counter over
the kernel's dispatches, plus derived ratios (MFMA busy share of busy cycles, LDS bank-conflict share
of LDS cycles, waiting / issue-stalled / active share of wave cycles).
    python scripts/pmc_summary.py <dir with *counter_collection.csv> [--top N]"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        print("no counter_collection.csv under", d)
        return 1
    agg, calls = {}, {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = {c.lower(): c for c in row}
                name = row[k["kernel_name"]][:70]
                cn, cv = row[k["counter_name"]], float(row[k["counter_value"]])
                a = agg.setdefault(name, {})
                a[cn] = a.get(cn, 0.0) + cv
                if cn == next(iter(a)):
                    calls[name] = calls.get(name, 0) + 1
    names = sorted(agg, key=lambda n: -agg[n].get("SQ_WAVE_CYCLES", agg[n].get("SQ_BUSY_CYCLES", 0.0)))[:top]
    cols = sorted({c for n in names for c in agg[n]})
    print("| kernel | calls | " + " | ".join(cols) + " | derived |")
    print("|---|---|" + "---|" * len(cols) + "---|")
    for n in names:
        a = agg[n]
        der = []
        if a.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            der.append(f"MFMA busy {100 * a['SQ_VALU_MFMA_BUSY_CYCLES'] / a['SQ_BUSY_CYCLES']:.1f}% of busy")
        if a.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in a:
            der.append(f"LDS conflict {100 * a['SQ_LDS_BANK_CONFLICT'] / a['SQ_LDS_IDX_ACTIVE']:.1f}% of LDS cycles")
        w = a.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in a:
                    der.append(f"{c[3:].lower()} {100 * a[c] / w:.0f}%")
        print(f"| {n} | {calls.get(n, 0)} | " + " | ".join(f"{a.get(c, 0):.3g}" for c in cols) + " | " +
              "; ".join(der) + " |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
