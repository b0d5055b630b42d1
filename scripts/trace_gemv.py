"""Workgroup timeline of the Q40 GEMV inside a hipGraph of back-to-back launches.

Every workgroup stamps s_memrealtime (100 MHz, one clock for the whole device) at entry, when the
ring's first round of weight loads has landed (prologue done), and at exit (GemvArgs::trace).
Per shape this prints, averaged over the launches after the first few:
  span   first entry -> last exit of a launch
  gap    last exit of launch i -> first entry of launch i+1 (the dependent-kernel boundary)
  entry  spread of workgroup entry times (dispatch ramp)
  loaded entry -> prologue loads landed (median; early path only)
  ready  entry -> prologue done (median / p90; late path: first ring round landed too)
  first  entry -> first ring slot consumed (median)
  exit   spread of exit times relative to the launch's first entry (median / p90 / max)
  [COPIES=n] python scripts/trace_gemv.py [shape ...]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl

C = dl.native()
PRO_GLOBAL, PRO_RESNORM = 0, 1
EPI_STORE, EPI_ACT, EPI_QKV, EPI_ACT_Q80 = 0, 1, 2, 3
SHAPES = {
    "qkv": (6144, 4096, PRO_RESNORM, EPI_QKV),
    "wo": (4096, 4096, PRO_GLOBAL, EPI_STORE),
    "w13": (28672, 4096, PRO_RESNORM, EPI_ACT_Q80),
    "w2": (4096, 14336, PRO_GLOBAL, EPI_STORE),
    "wcls": (128256, 4096, PRO_RESNORM, EPI_STORE),
    # rank shards of Llama-3.1-8B at TP8 (w2 takes the norm prologue there: hidden0 / 32 < 192)
    "qkv8": (768, 4096, PRO_RESNORM, EPI_QKV),
    "wo8": (4096, 512, PRO_GLOBAL, EPI_STORE),
    "w13_8": (3584, 4096, PRO_RESNORM, EPI_ACT),
    "w2_8": (4096, 1792, PRO_RESNORM, EPI_STORE),
    # their TP tails (EPI_STORE_TP in loopback: DL_BENCH_TP_WORLD / DL_BENCH_TP_Q80)
    "wo8tp": (4096, 512, PRO_GLOBAL, 5),
    # the same matrices with / without the norm prologue (plain store): its cost on the launch
    "w13n": (28672, 4096, PRO_RESNORM, EPI_STORE),
    "w13g": (28672, 4096, PRO_GLOBAL, EPI_STORE),
    "qkvn": (6144, 4096, PRO_RESNORM, EPI_STORE),
    "qkvg": (6144, 4096, PRO_GLOBAL, EPI_STORE),
    "w13_8n": (3584, 4096, PRO_RESNORM, EPI_STORE),
    "w13_8g": (3584, 4096, PRO_GLOBAL, EPI_STORE),
    "qkv8n": (768, 4096, PRO_RESNORM, EPI_STORE),
    "qkv8g": (768, 4096, PRO_GLOBAL, EPI_STORE),
    "w2_8tp": (4096, 1792, PRO_RESNORM, 5),
}
TICK_US = 0.01  # s_memrealtime runs at 100 MHz


def analyse(name, us, t, iters):
    t = t.reshape(iters, -1, 8).astype(np.int64)
    grid = t.shape[1]
    rows = []
    for i in range(4, iters):
        e, r, x, ld, f, lp = t[i, :, 0], t[i, :, 1], t[i, :, 2], t[i, :, 4], t[i, :, 5], t[i, :, 7]
        t0 = e.min()
        rows.append(dict(loaded=np.median(ld - e) if ld.min() > 0 else np.nan, first=np.median(f - e),
                         loop=np.median(lp - e), tail=np.median(x - lp),
                         summed=np.median(t[i, :, 6] - e) if t[i, :, 6].min() > 0 else np.nan,span=x.max() - t0, entry=e.max() - t0, ready_med=np.median(r - e), ready_p90=np.percentile(r - e, 90),
                         exit_med=np.median(x - t0), exit_p90=np.percentile(x - t0, 90), exit_min=x.min() - t0,
                         gap=(t[i + 1, :, 0].min() - x.max()) if i + 1 < iters else np.nan))
    avg = {k: np.nanmean([r[k] for r in rows]) * TICK_US for k in rows[0]}
    xcc = (t[-1, :, 3] & 0xF)
    per_xcc = np.bincount(xcc, minlength=8)
    # where does the tail come from? per-CU load (workgroups sharing a CU), XCC, entry order
    hw = (t[4:, :, 3] >> 32)
    cu = (t[4:, :, 3] & 0xF) * 4096 + ((hw >> 8) & 0xF) + 16 * ((hw >> 12) & 0x1) + 32 * ((hw >> 13) & 0x7)
    ex = (t[4:, :, 2] - t[4:, :, 0].min(axis=1, keepdims=True)) * TICK_US
    en = (t[4:, :, 0] - t[4:, :, 0].min(axis=1, keepdims=True)) * TICK_US
    share = np.zeros_like(cu)
    for i in range(cu.shape[0]):
        _, inv, cnt = np.unique(cu[i], return_inverse=True, return_counts=True)
        share[i] = cnt[inv]
    by_share = {int(k): round(float(ex[share == k].mean()), 2) for k in np.unique(share)}
    n_share = {int(k): int((share == k).sum() // cu.shape[0]) for k in np.unique(share)}
    xc = t[4:, :, 3] & 0xF
    by_xcc = [round(float(ex[xc == k].max(axis=-1).mean() if (xc == k).any() else 0), 2) for k in range(8)]
    last = ex >= np.percentile(ex, 95, axis=1, keepdims=True)
    print(f"    exit by WGs/CU {by_share} (WGs {n_share}) | max exit by XCC {by_xcc} | "
          f"corr(entry, exit) {np.corrcoef(en.ravel(), ex.ravel())[0, 1]:.2f} | last-5% entry {en[last].mean():.2f} vs all {en.mean():.2f} "
          f"| last-5% share {share[last].mean():.2f} vs all {share.mean():.2f} | blockIdx of last-5% mean {np.nonzero(last)[1].mean():.0f} of {grid}",
          flush=True)
    print(f"{name:5s} grid {grid:4d} | {us:6.2f} us/launch | span {avg['span']:5.2f} gap {avg['gap']:4.2f} | "
          f"entry spread {avg['entry']:4.2f} | loaded {avg['loaded']:4.2f} | norm summed {avg['summed']:4.2f} | first {avg['first']:4.2f} | ready med {avg['ready_med']:4.2f} p90 {avg['ready_p90']:4.2f} | "
          f"loop end {avg['loop']:4.2f} tail {avg['tail']:4.2f} | "
          f"exit min {avg['exit_min']:5.2f} med {avg['exit_med']:5.2f} p90 {avg['exit_p90']:5.2f} | WGs/XCC {per_xcc.tolist()}",
          flush=True)


def main():
    names = sys.argv[1:] or list(SHAPES)
    iters = int(os.environ.get("ITERS", "24"))
    for name in names:
        rows, n, pro, epi = SHAPES[name]
        # COPIES weight copies cycled per launch: 8 x a TP8 shard fits the 256 MB MALL, 48 do not
        us, t = C.trace_gemv_q40(rows, n, pro, epi, 1, 0, 0, int(os.environ.get("COPIES", "8")), iters)
        analyse(name, us, t, iters)


if __name__ == "__main__":
    main()
