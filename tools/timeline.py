#!/usr/bin/env python3
"""Kernel timeline of one bench phase from a rocprofv3 --kernel-trace CSV (tools/gpu session).

Prints the product kernels (sdrk / anonymous-namespace kernels, not torch's) in start order with
start and end relative to the first kernel of the window, their duration and queue, from the
dispatch of the n-th persistent PLL launch (the timed phase's) on:
  python tools/timeline.py gpurun_out/tr/kernel_trace.csv [--launch 1] [--rows 60]
  python tools/timeline.py gpurun_out/tr/kernel_trace.csv --by-grid k_frontend2
(--by-grid: that kernel's average duration per grid size -- whole-block launches apart from the
pipeline fill's part launches, which a plain --stats average mixes in)
"""
from __future__ import annotations

import argparse
import csv


def short(name: str) -> str:
    n = name.replace("void ", "").replace("sdrk::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--launch", type=int, default=1, help="which k_pll_multi dispatch (0 = warm-up phase)")
    ap.add_argument("--rows", type=int, default=60)
    ap.add_argument("--by-grid", default=None, metavar="KERNEL")
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.csv))]
    if args.by_grid:
        by: dict[int, list[float]] = {}
        for r in rows:
            if args.by_grid in r["Kernel_Name"]:
                by.setdefault(int(r["Grid_Size_X"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print(f"{args.by_grid}: grid_size_x  launches  avg_us  min_us  max_us")
        for g, v in sorted(by.items()):
            print(f"  {g:>10} {len(v):>9} {sum(v) / len(v):7.1f} {min(v):7.1f} {max(v):7.1f}")
        return
    ks = []
    for r in rows:
        n = r["Kernel_Name"]
        if "at::native" in n or "at::" in n:
            continue
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(n), r.get("Queue_Id", "?")))
    ks.sort()
    pll = [k for k in ks if k[2].startswith("k_pll_multi")]
    if len(pll) <= args.launch:
        raise SystemExit(f"only {len(pll)} persistent launches in the trace")
    p = pll[args.launch]
    # the phase: from the first product kernel after the previous launch ended up to this launch's end
    prev_end = pll[args.launch - 1][1] if args.launch > 0 else 0
    win = [k for k in ks if k[0] >= prev_end and k[0] <= p[1] + 2_000_000]
    t0 = min(k[0] for k in win if k[2] != "k_pll_multi")
    print(f"persistent launch {args.launch}: dispatched {(p[0] - t0) / 1e3:.1f} us, ends {(p[1] - t0) / 1e3:.1f} us "
          f"after the phase's first kernel")
    print(f"{'start_us':>9} {'end_us':>9} {'dur_us':>8}  queue  kernel")
    for s, e, n, q in win[: args.rows]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {q:>5}  {n}")


if __name__ == "__main__":
    main()
