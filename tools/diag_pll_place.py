#!/usr/bin/env python3
"""Where the waves of one k_pll launch ran, and how long each took (four waves per CU).
Needs a -DSDR_PLL_HWID=1 diagnosis build (SDR_AMD_LIB=build/variants/<name>.so): every wave records
its HW_ID (SIMD, CU, shader array, SE), XCC_ID, its shader cycles from entry to exit and its 100 MHz
entry/exit times. Prints one JSON line: waves per CU and per SIMD, cycles per step grouped by how many
waves shared the CU (and the SIMD), and how many of a CU's waves overlapped in time.
  SDR_AMD_LIB=build/variants/hwid.so python tools/diag_pll_place.py --channels 32768 [--cus 64]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import pathlib
import statistics
import sys
from collections import defaultdict

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

FIELDS = 5


def decode(hw: int, xcc: int) -> dict:
    # gfx9 HW_ID: wave slot [3:0], SIMD [5:4], pipe [7:6], CU [11:8], shader array [12], SE [15:13]
    return {"slot": hw & 15, "simd": (hw >> 4) & 3, "cu": (hw >> 8) & 15, "sh": (hw >> 12) & 1,
            "se": (hw >> 13) & 7, "xcc": xcc & 15}


def summarise(rows: list[dict], n: int) -> dict:
    by_cu: dict[tuple, list[dict]] = defaultdict(list)
    by_simd: dict[tuple, list[dict]] = defaultdict(list)
    for r in rows:
        k = (r["xcc"], r["se"], r["sh"], r["cu"])
        by_cu[k].append(r)
        by_simd[k + (r["simd"],)].append(r)
    for k, ws in by_cu.items():
        for w in ws:
            w["on_cu"] = len(ws)
            # waves of this CU whose [entry, exit] overlaps this wave's
            w["overlap_cu"] = sum(1 for o in ws if o["r0"] < w["r1"] and w["r0"] < o["r1"])
    for k, ws in by_simd.items():
        for w in ws:
            w["on_simd"] = len(ws)
            w["overlap_simd"] = sum(1 for o in ws if o["r0"] < w["r1"] and w["r0"] < o["r1"])

    def group(key: str) -> dict:
        g: dict[int, list[float]] = defaultdict(list)
        for r in rows:
            g[r[key]].append(r["cyc"] / n)
        return {str(k): {"waves": len(v), "cycles_per_step_mean": round(statistics.fmean(v), 1),
                         "min": round(min(v), 1), "max": round(max(v), 1)} for k, v in sorted(g.items())}

    t0 = min(r["r0"] for r in rows)
    starts = sorted((r["r0"] - t0) / 100.0 for r in rows)
    return {
        "waves": len(rows), "cus_used": len(by_cu), "simds_used": len(by_simd),
        "xccs": len({r["xcc"] for r in rows}),
        "waves_per_cu_hist": {str(k): v for k, v in sorted(
            ((c, sum(1 for ws in by_cu.values() if len(ws) == c)) for c in {len(ws) for ws in by_cu.values()}))},
        "waves_per_simd_hist": {str(k): v for k, v in sorted(
            ((c, sum(1 for ws in by_simd.values() if len(ws) == c)) for c in {len(ws) for ws in by_simd.values()}))},
        "by_waves_on_cu": group("on_cu"), "by_overlap_on_cu": group("overlap_cu"),
        "by_waves_on_simd": group("on_simd"), "by_overlap_on_simd": group("overlap_simd"),
        "entry_us": {"first": 0.0, "median": round(starts[len(starts) // 2], 2), "last": round(starts[-1], 2)},
        "span_us": round((max(r["r1"] for r in rows) - t0) / 100.0, 1),
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", type=int, default=32768)
    ap.add_argument("--n", type=int, default=7350)
    ap.add_argument("--cus", type=int, default=0)
    ap.add_argument("--raw", type=str, default="", help="also write the per-wave rows (JSON) here")
    args = ap.parse_args()
    import torch
    pkg = bench._load_pkg()
    lib = pkg.lib()
    probe = (C.c_ulonglong * FIELDS)()
    if lib.sdr_diag_pll_hwid(probe, 0) < 0:
        raise SystemExit("not a -DSDR_PLL_HWID=1 build (set SDR_AMD_LIB)")
    dev = torch.device("cuda", 0)
    nch, n = args.channels, args.n
    i = torch.arange(n, dtype=torch.float64, device=dev)
    ph0 = torch.rand(nch, 1, dtype=torch.float64, device=dev) * 2 * math.pi
    x = (0.1 * torch.cos(2 * math.pi * 19e3 / 240e3 * i + ph0)).float() + 0.01 * torch.randn(nch, n, device=dev)
    out = torch.empty(nch, n + 1, dtype=torch.float32, device=dev)
    st = pkg.pll_state_tensor(nch, device=dev)
    created = []
    s = (bench.cu_masked_streams(torch, pkg, dev, str(args.cus), created, all_cus=False)[1]
         if args.cus > 0 else torch.cuda.Stream(dev))
    for _ in range(3):
        pkg.fmpll(out, x, 19e3, 240e3, st, 2.0, 0.0, 0.01, stream=s)
    torch.cuda.synchronize()
    nw = (2 * nch + 63) // 64                     # lane pairs: two lanes per channel
    buf = (C.c_ulonglong * (FIELDS * nw))()
    got = lib.sdr_diag_pll_hwid(buf, nw)
    rows = []
    for w in range(got):
        hw, xcc, cyc, r0, r1 = (int(buf[FIELDS * w + f]) for f in range(FIELDS))
        rows.append({"wave": w, **decode(hw, xcc), "cyc": cyc, "r0": r0, "r1": r1})
    res = {"channels": nch, "cus": args.cus or None, **summarise(rows, n)}
    print(json.dumps(res))
    if args.raw:
        pathlib.Path(args.raw).write_text(json.dumps(rows))
    bench.destroy_masked_streams(torch, pkg, dev, created)


if __name__ == "__main__":
    main()
