#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of tools/bench_frontend.py per kernel.

rocprofv3 reports FETCH_SIZE and WRITE_SIZE in KiB per dispatch. Per MI355X_MICROARCH.md (HBM):
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores. The front end's loads are dword/16-byte coalesced.
  python tools/pmc_summary.py gpurun_out/<tag>
"""
from __future__ import annotations

import csv
import json
import pathlib
import sys
from collections import defaultdict


def load(path: pathlib.Path, counter: str) -> dict:
    per = defaultdict(list)
    if not path.exists():
        return {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            if "frontend" not in name:
                continue
            per[name].append(float(row["Counter_Value"]))
    return per


def kernel_name(name: str) -> str:
    # "void sdrk::(anonymous namespace)::k_frontend2<8, 10>(...)" -> "k_frontend2<8, 10>"
    for pre in ("void ", "sdrk::", "(anonymous namespace)::"):
        name = name.replace(pre, "")
    return name.split("(", 1)[0]


def mode_of(name: str) -> str:
    return "fast" if "frontend_mfma" in name or "true>" in name.split("(")[0] else "exact"


def main() -> None:
    d = pathlib.Path(sys.argv[1])
    fetch = load(d / "pmc_FETCH_SIZE.csv", "FETCH_SIZE")
    write = load(d / "pmc_WRITE_SIZE.csv", "WRITE_SIZE")
    out = {"channels": int(sys.argv[2]) if len(sys.argv) > 2 else 1024,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/bench_frontend.py; "
                     "FETCH_SIZE x2 (gfx950 wide-load correction, MI355X_MICROARCH.md HBM section)"}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None          # KiB -> B, x2 gfx950 correction
        wb = 1024 * sum(w) / len(w) if w else None
        out[mode_of(name)] = {"kernel": kernel_name(name), "dispatches": max(len(f), len(w)),
                              "fetch_bytes_corrected": fb, "write_bytes": wb,
                              "hbm_bytes_per_launch": (fb or 0) + (wb or 0) if fb is not None else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
