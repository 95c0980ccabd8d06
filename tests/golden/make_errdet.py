#!/usr/bin/env python3
"""Golden fixtures for error_detection (reference src/rds_utilities.cpp:202-311).

Builds tests/cpp/errdet_driver.cpp against the UNMODIFIED reference's rds_utilities.o (compiled
where it lies by `make -C oracle ref`, into oracle/_ref/obj/) and records, for each input case, the
driver's stderr (sha256, length, head) and final state (stdout). Cases: the reference program's own
decoded RDS bits of the golden channels (golden_mode0_long.json), the same with bit errors and with
a bit slip, and random bits. The bit streams are stored in the fixture; the test rebuilds the driver
against the drop-in library's rds_frame.cpp and compares.
  python tests/golden/make_errdet.py
"""
from __future__ import annotations

import hashlib
import json
import pathlib
import random
import subprocess
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[2]
REF_INC = pathlib.Path("/root/reference/include")
REF_OBJ = ROOT / "oracle" / "_ref" / "obj" / "rds_utilities.o"
OUT = ROOT / "tests" / "golden" / "golden_errdet.json"


def cases() -> dict[str, list[str]]:
    g = json.loads((ROOT / "tests" / "golden" / "golden_mode0_long.json").read_text())
    out = {}
    rng = random.Random(7)
    for ch, fx in sorted(g["channels"].items()):
        blocks = [b["bits"] if "offset" in b else "-" for b in fx["blocks"]]
        out[f"ch{ch}"] = blocks
        # ~1 % flipped bits: bad blocks, sync kept
        out[f"ch{ch}_flips"] = ["-" if b == "-" else "".join(c if rng.random() > 0.01 else "10"[int(c)] for c in b)
                                for b in blocks]
        # one dropped bit in the middle, then a burst of noise: sync lost and found again
        mid = len(blocks) // 2
        slip = list(blocks)
        if slip[mid] != "-" and len(slip[mid]) > 1:
            slip[mid] = slip[mid][1:]
        for k in range(mid + 1, min(mid + 60, len(slip))):
            if slip[k] != "-":
                slip[k] = "".join(rng.choice("01") for _ in slip[k])
        out[f"ch{ch}_slip_noise"] = slip
    out["random"] = ["".join(rng.choice("01") for _ in range(rng.randint(30, 42))) for _ in range(40)]
    return out


def run(exe: pathlib.Path, blocks: list[str]) -> dict:
    r = subprocess.run([str(exe)], input="\n".join(blocks) + "\n", capture_output=True, text=True, check=True,
                       timeout=120)
    return {"stderr_sha256": hashlib.sha256(r.stderr.encode()).hexdigest(), "stderr_len": len(r.stderr),
            "stderr_head": r.stderr[:3000], "state": r.stdout.strip()}


def main() -> None:
    if not REF_OBJ.exists():
        raise SystemExit(f"{REF_OBJ} missing: run `make -C oracle ref` (needs /root/reference)")
    with tempfile.TemporaryDirectory() as td:
        exe = pathlib.Path(td) / "errdet_ref"
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(REF_INC), str(ROOT / "tests" / "cpp" / "errdet_driver.cpp"),
                        str(REF_OBJ), "-o", str(exe)], check=True)
        fx = {"source": "reference src/rds_utilities.cpp:202-311 via tests/cpp/errdet_driver.cpp", "cases": {}}
        for name, blocks in cases().items():
            fx["cases"][name] = {"blocks": blocks, **run(exe, blocks)}
    OUT.write_text(json.dumps(fx, indent=0))
    print(f"wrote {OUT} ({len(fx['cases'])} cases)")


if __name__ == "__main__":
    main()
