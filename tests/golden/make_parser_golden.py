#!/usr/bin/env python3
"""Golden fixture for the RDS group parser on the reference's only real-station vectors.

/root/reference/test/parser_test.cpp:79-136 holds 56 recorded 64-bit RDS group registers (PI 0xC27A,
a station's 0A groups). That test runs its own, different parse (parser_test.cpp:53-76: shifts the
characters in instead of placing them by segment), so its printed text is not the product's. This
script runs the registers through the reference program's production parse
(src/rds_utilities.cpp:172-199, the one start_frame_sync -> check_block calls) instead: the driver
tests/cpp/parse_regs_driver.cpp linked against the UNMODIFIED reference's rds_utilities.o
(oracle/_ref/parse_regs_ref, built where the sources lie by `make -C oracle ref`), and records the
registers (data read from the test file), the stderr text byte for byte and the final
(chars, output, first_time) state. tests/test_dropin_host.py rebuilds the same driver against the
drop-in frame layer (real-time-sdr_amd/host/rds_frame.cpp) and compares.
  python tests/golden/make_parser_golden.py
"""
from __future__ import annotations

import base64
import hashlib
import json
import pathlib
import re
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[2]
REF_TEST = pathlib.Path("/root/reference/test/parser_test.cpp")
EXE = ROOT / "oracle" / "_ref" / "parse_regs_ref"
OUT = ROOT / "tests" / "golden" / "golden_parser_regs.json"


def registers() -> list[int]:
    """The initialiser of `uint64_t regs[]` (parser_test.cpp:79-136), as data."""
    text = REF_TEST.read_text()
    body = text[text.index("uint64_t regs[]"):]
    body = body[body.index("{") + 1:body.index("}")]
    regs = [int(v) for v in re.findall(r"\d+", body)]
    assert len(regs) == 56 and all(r >> 48 == 0xC27A for r in regs), len(regs)
    return regs


def main() -> None:
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True, capture_output=True)
    regs = registers()
    feed = "".join(f"{r}\n" for r in regs).encode()
    r = subprocess.run([str(EXE)], input=feed, capture_output=True, check=True, timeout=60)
    fx = {
        "source": "registers: /root/reference/test/parser_test.cpp:79-136; expected: the reference's own parse "
                  "(src/rds_utilities.cpp:172-199) via tests/cpp/parse_regs_driver.cpp (oracle/_ref/parse_regs_ref)",
        "registers": [str(v) for v in regs],
        "stderr_b64": base64.b64encode(r.stderr).decode(),
        "stderr_sha256": hashlib.sha256(r.stderr).hexdigest(),
        "state": r.stdout.decode().strip(),
    }
    OUT.write_text(json.dumps(fx, indent=1) + "\n")
    names = [ln for ln in r.stderr.decode(errors="replace").splitlines() if ln.startswith("Program Service")]
    print(f"wrote {OUT}: {len(regs)} registers, {len(r.stderr)} B stderr, {names}")


if __name__ == "__main__":
    main()
