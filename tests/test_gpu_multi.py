"""GPU: the multi-channel receiver real-time-sdr_amd/bin/sdr_multi (three stage threads on the C ABI,
device-resident FmBatch queue payload, pinned double-buffered I/O) on 6 channels x 24 blocks of
u8 I/Q from a file: the stereo PCM of every channel and block bit-exact against the oracle, and
the RDS text of channel 0 equal to the reference program's own (`project 0 r`,
tests/golden/project_e2e.json; stereo.cpp:100-111, rds.cpp:181-189)."""
from __future__ import annotations

import json
import subprocess

import numpy as np
import pytest

from conftest import GOLD, ROOT, channel_input

pytestmark = pytest.mark.gpu

NCH, NB = 6, 24


def test_sdr_multi_file_to_pcm_and_rds(synth, oracle, tmp_path):
    exe = ROOT / "real-time-sdr_amd" / "bin" / "sdr_multi"
    assert exe.exists(), "build with make"
    e2e = json.loads((GOLD / "project_e2e.json").read_text())
    iqs = [channel_input(synth, c, NB, e2e["input_sha256"] if c == 0 else None) for c in range(NCH)]
    np.ascontiguousarray(np.stack(iqs, axis=1)).tofile(tmp_path / "in.u8")   # [block][ch][bytes]
    r = subprocess.run([str(exe), str(NCH), "--in", str(tmp_path / "in.u8"), "--out", str(tmp_path / "rx")],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    assert f"{NCH} channels x {NB} blocks" in r.stderr, r.stderr
    pcm = np.fromfile(tmp_path / "rx.pcm", np.int16).reshape(NB, NCH, 2940)
    for c in range(NCH):
        ref = oracle.run_channel(iqs[c], 0, True)
        for b in range(NB):
            assert np.array_equal(pcm[b, c], ref["stereo"][b]), f"stereo ch{c} block {b}"
    text = {}
    for line in (tmp_path / "rx.rds").read_text().splitlines():
        ch, _, rest = line.partition(": ")
        text.setdefault(int(ch.split()[1]), []).append(rest)
    assert "\n".join(text[0]) + "\n" == e2e["r"]["stderr"]
    for c in range(NCH):
        assert f"PI: {0x1000 + c:x}" in text.get(c, []), f"channel {c}: {text.get(c)}"
