"""GPU: the multi-channel receiver (include/sdr_multi.h; the CLI real-time-sdr_amd/bin/sdr_multi:
three stage threads on the C ABI, device-resident FmBatch queue payload, pinned double-buffered
I/O) on 6 channels x 24 blocks of u8 I/Q: from a file (each consumer's PLL one persistent launch,
sdr_plls_launch_sel), from a pipe (per-block PLL dispatches) and from device memory through
sdr_multi_run (bench.py's queue_plumbed leg): the stereo PCM of every channel and block bit-exact
against the oracle, and the RDS text of channel 0 equal to the reference program's own
(`project 0 r`, tests/golden/project_e2e.json; stereo.cpp:100-111, rds.cpp:181-189)."""
from __future__ import annotations

import json
import subprocess

import numpy as np
import pytest

from conftest import GOLD, ROOT, channel_input

pytestmark = pytest.mark.gpu

NCH, NB = 6, 24


@pytest.fixture(scope="module")
def multi_input(synth):
    e2e = json.loads((GOLD / "project_e2e.json").read_text())
    iqs = [channel_input(synth, c, NB, e2e["input_sha256"] if c == 0 else None) for c in range(NCH)]
    return e2e, iqs


@pytest.fixture(scope="module")
def multi_ref(multi_input, oracle):
    return [oracle.run_channel(iq, 0, True) for iq in multi_input[1]]


@pytest.mark.parametrize("source", ["file", "pipe"])
def test_sdr_multi_file_to_pcm_and_rds(multi_input, multi_ref, tmp_path, source):
    exe = ROOT / "real-time-sdr_amd" / "bin" / "sdr_multi"
    assert exe.exists(), "build with make"
    e2e, iqs = multi_input
    blob = np.ascontiguousarray(np.stack(iqs, axis=1))   # [block][ch][bytes]
    blob.tofile(tmp_path / "in.u8")
    args = [str(exe), str(NCH), "--cus", "16", "--out", str(tmp_path / "rx")]
    if source == "file":
        r = subprocess.run(args + ["--in", str(tmp_path / "in.u8")], capture_output=True, text=True, timeout=180)
    else:
        r = subprocess.run(args + ["--in", "-"], input=blob.tobytes(), capture_output=True, timeout=180)
        r.stderr = r.stderr.decode()
    assert r.returncode == 0, r.stderr
    assert f"{NCH} channels x {NB} blocks" in r.stderr, r.stderr
    assert ("PLLs persistent" if source == "file" else "PLLs per-block dispatch") in r.stderr, r.stderr
    pcm = np.fromfile(tmp_path / "rx.pcm", np.int16).reshape(NB, NCH, 2940)
    for c in range(NCH):
        ref = multi_ref[c]
        for b in range(NB):
            assert np.array_equal(pcm[b, c], ref["stereo"][b]), f"stereo ch{c} block {b}"
    text = {}
    for line in (tmp_path / "rx.rds").read_text().splitlines():
        ch, _, rest = line.partition(": ")
        text.setdefault(int(ch.split()[1]), []).append(rest)
    assert "\n".join(text[0]) + "\n" == e2e["r"]["stderr"]
    for c in range(NCH):
        assert f"PI: {0x1000 + c:x}" in text.get(c, []), f"channel {c}: {text.get(c)}"


def test_sdr_multi_run_device_input_captures(pkg, tmp_path):
    """sdr_multi_run over blocks resident on the device, as bench.py's queue_plumbed leg runs it (its
    child mode: the bench's generator, 8 distinct channels x 12 blocks): the captured stereo rows and
    RDS bits of three channels equal the oracle's on the same input bytes, block for block, and the
    timed run -- on the engine's pooled contexts (sdr_ctx_reset), streams and pinned buffers, after
    the warm-up runs -- reproduces the first run's rows."""
    import hashlib
    import sys
    import torch
    sys.path.insert(0, str(ROOT))
    import bench
    nch, nb, ch = 8, 12, [0, 3, 7]
    out = tmp_path / "cap.npz"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--queue-child", "--channels", str(nch), "--blocks",
                        str(nb), "--cus", "16", "--cap-ch", ",".join(map(str, ch)), "--cap-out", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    q = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert q["blocks"] == nb and q["persistent"] == 1 and q["pll_period_ms"] > 0
    assert q["timed_run_equal"] is True
    iq = bench.make_input(torch, nch, nb, first_channel=0, device=torch.device("cuda", 0))[:, ch].cpu().numpy()
    assert hashlib.sha256(np.ascontiguousarray(iq).tobytes()).hexdigest() == q["iq_sha"]
    got = np.load(out)
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    for i, c in enumerate(ch):
        ref = oracle.run_channel(np.ascontiguousarray(iq[:, i]), 0, True)
        for b in range(nb):
            assert np.array_equal(got["lr"][b, i], ref["stereo"][b]), f"stereo ch{c} block {b}"
            rb = ref["bits"][b]
            if rb is None:
                assert got["nbits"][b, i] == -1, f"nbits ch{c} block {b}"
            else:
                assert got["nbits"][b, i] == len(rb)
                assert np.array_equal(got["bits"][b, i, :len(rb)], rb.astype(np.uint8)), f"bits ch{c} block {b}"
