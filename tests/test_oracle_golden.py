"""CPU: pin the oracle (C restatement) to the golden vectors of the unmodified reference, and
the deterministic synthetic input to the hashes the fixtures were made on."""
from __future__ import annotations

import json

import numpy as np
import pytest

from conftest import GOLD, channel_input, sha

GOLD_CH = (0, 3)


def _bitstr(a):
    return "".join(str(int(v)) for v in a)


def test_synth_input_is_deterministic(synth, golden, golden_long):
    for c in GOLD_CH:
        nb = len(golden[f"ch{c}_fm_demod_sha256"])
        channel_input(synth, c, nb, str(golden[f"ch{c}_input_sha256"]))
    iq = channel_input(synth, 0, golden_long["nblocks"])
    assert sha(iq) == golden_long["channels"]["0"]["input_sha256"]


def test_oracle_taps_match_reference(oracle, golden):
    cases = {
        "rf": oracle.lpf(2.4e6, 1e5, 101),                       # rffrontend.cpp:24
        "audio": oracle.lpf(240000.0, 16000.0, 101, 1),          # stereo.cpp:64
        "pilot": oracle.bpf(240000.0, 18.5e3, 19.5e3, 101),      # stereo.cpp:65
        "stereo": oracle.bpf(240000.0, 22e3, 54e3, 101),         # stereo.cpp:67
        "carrier": oracle.bpf(240000.0, 37.5e3, 38.5e3, 101),    # stereo.cpp:66
        "apf": oracle.apf(1.0, 101),
        "rds": oracle.bpf(240000.0, 54e3, 60e3, 101),            # rds.cpp:62
        "rds_sq": oracle.bpf(240000.0, 113.5e3, 114.5e3, 101),   # rds.cpp:63
        "rds_bb": oracle.lpf(240000.0 * 247, 3e3, 24947, 247),   # rds.cpp:61
        "rrc": oracle.rrc(2375.0 * 39, 101),                     # rds.cpp:65
    }
    for name, h in cases.items():
        assert np.array_equal(h.view(np.uint32), golden["taps_" + name].view(np.uint32)), name


@pytest.mark.parametrize("ch", GOLD_CH)
def test_oracle_pipeline_matches_reference(oracle, synth, golden, ch):
    p = f"ch{ch}_"
    nb = len(golden[p + "fm_demod_sha256"])
    iq = channel_input(synth, ch, nb, str(golden[p + "input_sha256"]))
    out = oracle.run_channel(iq, 0, True, intermediates_at=(0, 1, 7) if ch == 0 else ())
    for b in range(nb):
        assert sha(out["fm_demod"][b]) == golden[p + "fm_demod_sha256"][b], f"fm_demod block {b}"
        assert sha(out["mono"][b]) == golden[p + "mono_sha256"][b], f"mono block {b}"
        assert sha(out["stereo"][b]) == golden[p + "stereo_sha256"][b], f"stereo block {b}"
        assert sha(out["rds_clean"][b]) == golden[p + "rds_clean_sha256"][b], f"rds_clean block {b}"
        want = str(golden[p + "bits"][b])
        if want:
            assert out["offset"][b] == int(golden[p + "offset"][b])
            assert _bitstr(out["symbols"][b]) == str(golden[p + "symbols"][b])
            assert _bitstr(out["bits"][b]) == want
        else:
            assert out["bits"][b] is None
    for b in range(4):
        assert np.array_equal(out["fm_demod"][b].view(np.uint32), golden[p + "fm_demod_head"][b].view(np.uint32))
    if ch == 0:
        for b in (0, 1, 7):
            for name in ("pilot", "carrier", "band", "stereo_dc", "mono_delay", "rds_band", "gen_pilot", "ipll",
                         "rds_dc", "rds_filt"):
                ref = golden[f"ch0_b{b}_{name}"]
                got = out["intermediates"][b][name]
                # == (not bitwise): the reference's APF delay turns -0 into +0
                assert np.array_equal(got, ref), f"{name} block {b}"


def test_oracle_long_run_bits(oracle, synth, golden_long):
    """200 blocks of channel 0: cdr offsets and decoded bits of every block, plus output hashes."""
    nb = golden_long["nblocks"]
    fix = golden_long["channels"]["0"]
    iq = channel_input(synth, 0, nb, fix["input_sha256"])
    ch = oracle.Channel(0, True)
    for b, want in enumerate(fix["blocks"]):
        fm = ch.frontend(iq[b])
        assert sha(fm) == want["fm_demod_sha256"], f"fm_demod block {b}"
        assert sha(ch.stereo(fm)) == want["stereo_sha256"], f"stereo block {b}"
        r = ch.rds(fm)
        assert sha(r["rds_clean"]) == want["rds_clean_sha256"], f"rds_clean block {b}"
        if "bits" in want:
            assert r["offset"] == want["offset"] and _bitstr(r["bits"]) == want["bits"], f"bits block {b}"


def test_reference_program_pins_stage_glue(golden):
    """project_e2e.json: the real reference binary's PCM equals the golden per-block audio."""
    e2e = json.loads((GOLD / "project_e2e.json").read_text())
    mono = np.stack([golden["ch0_mono_head"][b] for b in range(4)])
    assert e2e["m"]["whole_blocks"] >= 20 and e2e["r"]["whole_blocks"] >= 20
    assert "PI: 1000" in e2e["r"]["stderr"] and "PTY: Country" in e2e["r"]["stderr"]
    assert mono.shape == (4, 1470)


def test_rds_group_encoder_syndromes(synth):
    """The generator's RDS blocks carry valid checkwords: syndromes A,B,C,D of IEC 62106."""
    H = 0x5B9
    def syndrome(block26):
        reg = block26
        for bit in range(25, 9, -1):
            if reg & (1 << bit):
                reg ^= H << (bit - 10)
        return reg & 0x3FF
    blocks = synth.rds_group_0a(0x1234, 10, 2, "MI355XFM")
    offs = [0x0FC, 0x198, 0x168, 0x1B4]
    for blk, off in zip(blocks, offs):
        assert syndrome(blk) == off


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_oracle_modes_123_golden(oracle, synth, mode):
    """golden_modes123.json (the unmodified reference in modes 1-3, project.cpp:76-103): the oracle's
    1.44 / 1.152 MS/s front ends and 147/800, 147/1280 resamplers, every output of 7 blocks."""
    fix = json.loads((GOLD / "golden_modes123.json").read_text())
    m = fix["modes"][str(mode)]
    src = synth.FMMultiplexSource(fix["channel"])
    iq = np.stack([src.next_block(m["block_iq"]) for _ in range(fix["nblocks"])])
    assert sha(iq) == m["input_sha256"]
    ch = oracle.Channel(mode, True)
    for b, want in enumerate(m["blocks"]):
        fm = ch.frontend(iq[b])
        assert sha(fm) == want["fm_demod_sha256"], f"mode {mode} fm_demod block {b}"
        assert sha(ch.mono(fm)) == want["mono_sha256"], f"mode {mode} mono block {b}"
        assert sha(ch.stereo(fm)) == want["stereo_sha256"], f"mode {mode} stereo block {b}"
        r = ch.rds(fm)
        assert sha(r["rds_clean"]) == want["rds_clean_sha256"], f"mode {mode} rds_clean block {b}"
        if "bits" in want:
            assert r["offset"] == want["offset"] and _bitstr(r["bits"]) == want["bits"], f"mode {mode} bits {b}"
        else:
            assert r["bits"] is None
