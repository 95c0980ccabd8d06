#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the UNMODIFIED reference (run in the build container only).

Needs /root/reference (read-only) and g++: `make -C oracle ref` compiles the reference sources
where they lie into oracle/_ref/ (git-ignored). Nothing from the reference is copied here; the
fixtures are data: inputs are regenerated from real-time-sdr_amd/synth.py (their SHA-256 is
stored) and the outputs are what the reference computes on them.

  golden_mode0.npz        mode 0, channels 0 and 3, 24 blocks: taps, per-block SHA-256 of every
                          output, full arrays for blocks 0-3, intermediates for blocks 0, 1, 7 (ch 0)
  golden_mode0_long.json  mode 0, channels 0 and 3, 200 blocks (6.1 s, PLL phase > 2^21 rad):
                          per-block cdr offset, symbols, decoded RDS bits, output hashes, RDS text
  project_e2e.json        the real reference program `project 0 m|s|r` on channel 0's input:
                          SHA-256 of its stdout PCM (whole blocks) and its RDS stderr text,
                          which pins the stage glue of oracle/ref_harness.cpp
  golden_modes123.json    modes 1-3 (project.cpp:76-103: 1.44 / 2.4 / 1.152 MS/s front ends, the
                          147/800 and 147/1280 audio resamplers), channel 7, 7 blocks each: per-block
                          SHA-256 of every output, cdr offsets, symbols and bits

usage: python tests/golden/make_golden.py [--modes-only]
"""
from __future__ import annotations

import hashlib
import json
import pathlib
import subprocess
import sys
import tempfile

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT / "real-time-sdr_amd"))
import synth  # noqa: E402

REF = ROOT / "oracle" / "_ref"
CHANNELS = (0, 3)
N_SHORT = 24
N_LONG = 200
DUMP_BLOCKS = (0, 1, 7)
BLOCK_IF = 7350
N_AUDIO = 1470
N_RDS = 2836


def sha(a: np.ndarray | bytes) -> str:
    return hashlib.sha256(a if isinstance(a, bytes) else np.ascontiguousarray(a).tobytes()).hexdigest()


def gen_input(ch: int, nblocks: int) -> np.ndarray:
    src = synth.FMMultiplexSource(ch)
    return np.stack([src.next_block() for _ in range(nblocks)])


def run_harness(iq: np.ndarray, tmp: pathlib.Path, tag: str, dump=DUMP_BLOCKS) -> dict:
    inp = tmp / f"{tag}.u8"
    iq.tofile(inp)
    pre = str(tmp / f"{tag}_")
    subprocess.run([str(REF / "ref_harness"), str(inp), str(len(iq)), "0", "1", pre] + [str(b) for b in dump],
                   check=True)
    nb = len(iq)
    ld = lambda n, dt=np.float32: np.fromfile(pre + n, dt)  # noqa: E731
    out = {
        "fm_demod": ld("fm_demod.f32").reshape(nb, BLOCK_IF),
        "mono": ld("mono.i16", np.int16).reshape(nb, N_AUDIO),
        "stereo": ld("stereo.i16", np.int16).reshape(nb, 2 * N_AUDIO),
        "rds_clean": ld("rds_clean.f32").reshape(nb, N_RDS),
        "rds_text": open(pre + "rds_text.txt").read(),
        "taps": {t: ld(f"taps_{t}.f32") for t in ("rf", "audio", "pilot", "stereo", "carrier", "apf", "rds",
                                                   "rds_sq", "rds_bb", "rrc")},
        "inter": {b: {n: ld(f"b{b}_{n}.f32") for n in ("I_ds", "Q_ds", "pilot", "carrier", "band", "stereo_dc",
                                                       "mono_delay", "rds_band", "gen_pilot", "ipll", "rds_dc",
                                                       "rds_filt")}
                  for b in dump},
        "blocks": [],
    }
    for line in open(pre + "bits.txt").read().splitlines():
        p = line.split()
        if len(p) > 1:
            out["blocks"].append({"block": int(p[0]), "offset": int(p[1]), "symbols": p[2], "bits": p[3]})
        else:
            out["blocks"].append({"block": int(p[0])})
    return out


MODES_CHANNEL = 7
MODES_NBLOCKS = 7


def make_modes(tmp: pathlib.Path) -> dict:
    """golden_modes123.json: the reference harness in modes 1-3 on channel 7's input."""
    fix = {"channel": MODES_CHANNEL, "nblocks": MODES_NBLOCKS, "modes": {}}
    for mode in (1, 2, 3):
        U, D, decim = {1: (1, 9, 4), 2: (147, 800, 10), 3: (147, 1280, 3)}[mode]
        block_iq = (1470 * decim * D) // U
        src = synth.FMMultiplexSource(MODES_CHANNEL)
        iq = np.stack([src.next_block(block_iq) for _ in range(MODES_NBLOCKS)])
        inp = tmp / f"m{mode}.u8"
        iq.tofile(inp)
        pre = str(tmp / f"m{mode}_")
        subprocess.run([str(REF / "ref_harness"), str(inp), str(MODES_NBLOCKS), str(mode), "1", pre], check=True)
        nb = MODES_NBLOCKS
        outs = {"fm_demod": np.fromfile(pre + "fm_demod.f32", np.float32).reshape(nb, -1),
                "mono": np.fromfile(pre + "mono.i16", np.int16).reshape(nb, -1),
                "stereo": np.fromfile(pre + "stereo.i16", np.int16).reshape(nb, -1),
                "rds_clean": np.fromfile(pre + "rds_clean.f32", np.float32).reshape(nb, -1)}
        blocks = []
        for i, line in enumerate(open(pre + "bits.txt").read().splitlines()):
            p = line.split()
            b = {"block": int(p[0])}
            if len(p) > 1:
                b.update({"offset": int(p[1]), "symbols": p[2], "bits": p[3]})
            b.update({k + "_sha256": sha(v[i]) for k, v in outs.items()})
            blocks.append(b)
        fix["modes"][str(mode)] = {"block_iq": block_iq, "input_sha256": sha(iq),
                                   "lengths": {k: int(v.shape[1]) for k, v in outs.items()},
                                   "blocks": blocks}
    return fix


def main() -> None:
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref", "oracle"], check=True)
    if "--modes-only" in sys.argv:
        with tempfile.TemporaryDirectory() as td:
            fix = make_modes(pathlib.Path(td))
        (GOLD / "golden_modes123.json").write_text(json.dumps(fix, indent=0) + "\n")
        print("wrote golden_modes123.json")
        return
    npz: dict[str, np.ndarray] = {}
    long_fix: dict = {"channels": {}, "nblocks": N_LONG, "mode": 0}
    with tempfile.TemporaryDirectory() as td:
        tmp = pathlib.Path(td)
        for ch in CHANNELS:
            iq = gen_input(ch, N_LONG)
            short = run_harness(iq[:N_SHORT], tmp, f"s{ch}")
            p = f"ch{ch}_"
            npz[p + "input_sha256"] = np.array(sha(iq[:N_SHORT]))
            for k in ("fm_demod", "mono", "stereo", "rds_clean"):
                npz[p + k + "_head"] = short[k][:4]
                npz[p + k + "_sha256"] = np.array([sha(x) for x in short[k]])
            npz[p + "offset"] = np.array([b.get("offset", -1) for b in short["blocks"]], np.int32)
            npz[p + "symbols"] = np.array([b.get("symbols", "") for b in short["blocks"]])
            npz[p + "bits"] = np.array([b.get("bits", "") for b in short["blocks"]])
            if ch == CHANNELS[0]:
                for t, h in short["taps"].items():
                    npz["taps_" + t] = h
                for b, d in short["inter"].items():
                    for n, a in d.items():
                        npz[f"ch{ch}_b{b}_{n}"] = a
            lg = run_harness(iq, tmp, f"l{ch}", dump=())
            long_fix["channels"][str(ch)] = {
                "input_sha256": sha(iq),
                "rds_text": lg["rds_text"],
                "blocks": [dict(b, **{k + "_sha256": sha(lg[k][i]) for k in ("fm_demod", "mono", "stereo",
                                                                            "rds_clean")})
                           for i, b in enumerate(lg["blocks"])],
            }
            if ch == CHANNELS[0]:
                e2e = {"input": f"synth channel {ch}, {N_SHORT} blocks", "input_sha256": sha(iq[:N_SHORT])}
                inp = tmp / "e2e.u8"
                iq[:N_SHORT].tofile(inp)
                for t in ("m", "s", "r"):
                    with open(inp, "rb") as fi:
                        r = subprocess.run([str(REF / "project"), "0", t], stdin=fi, capture_output=True)
                    pcm = np.frombuffer(r.stdout, np.int16)
                    per = N_AUDIO if t == "m" else 2 * N_AUDIO
                    nwhole = len(pcm) // per
                    # the reference's exit(1) on EOF races the consumer threads: the last
                    # 1-2 blocks may be missing, so pin whole blocks only
                    want = (short["mono"] if t == "m" else short["stereo"])[:nwhole].reshape(-1)
                    assert np.array_equal(pcm[: nwhole * per], want), f"project 0 {t} disagrees with harness"
                    e2e[t] = {"whole_blocks": int(nwhole), "pcm_sha256": sha(pcm[: nwhole * per]),
                              "stderr": r.stderr.decode()}
                assert e2e["r"]["stderr"] == short["rds_text"], "RDS text of project 0 r != harness"
                (GOLD / "project_e2e.json").write_text(json.dumps(e2e, indent=1) + "\n")
        (GOLD / "golden_modes123.json").write_text(json.dumps(make_modes(tmp), indent=0) + "\n")
    np.savez_compressed(GOLD / "golden_mode0.npz", **npz)
    (GOLD / "golden_mode0_long.json").write_text(json.dumps(long_fix, indent=0) + "\n")
    print("wrote", sorted(p.name for p in GOLD.iterdir()))


if __name__ == "__main__":
    main()
