"""GPU parity of the fused batched pipeline (libsdr_amd.so via the C ABI) against the golden
vectors of the unmodified reference and against the oracle. Bar: bit-exact (exact mode)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import ROOT, channel_input, sha

pytestmark = pytest.mark.gpu

GOLD_CH = (0, 3)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _run_pipeline(pkg, torch, iq_by_ch, nblocks, mode=0, rds_on=True, flags=0, row_align=1):
    """iq_by_ch: list of [nblocks][2*block_iq] u8 arrays. Returns per-block host outputs.
    row_align > 1 pads every channel row to that many bytes (a strided view is passed)."""
    nch = len(iq_by_ch)
    pipe = pkg.Pipeline(nch, mode=mode, rds_on=rds_on, flags=flags)
    host = np.stack(iq_by_ch, axis=1)  # [blk][ch][bytes]
    row = host.shape[2]
    iq = torch.empty(host.shape[0], nch, (row + row_align - 1) // row_align * row_align, dtype=torch.uint8,
                     device="cuda")[:, :, :row]
    iq.copy_(torch.from_numpy(host))
    out = {k: [] for k in ("fm", "mono", "stereo", "clean", "offset", "nsym", "symbols", "nbits", "bits")}
    for b in range(nblocks):
        pipe.frontend(iq[b])
        out["fm"].append(pipe.fm_demod().cpu().numpy())
        out["mono"].append(pipe.mono().cpu().numpy())
        out["stereo"].append(pipe.stereo().cpu().numpy())
        out["clean"].append(pipe.rds().cpu().numpy())
        out["offset"].append(pipe.offset.cpu().numpy().copy())
        out["nsym"].append(pipe.nsym.cpu().numpy().copy())
        out["symbols"].append(pipe.symbols.cpu().numpy().copy())
        out["nbits"].append(pipe.nbits.cpu().numpy().copy())
        out["bits"].append(pipe.bits.cpu().numpy().copy())
    pipe.close()
    return out


def _bitstr(a, n):
    return "".join(str(int(v)) for v in a[:n])


def test_pipeline_matches_reference_golden(pkg, synth, golden, torch_cuda):
    nb = len(golden["ch0_fm_demod_sha256"])
    iqs = [channel_input(synth, c, nb, str(golden[f"ch{c}_input_sha256"])) for c in GOLD_CH]
    out = _run_pipeline(pkg, torch_cuda, iqs, nb)
    for j, c in enumerate(GOLD_CH):
        p = f"ch{c}_"
        for b in range(nb):
            assert sha(out["fm"][b][j]) == golden[p + "fm_demod_sha256"][b], f"fm_demod ch{c} block {b}"
            assert sha(out["mono"][b][j]) == golden[p + "mono_sha256"][b], f"mono ch{c} block {b}"
            assert sha(out["stereo"][b][j]) == golden[p + "stereo_sha256"][b], f"stereo ch{c} block {b}"
            assert sha(out["clean"][b][j]) == golden[p + "rds_clean_sha256"][b], f"rds_clean ch{c} block {b}"
            want_bits = str(golden[p + "bits"][b])
            if want_bits:
                assert int(out["offset"][b][j]) == int(golden[p + "offset"][b])
                ns = int(out["nsym"][b][j])
                assert _bitstr(out["symbols"][b][j], ns) == str(golden[p + "symbols"][b]), f"symbols ch{c} b{b}"
                assert _bitstr(out["bits"][b][j], int(out["nbits"][b][j])) == want_bits, f"bits ch{c} block {b}"
            else:
                assert int(out["nbits"][b][j]) == -1


def test_pipeline_long_run_bits(pkg, synth, golden_long, torch_cuda):
    """200 blocks (6.1 s): the 114 kHz PLL phase passes 2^21 rad; RDS bits must stay bit-exact."""
    nb = golden_long["nblocks"]
    chans = [int(c) for c in golden_long["channels"]]
    iqs = [channel_input(synth, c, nb, golden_long["channels"][str(c)]["input_sha256"]) for c in chans]
    out = _run_pipeline(pkg, torch_cuda, iqs, nb)
    float_mismatch = 0
    for j, c in enumerate(chans):
        blocks = golden_long["channels"][str(c)]["blocks"]
        for b, want in enumerate(blocks):
            if "bits" in want:
                assert int(out["offset"][b][j]) == want["offset"], f"cdr offset ch{c} block {b}"
                assert _bitstr(out["bits"][b][j], int(out["nbits"][b][j])) == want["bits"], f"bits ch{c} block {b}"
            for k, key in (("fm", "fm_demod"), ("mono", "mono"), ("stereo", "stereo"), ("clean", "rds_clean")):
                if sha(out[k][b][j]) != want[key + "_sha256"]:
                    float_mismatch += 1
    # the front end has no transcendental: it must be exact on every block
    for j, c in enumerate(chans):
        for b, want in enumerate(golden_long["channels"][str(c)]["blocks"]):
            assert sha(out["fm"][b][j]) == want["fm_demod_sha256"], f"fm_demod ch{c} block {b}"
    assert float_mismatch == 0, f"{float_mismatch} block outputs differ from the reference"


@pytest.mark.parametrize("row_align", [1, 16], ids=["rows_8B_aligned", "rows_16B_aligned"])
def test_pipeline_many_channels_vs_oracle(pkg, synth, oracle, torch_cuda, row_align):
    """A wider batch (ragged: 67 channels) checked per channel against the oracle on a few blocks
    (channel 63 and 64 straddle a k_frontend3 wave's channel boundary at some segment)."""
    nch, nb = 67, 8
    iqs = [channel_input(synth, 100 + c, nb) for c in range(nch)]
    out = _run_pipeline(pkg, torch_cuda, iqs, nb, row_align=row_align)
    for c in (0, 1, 31, 63, 64, 66):
        ref = oracle.run_channel(iqs[c], 0, True)
        for b in range(nb):
            assert np.array_equal(out["fm"][b][c].view(np.uint32), ref["fm_demod"][b].view(np.uint32))
            assert np.array_equal(out["stereo"][b][c], ref["stereo"][b])
            assert np.array_equal(out["mono"][b][c], ref["mono"][b])
            assert np.array_equal(out["clean"][b][c].view(np.uint32), ref["rds_clean"][b].view(np.uint32))
            if ref["bits"][b] is not None:
                assert _bitstr(out["bits"][b][c], int(out["nbits"][b][c])) == _bitstr(ref["bits"][b], len(ref["bits"][b]))


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_other_modes_vs_oracle(pkg, synth, oracle, torch_cuda, mode):
    """Modes 1-3 (project.cpp:76-103): other decimations and the 147/800, 147/1280 resamplers."""
    import real_time_sdr_amd.synth as s
    ch = oracle.Channel(mode, True)
    nb = 7
    src = s.FMMultiplexSource(7)
    iq = np.stack([src.next_block(ch.block_iq) for _ in range(nb)])
    out = _run_pipeline(pkg, torch_cuda, [iq], nb, mode=mode)
    ref = oracle.run_channel(iq, mode, True)
    # pinned to the unmodified reference (tests/golden/golden_modes123.json)
    import json
    from conftest import GOLD
    fix = json.loads((GOLD / "golden_modes123.json").read_text())["modes"][str(mode)]
    assert sha(iq) == fix["input_sha256"]
    for b, want in enumerate(fix["blocks"]):
        for k, key in (("fm", "fm_demod"), ("mono", "mono"), ("stereo", "stereo"), ("clean", "rds_clean")):
            assert sha(out[k][b][0]) == want[key + "_sha256"], f"mode {mode} {key} block {b} vs reference"
        if "bits" in want:
            assert _bitstr(out["bits"][b][0], int(out["nbits"][b][0])) == want["bits"], f"mode {mode} bits {b}"
    for b in range(nb):
        assert np.array_equal(out["fm"][b][0].view(np.uint32), ref["fm_demod"][b].view(np.uint32)), f"fm b{b}"
        assert np.array_equal(out["mono"][b][0], ref["mono"][b]), f"mono b{b}"
        assert np.array_equal(out["stereo"][b][0], ref["stereo"][b]), f"stereo b{b}"
        assert np.array_equal(out["clean"][b][0].view(np.uint32), ref["rds_clean"][b].view(np.uint32)), f"rds b{b}"
        if ref["bits"][b] is not None:
            assert _bitstr(out["bits"][b][0], int(out["nbits"][b][0])) == _bitstr(ref["bits"][b], len(ref["bits"][b]))


@pytest.mark.parametrize("row_align", [1, 16], ids=["rows_8B_aligned", "rows_16B_aligned"])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_fast_frontend_modes_vs_oracle(pkg, synth, oracle, torch_cuda, mode, row_align):
    """The MFMA front end for every decimation (D = 10, 4, 10, 3): fm_demod within 1e-5 of the
    reference (normwise per block) on 3 channels x 7 blocks, including the first block (previous
    block's tail) and the end of each block (padding)."""
    import real_time_sdr_amd.synth as s
    ch = oracle.Channel(mode, True)
    nb, nch = 7, 3
    iqs = []
    for c in range(nch):
        src = s.FMMultiplexSource(40 + c)
        iqs.append(np.stack([src.next_block(ch.block_iq) for _ in range(nb)]))
    out = _run_pipeline(pkg, torch_cuda, iqs, nb, mode=mode, flags=pkg.FLAG_FAST_FRONTEND, row_align=row_align)
    for c in range(nch):
        ref = oracle.run_channel(iqs[c], mode, True)
        for b in range(nb):
            got, want = out["fm"][b][c].astype(np.float64), ref["fm_demod"][b].astype(np.float64)
            scale = np.max(np.abs(want))
            err = np.max(np.abs(got - want))
            assert err <= 1e-5 * scale, f"mode {mode} ch {c} block {b}: {err / scale:.2e}"


@pytest.mark.parametrize("fast", [False, True], ids=["exact", "fast_mfma"])
@pytest.mark.parametrize("mode", [0, 1, 3])
def test_frontend_timing_stamps(pkg, synth, torch_cuda, fast, mode):
    """sdr_frontend_timing on the exact (k_frontend2) and MFMA (k_frontend_mfma) front ends: the
    timed launches stamp their workgroups (bench.py's roofline launch time), report one positive span
    per launch, in order and without overlap on one stream, and leave fm_demod bit-identical to
    untimed launches on the same bytes (modes 0, 1, 3: D = 10, 4, 3)."""
    import real_time_sdr_amd.synth as s
    torch = torch_cuda
    nch, nb = 40, 4
    flags = pkg.FLAG_FAST_FRONTEND if fast else 0
    p0 = pkg.Pipeline(1, mode=mode)
    block_iq = p0.info.block_iq
    p0.close()
    srcs = [s.FMMultiplexSource(70 + c) for c in range(nch)]
    host = np.stack([np.stack([src.next_block(block_iq) for src in srcs]) for _ in range(nb)])
    iq = torch.from_numpy(host).cuda()
    fms = []
    for timed in (False, True):
        pipe = pkg.Pipeline(nch, mode=mode, flags=flags)
        if timed:
            pipe.frontend_timing(nb)
        got = []
        for b in range(nb):
            pipe.frontend(iq[b])
            got.append(pipe.fm_demod().cpu().numpy())
        if timed:
            ms = pipe.frontend_times(nb)
            t0, t1 = pipe.frontend_stamps(nb)
            assert len(ms) == nb and all(0.0 < v < 50.0 for v in ms), ms
            assert all(t1[i] <= t0[i + 1] for i in range(nb - 1)), (t0, t1)
        fms.append(got)
        pipe.close()
    for b in range(nb):
        assert np.array_equal(fms[0][b], fms[1][b]), f"block {b}: timing changed fm_demod"


def test_reset_restarts_stream(pkg, synth, torch_cuda):
    iq = channel_input(synth, 0, 3)
    torch = torch_cuda
    pipe = pkg.Pipeline(1)
    d = torch.from_numpy(iq).cuda()
    first = []
    for b in range(3):
        pipe.frontend(d[b:b + 1])
        first.append(pipe.fm_demod().cpu().numpy())
        pipe.stereo(); pipe.rds()
    pipe.reset()
    for b in range(3):
        pipe.frontend(d[b:b + 1])
        assert np.array_equal(pipe.fm_demod().cpu().numpy(), first[b])
        pipe.stereo(); pipe.rds()
    with pytest.raises(pkg.SdrError):
        pipe.stereo()   # at most once per block
    pipe.close()


def test_fast_pll_matches_libm_pll(pkg, synth, torch_cuda):
    """A/B on the GPU: the correctly-rounded fast PLL (default) against the per-step f64-libm PLL
    (SDR_FLAG_PLL_LIBM, the literal pll.cpp restatement) -- identical NCO outputs and RDS bits."""
    torch = torch_cuda
    nch, nb = 48, 40
    iqs = [channel_input(synth, 200 + c, nb) for c in range(nch)]
    d = torch.from_numpy(np.stack(iqs, axis=1)).cuda()
    pa = pkg.Pipeline(nch, flags=pkg.FLAG_KEEP_INTERMEDIATES)
    pb = pkg.Pipeline(nch, flags=pkg.FLAG_PLL_LIBM | pkg.FLAG_KEEP_INTERMEDIATES)
    for b in range(nb):
        for p in (pa, pb):
            p.frontend(d[b])
            p.stereo()
            p.rds()
        for name in ("carrier", "ipll"):
            xa, xb = pa.buffer(name).cpu().numpy(), pb.buffer(name).cpu().numpy()
            assert np.array_equal(xa.view(np.uint32), xb.view(np.uint32)), f"{name} block {b}"
        assert torch.equal(pa.nbits, pb.nbits) and torch.equal(pa.bits, pb.bits)
    pa.close()
    pb.close()


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_fused_post_stages_match_unfused(pkg, synth, torch_cuda, mode):
    """The default post stages (NCO + mixer + mono delay + both audio resamplers in one kernel;
    NCO + delay + mixer in one kernel for RDS; register-blocked mono resampler) against the
    unfused kernels that store every intermediate row (SDR_FLAG_KEEP_INTERMEDIATES): identical
    mono, stereo, rds_clean and RDS bits, block by block (stereo.cpp:83-107, rds.cpp:119-127,
    mono.cpp:34-42). Mode 0 resamples by 5, mode 1 by 9, mode 2 by 147/800 (unfused stereo path)."""
    torch = torch_cuda
    nch, nb = 24, 12
    pa = pkg.Pipeline(nch, mode=mode)
    pb = pkg.Pipeline(nch, mode=mode, flags=pkg.FLAG_KEEP_INTERMEDIATES)
    info = pa.info
    srcs = [synth.FMMultiplexSource(700 + c) for c in range(nch)]
    for b in range(nb):
        d = torch.from_numpy(np.stack([s_.next_block(info.block_iq) for s_ in srcs])).cuda()
        outs = []
        for p in (pa, pb):
            p.frontend(d)
            outs.append((p.mono().cpu().numpy(), p.stereo().cpu().numpy(), p.rds().cpu().numpy(),
                         p.nbits.cpu().numpy().copy(), p.bits.cpu().numpy().copy()))
        for k, name in enumerate(("mono", "stereo", "rds_clean", "nbits", "bits")):
            x, y = outs[0][k], outs[1][k]
            if x.dtype == np.float32:
                x, y = x.view(np.uint32), y.view(np.uint32)
            assert np.array_equal(x, y), f"mode {mode} block {b}: {name}"
    pa.close()
    pb.close()


@pytest.mark.parametrize("row_align", [1, 16], ids=["rows_8B_aligned", "rows_16B_aligned"])
def test_fast_frontend_tolerance_and_rds_bits(pkg, synth, golden_long, oracle, torch_cuda, row_align):
    """SDR_FLAG_FAST_FRONTEND (the int8 MFMA front end; 16-byte staging when rows are 16-byte
    aligned): fm_demod within 1e-5 relative (north-star tolerance) of the reference, and the RDS
    bit decisions of the 200-block golden run still bit-exact."""
    nb = golden_long["nblocks"]
    chans = [int(c) for c in golden_long["channels"]]
    iqs = [channel_input(synth, c, nb, golden_long["channels"][str(c)]["input_sha256"]) for c in chans]
    out = _run_pipeline(pkg, torch_cuda, iqs, nb, flags=pkg.FLAG_FAST_FRONTEND, row_align=row_align)
    ref = oracle.run_channel(iqs[0][:8], 0, True)
    for b in range(8):
        got, want = out["fm"][b][0].astype(np.float64), ref["fm_demod"][b].astype(np.float64)
        scale = np.max(np.abs(want))
        assert np.max(np.abs(got - want)) <= 1e-5 * scale, f"fm_demod block {b}"
    for j, c in enumerate(chans):
        for b, want in enumerate(golden_long["channels"][str(c)]["blocks"]):
            if "bits" in want:
                assert _bitstr(out["bits"][b][j], int(out["nbits"][b][j])) == want["bits"], f"bits ch{c} block {b}"


@pytest.mark.parametrize("fused_plls,cu_masked,pre3", [(False, False, False), (True, False, True), (True, True, False),
                                                       ("persistent", True, True)],
                         ids=["two_pll_streams", "sdr_plls_pre3", "sdr_plls_cu_masked", "persistent_cu_masked_pre3"])
def test_split_stages_on_streams_match_sequential(pkg, synth, torch_cuda, fused_plls, cu_masked, pre3):
    """bench.py's schedule: the stereo/RDS bodies split at the PLL (sdr_*_pre/_pll/_post, or both
    PLLs in one sdr_plls dispatch) on separate streams with the PLLs of block b+1 overlapping block
    b's post part -- identical audio, rds_clean and RDS bits to the one-stream sequential pipeline,
    block by block. pre3: the pre-PLL FIRs as bench.py runs them (sdr_pre: the 3-filter pass with the
    pilot and band filters as packed pairs) instead of sdr_stereo_pre + sdr_rds_pre."""
    torch = torch_cuda
    nch, nb = 40, 14
    iqs = [channel_input(synth, 300 + c, nb) for c in range(nch)]
    d = torch.from_numpy(np.stack(iqs, axis=1)).cuda()
    ref = _run_pipeline(pkg, torch, iqs, nb)
    pipe = pkg.Pipeline(nch)
    info = pipe.info
    s_fe, s_pst, s_prd, s_post = (torch.cuda.Stream() for _ in range(4))
    handles = []
    if cu_masked:   # bench.py's placement: PLLs on CUs [0, 64) (sdr_stream_create_cu_range), rest elsewhere
        import ctypes as C
        L = pkg.lib()
        L.sdr_stream_create_cu_range.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int]
        L.sdr_stream_destroy.argtypes = [C.c_void_p]
        for exclude in (1, 0, 1):
            h = C.c_void_p()
            assert L.sdr_stream_create_cu_range(C.byref(h), torch.cuda.current_device(), 0, 64, exclude) == 0
            handles.append(h.value)
        s_fe, s_pst, s_post = (torch.cuda.ExternalStream(h) for h in handles)
    ev = lambda: torch.cuda.Event()  # noqa: E731
    pre, pst, prd, post = ([ev() for _ in range(nb)] for _ in range(4))
    lr = [torch.empty(nch, 2 * info.n_audio, dtype=torch.int16, device="cuda") for _ in range(2)]
    mono = torch.empty(nch, info.n_audio, dtype=torch.int16, device="cuda")
    clean = torch.empty(nch, info.n_rds, dtype=torch.float32, device="cuda")
    got = {"mono": [], "stereo": [], "clean": [], "bits": [], "nbits": []}
    if fused_plls == "persistent":   # two launches: the second covers the rest
        pipe.plls_launch(5, stream=s_pst)
    for b in range(nb):
        if fused_plls == "persistent" and b == 5:
            pipe.plls_launch(nb - 5, stream=s_pst)
        if b >= 2:
            s_fe.wait_event(post[b - 2])
        pipe.frontend(d[b], stream=s_fe)
        pipe.mono(mono, stream=s_fe)
        with torch.cuda.stream(s_fe):
            got["mono"].append(mono.clone())
        if pre3:
            pipe.pre(stream=s_fe)
        else:
            pipe.stereo_pre(stream=s_fe)
            pipe.rds_pre(stream=s_fe)
        pre[b].record(s_fe)
        if fused_plls == "persistent":   # no events: device flags written / waited in stream order
            pipe.plls_signal(stream=s_fe)
            pipe.plls_wait(stream=s_post)
        elif fused_plls:
            s_pst.wait_event(pre[b])
            pipe.plls(stream=s_pst)
            pst[b].record(s_pst)
            prd[b].record(s_pst)
        else:
            s_pst.wait_event(pre[b])
            pipe.stereo_pll(stream=s_pst)
            pst[b].record(s_pst)
            s_prd.wait_event(pre[b])
            pipe.rds_pll(stream=s_prd)
            prd[b].record(s_prd)
        if fused_plls != "persistent":
            s_post.wait_event(pst[b])
            s_post.wait_event(prd[b])
        pipe.stereo_post(lr[b % 2], stream=s_post)
        pipe.rds_post(clean, bits=True, stream=s_post)
        with torch.cuda.stream(s_post):
            got["stereo"].append(lr[b % 2].clone())
            got["clean"].append(clean.clone())
            got["bits"].append(pipe.bits.clone())
            got["nbits"].append(pipe.nbits.clone())
        post[b].record(s_post)
    torch.cuda.synchronize()
    if fused_plls == "persistent":
        ms = pipe.plls_report(stream=s_pst)
        assert len(ms) == nb - 5 and all(0 < m < 100 for m in ms), ms
    for h in handles:
        assert pkg.lib().sdr_stream_destroy(C.c_void_p(h)) == 0
    for b in range(nb):
        assert np.array_equal(got["mono"][b].cpu().numpy(), ref["mono"][b]), f"mono block {b}"
        assert np.array_equal(got["stereo"][b].cpu().numpy(), ref["stereo"][b]), f"stereo block {b}"
        assert np.array_equal(got["clean"][b].cpu().numpy().view(np.uint32), ref["clean"][b].view(np.uint32)), \
            f"rds_clean block {b}"
        assert np.array_equal(got["nbits"][b].cpu().numpy(), ref["nbits"][b]), f"nbits block {b}"
        assert np.array_equal(got["bits"][b].cpu().numpy(), ref["bits"][b]), f"bits block {b}"
    pipe.close()


# Fast-mode bounds per output (max over a block of |got - ref|: LSB for int16, relative to the
# block's max |ref| for floats), for the PLL acquisition (blocks < FAST_LOCK_BLOCKS) and the
# locked stream. fm_demod and mono meet the north-star 1e-5 (1 LSB after short(16384 y)). The
# outputs behind the PLLs do not: pll.cpp's recurrence carries every f32 rounding of its input
# forward, so an input that differs by ~1e-6 relative moves the 19 kHz and 114 kHz PLL
# trajectories, the stereo difference signal (L-R through the 38 kHz carrier) by up to ~1 % of full
# scale and rds_clean by up to ~1 % -- measured worst: stereo 190 LSB, rds_clean 7.7e-3 (DESIGN.md
# 2). The RDS bit decisions stay bit-exact. The exact mode (the default, and what bench.py
# measures) is bit-exact everywhere.
FAST_LOCK_BLOCKS = 10
FAST_BOUNDS = {"mono": (1, 1), "stereo": (512, 512), "clean": (2e-2, 2e-2)}   # (acquisition, locked)


@pytest.mark.parametrize("row_align", [1, 16], ids=["rows_8B_aligned", "rows_16B_aligned"])
def test_fast_frontend_all_outputs_tolerance(pkg, synth, golden_long, oracle, torch_cuda, row_align):
    """SDR_FLAG_FAST_FRONTEND over the 200-block golden run (2 channels, 6.1 s, PLL phases past
    2^21 rad), every output against the oracle: fm_demod within 1e-5 relative (north star), RDS
    bits bit-exact, mono/stereo int16 and rds_clean within FAST_BOUNDS (mono.cpp:40-42,
    stereo.cpp:100-107, rds.cpp:130-167): see the comment above for why the PLL-derived outputs
    (stereo, rds_clean) cannot meet 1e-5 with any input that is not bit-identical."""
    nb = golden_long["nblocks"]
    chans = [int(c) for c in golden_long["channels"]]
    iqs = [channel_input(synth, c, nb, golden_long["channels"][str(c)]["input_sha256"]) for c in chans]
    out = _run_pipeline(pkg, torch_cuda, iqs, nb, flags=pkg.FLAG_FAST_FRONTEND, row_align=row_align)
    worst = {k: [0.0, 0.0] for k in ("fm", "clean", "mono", "stereo")}
    bad = []
    for j, c in enumerate(chans):
        ref = oracle.run_channel(iqs[j], 0, True)
        for b in range(nb):
            ph = 0 if b < FAST_LOCK_BLOCKS else 1
            for k, key in (("fm", "fm_demod"), ("clean", "rds_clean")):
                got, want = out[k][b][j].astype(np.float64), ref[key][b].astype(np.float64)
                rel = float(np.max(np.abs(got - want)) / max(np.max(np.abs(want)), 1e-30))
                worst[k][ph] = max(worst[k][ph], rel)
                lim = 1e-5 if k == "fm" else FAST_BOUNDS[k][ph]
                if rel > lim:
                    bad.append(f"{key} ch{c} block {b}: {rel:.2e}")
            for k in ("mono", "stereo"):
                d = int(np.max(np.abs(out[k][b][j].astype(np.int32) - ref[k][b].astype(np.int32))))
                worst[k][ph] = max(worst[k][ph], d)
                if d > FAST_BOUNDS[k][ph]:
                    bad.append(f"{k} ch{c} block {b}: {d} LSB")
            if ref["bits"][b] is not None:
                if _bitstr(out["bits"][b][j], int(out["nbits"][b][j])) != _bitstr(ref["bits"][b], len(ref["bits"][b])):
                    bad.append(f"bits ch{c} block {b}")
            elif int(out["nbits"][b][j]) != -1:
                bad.append(f"nbits ch{c} block {b}")
    print("fast front end worst (acquisition, locked):", worst)
    assert not bad, f"{len(bad)} out of bounds: {bad[:12]}"


@pytest.fixture
def own_queue_stream(pkg, torch_cuda):
    """Makes streams on CUs [0, 64) with their own hardware queue (sdr_stream_create_cu_range), as
    the persistent launch requires (include/sdr_amd.h); destroyed after the test."""
    import ctypes as C
    L = pkg.lib()
    L.sdr_stream_create_cu_range.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int]
    L.sdr_stream_destroy.argtypes = [C.c_void_p]
    made = []

    def make(n_cu: int = 64):
        h = C.c_void_p()
        assert L.sdr_stream_create_cu_range(C.byref(h), torch_cuda.cuda.current_device(), 0, n_cu, 0) == 0
        made.append(h.value)
        return torch_cuda.cuda.ExternalStream(h.value)

    yield make
    torch_cuda.cuda.synchronize()
    for h in made:
        L.sdr_stream_destroy(C.c_void_p(h))


def test_persistent_plls_missing_signal_times_out(pkg, synth, torch_cuda, own_queue_stream):
    """A persistent launch whose block 2 is signalled too late (after the 5 s bounded wait) ends by
    itself and never hands out a block it did not compute: blocks before it come out as in the
    one-stream pipeline, the late block's post stages write SDR_PCM_POISON audio, NaN rds_clean and
    nbits = SDR_NBITS_POISONED (include/sdr_amd.h), sdr_plls_report raises, the post calls of that
    launch's blocks then fail, and sdr_ctx_reset + a new launch recover
    (/root/reference/include/threadsafequeue.h:24-44: a consumer never sees an unpublished block)."""
    import time
    torch = torch_cuda
    nch, nb = 8, 3
    iqs = [channel_input(synth, 500 + c, nb) for c in range(nch)]
    d = torch.from_numpy(np.stack(iqs, axis=1)).cuda()
    ref = _run_pipeline(pkg, torch, iqs, nb)
    pipe = pkg.Pipeline(nch)
    s_pll, s_post = own_queue_stream(), torch.cuda.Stream()   # the PLL stream owns its queue
    # nothing on the legacy null stream while a launch is pending: the CU-masked PLL stream is a
    # blocking stream, so null-stream work (and .cpu() copies on it) would wait for the launch
    with torch.cuda.stream(torch.cuda.Stream()):
        pipe.plls_launch(nb, stream=s_pll)
        lr = torch.empty(nch, 2 * pipe.info.n_audio, dtype=torch.int16, device="cuda")
        clean = torch.empty(nch, pipe.info.n_rds, dtype=torch.float32, device="cuda")

        def block(b):
            pipe.frontend(d[b])
            pipe.stereo_pre()
            pipe.rds_pre()
            pipe.plls_signal()
            pipe.plls_wait(stream=s_post)
            pipe.stereo_post(lr, stream=s_post)
            pipe.rds_post(clean, bits=True, stream=s_post)
            s_post.synchronize()   # not torch.cuda.synchronize(): the persistent PLL may still run

        for b in range(nb - 1):
            block(b)
            assert np.array_equal(lr.cpu().numpy(), ref["stereo"][b]), f"stereo block {b}"
        time.sleep(6.5)            # the waves give up on block 2 after 5 s of waiting
        block(nb - 1)              # signalled too late: the PLL never computes it
        assert (lr.cpu().numpy() == pkg.SDR_PCM_POISON).all(), "late block: audio not poisoned"
        assert np.isnan(clean.cpu().numpy()).all(), "late block: rds_clean not poisoned"
        assert (pipe.nbits.cpu().numpy() == pkg.SDR_NBITS_POISONED).all(), "late block: nbits not poisoned"
        with pytest.raises(pkg.SdrError, match="timed out"):
            pipe.plls_report(stream=s_pll)
        # a reset context run with per-block PLL dispatches: the block whose index the timed-out
        # launch last signalled (2) reads no stale error word (pers_block kept by reset)
        pipe.reset()
        for b in range(nb):
            pipe.frontend(d[b])
            pipe.pre()
            pipe.plls()
            pipe.stereo_post(lr)
            pipe.rds_post(clean, bits=True)
            assert np.array_equal(lr.cpu().numpy(), ref["stereo"][b]), f"dispatch after reset: stereo block {b}"
            assert np.array_equal(clean.cpu().numpy().view(np.uint32), ref["clean"][b].view(np.uint32))
            assert np.array_equal(pipe.nbits.cpu().numpy(), ref["nbits"][b])
        # recovery: reset the state the poisoned launch left, a new launch, block 0 again
        pipe.reset()
        pipe.plls_launch(1, stream=s_pll)
        block(0)
        assert np.array_equal(lr.cpu().numpy(), ref["stereo"][0]), "stereo after recovery"
        assert np.array_equal(clean.cpu().numpy().view(np.uint32), ref["clean"][0].view(np.uint32))
        assert len(pipe.plls_report(stream=s_pll)) == 1
    pipe.close()


def test_release_timeout_poisons_and_fails(pkg, synth, torch_cuda):
    """A reader that never releases its block (the parity-release wait, include/sdr_amd.h): block 0's
    mono, stereo post and RDS post are queued on a stream held by a one-wave kernel for 6.5 s, so
    block 2's front end -- the same buffer parity -- waits the bounded 5 s for them and then goes on.
    That is an error, never wrong output (the reference's producer never overwrites a slot its
    consumers hold, /root/reference/include/threadsafequeue.h:24-44): the late readers, which would
    read block 2's fm_demod, and every output stage after the timeout write SDR_PCM_POISON audio, NaN
    rds_clean and nbits = SDR_NBITS_POISONED; every later call returns SDR_E_TIMEOUT; sdr_ctx_reset
    recovers (block 0 again, bit-exact)."""
    import ctypes as C
    torch = torch_cuda
    nch, nb = 8, 3
    iqs = [channel_input(synth, 600 + c, nb) for c in range(nch)]
    d = torch.from_numpy(np.stack(iqs, axis=1)).cuda()
    ref = _run_pipeline(pkg, torch, iqs, 1)
    pipe = pkg.Pipeline(nch)
    L = pkg.lib()
    L.sdr_diag_hold.argtypes = [C.c_void_p, C.c_int]
    L.sdr_diag_hold.restype = C.c_int
    info = pipe.info
    s_fe, s_rd = torch.cuda.Stream(), torch.cuda.Stream()
    mono = [torch.zeros(nch, info.n_audio, dtype=torch.int16, device="cuda") for _ in range(nb)]
    lr = [torch.zeros(nch, 2 * info.n_audio, dtype=torch.int16, device="cuda") for _ in range(nb)]
    clean = [torch.zeros(nch, info.n_rds, dtype=torch.float32, device="cuda") for _ in range(nb)]
    bits = [torch.zeros(nch, pkg.SDR_MAX_BITS, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    torch.cuda.synchronize()
    # block 0 on s_fe; its three readers on s_rd, behind the hold
    pipe.frontend(d[0], stream=s_fe)
    pipe.pre(stream=s_fe)
    pipe.plls(stream=s_fe)
    ev = torch.cuda.Event()
    ev.record(s_fe)
    s_rd.wait_event(ev)
    pkg.check(L.sdr_diag_hold(C.c_void_p(s_rd.cuda_stream), 6500), "sdr_diag_hold")
    pipe.mono(mono[0], stream=s_rd)
    pipe.stereo_post(lr[0], stream=s_rd)
    pipe.rds_post(clean[0], bits=True, stream=s_rd, bits_out=bits[0])
    # block 1: produced, not read; block 2 reuses block 0's parity and waits for its readers
    pipe.frontend(d[1], stream=s_fe)
    pipe.pre(stream=s_fe)
    pipe.plls(stream=s_fe)
    pipe.frontend(d[2], stream=s_fe)
    pipe.mono(mono[2], stream=s_fe)
    pipe.pre(stream=s_fe)
    pipe.plls(stream=s_fe)
    pipe.stereo_post(lr[2], stream=s_fe)
    pipe.rds_post(clean[2], bits=True, stream=s_fe, bits_out=bits[2])
    torch.cuda.synchronize()    # ~6.5 s: the wait gave up at 5 s, the held readers ran after it
    for b in (0, 2):
        assert (mono[b].cpu().numpy() == pkg.SDR_PCM_POISON).all(), f"block {b}: mono not poisoned"
        assert (lr[b].cpu().numpy() == pkg.SDR_PCM_POISON).all(), f"block {b}: stereo not poisoned"
        assert np.isnan(clean[b].cpu().numpy()).all(), f"block {b}: rds_clean not poisoned"
    assert (pipe.nbits.cpu().numpy() == pkg.SDR_NBITS_POISONED).all(), "nbits not poisoned"
    with pytest.raises(pkg.SdrError, match="release wait timed out") as ei:
        pipe.frontend(d[0], stream=s_fe)
    assert ei.value.code == pkg.SDR_E_TIMEOUT
    with pytest.raises(pkg.SdrError) as ei:
        pipe.mono(mono[1], stream=s_fe)
    assert ei.value.code == pkg.SDR_E_TIMEOUT
    # recovery
    pipe.reset()
    pipe.frontend(d[0])
    assert np.array_equal(pipe.mono().cpu().numpy(), ref["mono"][0]), "mono after reset"
    assert np.array_equal(pipe.stereo().cpu().numpy(), ref["stereo"][0]), "stereo after reset"
    assert np.array_equal(pipe.rds().cpu().numpy().view(np.uint32), ref["clean"][0].view(np.uint32))
    pipe.close()


def test_persistent_plls_refuses_pool_stream(pkg, torch_cuda):
    """sdr_plls_launch only accepts a stream sdr_stream_create_cu_range made (its own hardware
    queue): a plain torch stream is refused before anything is dispatched."""
    torch = torch_cuda
    pipe = pkg.Pipeline(4)
    with pytest.raises(pkg.SdrError, match="sdr_stream_create_cu_range"):
        pipe.plls_launch(2, stream=torch.cuda.Stream())
    torch.cuda.synchronize()   # nothing was launched: a pending launch would hold this for 5 s
    pipe.close()


def test_persistent_plls_refuses_unresident_waves(pkg, torch_cuda, own_queue_stream):
    """8192 channels = 512 PLL waves: at most one wave per SIMD (256 VGPRs), four per CU in groups
    sharing one trigArg table -- 256 waves on a 64-CU stream, so the launch is refused before any
    dispatch (round 3 timed out on a configuration that did not fit: 4096 channels with one table
    per wave)."""
    torch = torch_cuda
    pipe = pkg.Pipeline(8192)
    with pytest.raises(pkg.SdrError, match="do not fit"):
        pipe.plls_launch(2, stream=own_queue_stream())
    torch.cuda.synchronize()   # returns at once: nothing is pending
    pipe.close()


def test_persistent_plls_refuses_unbalanced_cu_mask(pkg, torch_cuda, own_queue_stream):
    """1536 channels = 96 PLL waves on a 48-CU stream: 2 per CU fit the CU count, but the mask puts
    2, 2, 1 and 1 of each XCC's 6 CUs on its four shader engines while workgroups are dealt to the
    engines evenly, so only 64 workgroups are resident at once (tools/microbench/cumask_probe.hip,
    profiles/r06/cumask/) -- round 5's bench hung on exactly this launch until the 5 s waits expired.
    The launch is refused before anything is enqueued, and sdr_plls_fits says so; the SE-balanced
    masks the bench uses are still accepted (/root/reference/include/threadsafequeue.h:24-44: the
    producer never waits on a consumer that cannot run)."""
    import time
    torch = torch_cuda
    pipe = pkg.Pipeline(1536)
    f48 = pipe.plls_fits(48)
    assert f48 == {"waves": 96, "groups": 96, "resident": 64, "fits": False}
    t0 = time.perf_counter()
    with pytest.raises(pkg.SdrError, match="do not fit"):
        pipe.plls_launch(2, stream=own_queue_stream(48))
    torch.cuda.synchronize()   # nothing is pending: no 5 s wait
    assert time.perf_counter() - t0 < 2.0
    assert pipe.plls_fits(64)["fits"]
    pipe.close()
    # the headline's 1024 channels: one or two waves per CU on 32 or 64 CUs, packed groups of four on
    # 16 and 24 (the staged loop, tests/test_gpu_width.py runs 16 against the oracle)
    pipe = pkg.Pipeline(1024)
    for n_cu in (16, 24, 32, 64):
        assert pipe.plls_fits(n_cu)["fits"], n_cu
    pipe.close()


def test_persistent_plls_signal_checks_block_order(pkg, synth, torch_cuda, own_queue_stream):
    """A launch fixes each block's buffer parity from the block that follows it: signalling a block
    the launch does not cover next (here: the block that was already produced when the launch was
    made) is rejected; the blocks that do follow it run and match the one-stream pipeline."""
    torch = torch_cuda
    nch, nb = 4, 3
    iqs = [channel_input(synth, 600 + c, nb) for c in range(nch)]
    d = torch.from_numpy(np.stack(iqs, axis=1)).cuda()
    ref = _run_pipeline(pkg, torch, iqs, nb)
    pipe = pkg.Pipeline(nch)
    # the PLL stream owns its hardware queue (a CU-masked stream does, include/sdr_amd.h): on a
    # pool stream the launch's waiting waves can sit in front of the signal on a shared queue
    s_pll, s_post = own_queue_stream(), torch.cuda.Stream()
    # nothing on the legacy null stream while a launch is pending: the CU-masked PLL stream is a
    # blocking stream, so null-stream work (and .cpu() copies on it) would wait for the launch
    with torch.cuda.stream(torch.cuda.Stream()):
        lr = torch.empty(nch, 2 * pipe.info.n_audio, dtype=torch.int16, device="cuda")
        pipe.frontend(d[0])
        pipe.plls_launch(nb - 1, stream=s_pll)       # covers blocks 1 and 2
        pipe.stereo_pre()
        pipe.rds_pre()
        with pytest.raises(pkg.SdrError, match="expects block 1"):
            pipe.plls_signal()
        pipe.stereo_pll()                            # block 0 the ordinary way
        pipe.rds_pll()
        pipe.stereo_post(lr)
        pipe.rds_post(None, bits=False)
        torch.cuda.current_stream().synchronize()
        assert np.array_equal(lr.cpu().numpy(), ref["stereo"][0])
        for b in range(1, nb):
            pipe.frontend(d[b])
            pipe.stereo_pre()
            pipe.rds_pre()
            pipe.plls_signal()
            pipe.plls_wait(stream=s_post)
            pipe.stereo_post(lr, stream=s_post)
            pipe.rds_post(None, bits=False, stream=s_post)
            s_post.synchronize()
            assert np.array_equal(lr.cpu().numpy(), ref["stereo"][b]), f"stereo block {b}"
        assert len(pipe.plls_report(stream=s_pll)) == nb - 1
    pipe.close()


@pytest.mark.parametrize("nch", [512, 256])
def test_persistent_plls_packed_groups_match_sequential(pkg, synth, torch_cuda, nch):
    """More PLL waves than CUs of the PLL stream: 512 channels = 32 waves on an 8-CU stream, packed in
    groups of four (one wave per SIMD) sharing one trigArg table per CU, whose blocks after the fill
    run the chunk loop that stages inputs and phases through LDS (pll_run_split_coal); 256 channels
    = 16 waves, two one-wave groups per CU (the register-prefetch loop). Audio, rds_clean and RDS
    bits equal the one-stream pipeline's, block by block."""
    import ctypes as C
    import sys
    sys.path.insert(0, str(ROOT))
    import bench
    torch = torch_cuda
    nb = 4
    d = bench.make_input(torch, nch, nb, first_channel=700, device=torch.device("cuda", 0))   # distinct channels
    ref = {"stereo": [], "clean": [], "bits": [], "nbits": []}
    one = pkg.Pipeline(nch)                         # the one-stream pipeline on the same bytes
    for b in range(nb):
        one.frontend(d[b])
        ref["stereo"].append(one.stereo().cpu().numpy())
        ref["clean"].append(one.rds().cpu().numpy())
        ref["bits"].append(one.bits.cpu().numpy().copy())
        ref["nbits"].append(one.nbits.cpu().numpy().copy())
    one.close()
    L = pkg.lib()
    L.sdr_stream_create_cu_range.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int]
    L.sdr_stream_destroy.argtypes = [C.c_void_p]
    handles = []
    for lo, n, exclude in ((0, 8, 0), (0, 8, 1), (0, 8, 1)):   # PLL on CUs [0, 8), the rest elsewhere
        h = C.c_void_p()
        assert L.sdr_stream_create_cu_range(C.byref(h), torch.cuda.current_device(), lo, n, exclude) == 0
        handles.append(h.value)
    s_pll, s_fe, s_post = (torch.cuda.ExternalStream(h) for h in handles)
    pipe = pkg.Pipeline(nch)
    info = pipe.info
    lr = [torch.empty(nch, 2 * info.n_audio, dtype=torch.int16, device="cuda") for _ in range(2)]
    clean = torch.empty(nch, info.n_rds, dtype=torch.float32, device="cuda")
    got = {"stereo": [], "clean": [], "bits": [], "nbits": []}
    post = [torch.cuda.Event() for _ in range(nb)]
    with torch.cuda.stream(torch.cuda.Stream()):    # nothing on the null stream while the launch waits
        pipe.plls_launch(nb, stream=s_pll)
        for b in range(nb):
            if b >= 2:
                s_fe.wait_event(post[b - 2])
            if b == 0:
                pipe.frontend_pre_parts(d[b], 4, stream=s_fe)    # the fill, with the packed groups
            else:
                pipe.frontend(d[b], stream=s_fe)
                pipe.pre(stream=s_fe)
                pipe.plls_signal(stream=s_fe)
            pipe.plls_wait(stream=s_post)
            pipe.stereo_post(lr[b % 2], stream=s_post)
            pipe.rds_post(clean, bits=True, stream=s_post)
            with torch.cuda.stream(s_post):
                got["stereo"].append(lr[b % 2].clone())
                got["clean"].append(clean.clone())
                got["bits"].append(pipe.bits.clone())
                got["nbits"].append(pipe.nbits.clone())
            post[b].record(s_post)
        s_post.synchronize()
        ms = pipe.plls_report(stream=s_pll)
    torch.cuda.synchronize()
    for h in handles:
        assert L.sdr_stream_destroy(C.c_void_p(h)) == 0
    assert len(ms) == nb and all(0 < m < 100 for m in ms), ms
    for b in range(nb):
        assert np.array_equal(got["stereo"][b].cpu().numpy(), ref["stereo"][b]), f"stereo block {b}"
        assert np.array_equal(got["clean"][b].cpu().numpy().view(np.uint32), ref["clean"][b].view(np.uint32)), \
            f"rds_clean block {b}"
        assert np.array_equal(got["nbits"][b].cpu().numpy(), ref["nbits"][b]), f"nbits block {b}"
        assert np.array_equal(got["bits"][b].cpu().numpy(), ref["bits"][b]), f"bits block {b}"
    pipe.close()
