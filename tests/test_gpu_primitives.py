"""GPU parity of the batched primitives (the reference's function signatures, batched over rows)
against the oracle on seeded random inputs, including ragged sizes. Bit-exact."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _u32(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("nx,D,ntaps", [(7350, 1, 101), (73500, 10, 101), (1001, 3, 31), (37, 1, 101), (2836, 1, 101)])
def test_convolve_fir(pkg, oracle, torch_cuda, nx, D, ntaps):
    torch = torch_cuda
    rng = np.random.default_rng(nx + D)
    nch = 5
    h = rng.standard_normal(ntaps).astype(np.float32) * 0.05
    x = [rng.standard_normal((nch, nx)).astype(np.float32) for _ in range(3)]
    st_ref = [np.zeros(ntaps - 1, np.float32) for _ in range(nch)]
    d_state = torch.zeros(nch, ntaps - 1, device="cuda")
    d_h = torch.from_numpy(h).cuda()
    for blk in range(3):
        d_x = torch.from_numpy(x[blk]).cuda()
        d_y = torch.zeros(nch, nx // D, device="cuda")
        pkg.convolve_fir(d_y, d_x, d_h, d_state, D)
        y = d_y.cpu().numpy()
        for c in range(nch):
            ref = oracle.fir_decim(x[blk][c], h, st_ref[c], D)
            assert np.array_equal(_u32(y[c]), _u32(ref)), f"block {blk} ch {c}"
            assert np.array_equal(_u32(d_state[c].cpu().numpy()), _u32(st_ref[c]))


@pytest.mark.parametrize("nx,U,D,ntaps", [(7350, 1, 5, 101), (7350, 247, 640, 24947), (8000, 147, 800, 14847),
                                          (13230, 1, 9, 101)])
def test_convolve_fir_resample(pkg, oracle, torch_cuda, nx, U, D, ntaps):
    torch = torch_cuda
    rng = np.random.default_rng(U * 7 + D)
    nch = 3
    h = rng.standard_normal(ntaps).astype(np.float32) * 0.01
    st_ref = [np.zeros(100, np.float32) for _ in range(nch)]
    d_state = torch.zeros(nch, 100, device="cuda")
    d_h = torch.from_numpy(h).cuda()
    for blk in range(3):
        x = rng.standard_normal((nch, nx)).astype(np.float32)
        d_y = torch.zeros(nch, nx * U // D, device="cuda")
        pkg.convolve_fir_resample(d_y, torch.from_numpy(x).cuda(), d_h, d_state, U, D)
        y = d_y.cpu().numpy()
        for c in range(nch):
            ref = oracle.fir_resample(x[c], h, st_ref[c], U, D)
            assert np.array_equal(_u32(y[c]), _u32(ref)), f"block {blk} ch {c}"


def test_fm_demod(pkg, oracle, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(5)
    nch, n = 4, 7350
    prev_ref = [np.zeros(2, np.float32) for _ in range(nch)]
    d_prev = torch.zeros(nch, 2, device="cuda")
    for blk in range(3):
        I = rng.standard_normal((nch, n)).astype(np.float32)
        Q = rng.standard_normal((nch, n)).astype(np.float32)
        I[0, 5] = 0.0
        Q[0, 5] = 0.0   # the I = Q = 0 branch (demod.cpp:11-12)
        d_out = torch.zeros(nch, n, device="cuda")
        pkg.fm_demod(d_out, torch.from_numpy(I).cuda(), torch.from_numpy(Q).cuda(), d_prev)
        out = d_out.cpu().numpy()
        for c in range(nch):
            ref = oracle.fm_demod(I[c], Q[c], prev_ref[c])
            assert np.array_equal(_u32(out[c]), _u32(ref))
            assert np.array_equal(d_prev[c].cpu().numpy(), prev_ref[c])


def test_rcp64_error_within_discriminator_bound(pkg, torch_cuda):
    """The exact front end's discriminator (sdr_frontend.hip, SDR_FE_DISC) takes RN32(num * r1) with
    r1 = v_rcp_f64(den) + one Newton step as the reference's RN32(RN64(num / den)) (demod.cpp:11-18)
    when no f32 tie lies within 2048 ulps; its bound needs the hardware reciprocal within 2^-22
    relative. Every one of the 2^24 leading-mantissa patterns (random low bits, exponents over the
    discriminator's range of I^2 + Q^2), through the library's residual kernel."""
    import ctypes as C
    torch = torch_cuda
    rng = np.random.default_rng(11)
    n = 1 << 24
    mant = (np.arange(n, dtype=np.uint64) << np.uint64(28)) | rng.integers(0, 1 << 28, n, dtype=np.uint64)
    expo = rng.integers(1023 - 200, 1023 + 40, n, dtype=np.uint64)
    x = torch.from_numpy((mant | (expo << np.uint64(52))).view(np.float64)).cuda()
    res = torch.empty_like(x)
    L = pkg.lib()
    L.sdr_diag_rcp64_residual.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.sdr_diag_rcp64_residual.restype = C.c_int
    pkg.check(L.sdr_diag_rcp64_residual(C.c_void_p(x.data_ptr()), C.c_void_p(res.data_ptr()), n,
                                        C.c_void_p(torch.cuda.current_stream().cuda_stream)), "rcp64")
    worst = float(res.abs().max().item())
    print(f"v_rcp_f64 max relative error 2^{np.log2(worst):.2f}")
    assert worst < 2.0 ** -22


@pytest.mark.parametrize("freq,nco,bw", [(19e3, 2.0, 0.01), (114e3, 0.5, 0.001)])
def test_fmpll(pkg, oracle, torch_cuda, freq, nco, bw):
    torch = torch_cuda
    nch, n = 3, 7350
    t = np.arange(4 * n) / 240000.0
    st_ref = [oracle.new_pll_state() for _ in range(nch)]
    out_ref = [np.zeros(n + 1, np.float32) for _ in range(nch)]
    for o in out_ref:
        o[-1] = 1.0
    d_st = pkg.pll_state_tensor(nch)
    for blk in range(4):
        x = np.stack([(0.1 * np.cos(2 * np.pi * freq * t[blk * n:(blk + 1) * n] + 0.3 * c)).astype(np.float32)
                      for c in range(nch)])
        d_out = torch.zeros(nch, n + 1, device="cuda")
        pkg.fmpll(d_out, torch.from_numpy(x).cuda(), freq, 240000.0, d_st, nco, 0.0, bw)
        out = d_out.cpu().numpy()
        for c in range(nch):
            oracle.fmpll(x[c], freq, 240000.0, out_ref[c], st_ref[c], nco, 0.0, bw)
            assert np.array_equal(_u32(out[c]), _u32(out_ref[c])), f"block {blk} ch {c}"
        st = pkg.pll_state_from_tensor(d_st)
        for c in range(nch):
            assert st[c].phaseEst == st_ref[c].phaseEst and st[c].trigOffset == st_ref[c].trigOffset


def test_fmpll_mixed_states(pkg, oracle, torch_cuda):
    """Channels whose PLL states differ: distinct trigOffsets (the per-lane trigArg path instead of
    the LDS table), states whose feedback does not match their trigArg (the fallback of the first
    step) and a large trigOffset (coarse f32 trigArg, pll.cpp:47), bit-exact against the oracle."""
    torch = torch_cuda
    n = 7350
    states = [(1.0, 0.0, 0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0, 12345.0),
              (0.6, 0.8, 1e-4, 0.3, 7350.0 * 40), (1.0, 0.0, 0.0, 0.0, 3.0e6), (-1.0, 0.0, 2e-5, 2.0, 99.0)]
    nch = len(states)
    for freq, nco, bw in ((19e3, 2.0, 0.01), (114e3, 0.5, 0.001)):
        arr = (pkg.PllState * nch)()
        refs = []
        for i, (fi, fq, ig, ph, to) in enumerate(states):
            arr[i] = pkg.PllState(fi, fq, ig, ph, to, 1.0)
            refs.append(oracle.PllState(fi, fq, ig, ph, to, 1.0))
        d_st = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).cuda()
        out_ref = [np.zeros(n + 1, np.float32) for _ in range(nch)]
        for o in out_ref:
            o[-1] = 1.0
        rng = np.random.default_rng(11)
        t = np.arange(2 * n) / 240000.0
        for blk in range(2):
            x = np.stack([(0.1 * np.cos(2 * np.pi * (freq + 2.0 * c) * t[blk * n:(blk + 1) * n] + 0.7 * c)
                           + 0.01 * rng.standard_normal(n)).astype(np.float32) for c in range(nch)])
            d_out = torch.zeros(nch, n + 1, device="cuda")
            pkg.fmpll(d_out, torch.from_numpy(x).cuda(), freq, 240000.0, d_st, nco, 0.0, bw)
            out = d_out.cpu().numpy()
            for c in range(nch):
                oracle.fmpll(x[c], freq, 240000.0, out_ref[c], refs[c], nco, 0.0, bw)
                assert np.array_equal(_u32(out[c]), _u32(out_ref[c])), f"{freq} block {blk} ch {c}"
            got = pkg.pll_state_from_tensor(d_st)
            for c in range(nch):
                for f in ("feedbackI", "feedbackQ", "integrator", "phaseEst", "trigOffset"):
                    assert getattr(got[c], f) == getattr(refs[c], f), f"{freq} block {blk} ch {c} {f}"


def test_cdr(pkg, oracle, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(9)
    nch, n = 6, 2836
    x = (rng.standard_normal((nch, n)) * 2.6).astype(np.float32)
    x[5] = 0.0          # all sums zero -> offset 0
    x[4, ::39] = 0.0
    d_off = torch.zeros(nch, dtype=torch.int32, device="cuda")
    pkg.cdr(d_off, torch.from_numpy(x).cuda(), 39)
    got = d_off.cpu().numpy()
    for c in range(nch):
        assert got[c] == oracle.cdr(39, x[c])


@pytest.mark.parametrize("freq,nco,bw", [(19e3, 2.0, 0.01), (114e3, 0.5, 0.001)])
def test_fmpll_full_width(pkg, oracle, torch_cuda, freq, nco, bw):
    """The bench's width: 1024 channels x 2 blocks (15M PLL steps per config) with noisy,
    per-channel detuned pilots, bit-exact against the oracle. At this size the fast path falls back
    ~170 times per config, so the fallbacks' glibc-equivalent results (pll_math.h, double-double)
    are exercised on real near-midpoint inputs, not only the proven path."""
    torch = torch_cuda
    nch, n = 1024, 7350
    rng = np.random.default_rng(5)
    st_ref = [oracle.new_pll_state() for _ in range(nch)]
    out_ref = np.zeros((nch, n + 1), np.float32)
    out_ref[:, -1] = 1.0
    d_st = pkg.pll_state_tensor(nch)
    det = rng.uniform(-3.0, 3.0, nch)[:, None]
    ph0 = rng.uniform(0, 2 * np.pi, nch)[:, None]
    amp = rng.uniform(0.02, 0.2, nch)[:, None]
    for blk in range(2):
        t = (np.arange(n) + blk * n)[None, :] / 240000.0
        x = (amp * np.cos(2 * np.pi * (freq + det) * t + ph0)
             + 0.02 * rng.standard_normal((nch, n))).astype(np.float32)
        d_out = torch.zeros(nch, n + 1, device="cuda")
        pkg.fmpll(d_out, torch.from_numpy(x).cuda(), freq, 240000.0, d_st, nco, 0.0, bw)
        out = d_out.cpu().numpy()
        bad = []
        for c in range(nch):
            oracle.fmpll(x[c], freq, 240000.0, out_ref[c], st_ref[c], nco, 0.0, bw)
            if not np.array_equal(_u32(out[c]), _u32(out_ref[c])):
                bad.append(c)
        assert not bad, f"block {blk}: {len(bad)} channels differ, first {bad[:8]}"


@pytest.mark.parametrize("freq,nco,bw", [(19e3, 2.0, 0.01), (114e3, 0.5, 0.001)])
def test_fmpll_long_stream(pkg, oracle, torch_cuda, freq, nco, bw):
    """Hours into a stream: trigOffset from 2e8 to 1.5e9 samples (pll.cpp:46-47), so trigArg passes
    the table bound (|w toff| < 1.375 * 2^29), the two-fma reduction's 2^30 (25 min for the 114 kHz
    PLL) and 2^32; past 2^30 every cos/sin is the Payne-Hanek double-double fallback (glibc's f64
    value), and the NCO's cos(t * ncoScale) with it. Two blocks, bit-exact against the oracle,
    outputs and state (the first block starts from feedback that does not match trigArg)."""
    torch = torch_cuda
    n = 7350
    toffs = [2.0e8, 2.6e8, 3.55e8, 3.6e8, 4.0e8, 7.2e8, 1.5e9, 1.5e9 + 7.0]
    nch = len(toffs)
    arr = (pkg.PllState * nch)()
    refs = []
    for i, to in enumerate(toffs):
        arr[i] = pkg.PllState(1.0, 0.0, 1e-5, 0.25, to, 1.0)
        refs.append(oracle.PllState(1.0, 0.0, 1e-5, 0.25, to, 1.0))
    d_st = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).cuda()
    out_ref = [np.zeros(n + 1, np.float32) for _ in range(nch)]
    for o in out_ref:
        o[-1] = 1.0
    rng = np.random.default_rng(23)
    for blk in range(2):
        t = (np.arange(n) + blk * n) / 240000.0
        x = np.stack([(0.1 * np.cos(2 * np.pi * (freq + 1.5 * c) * t + 0.4 * c)
                       + 0.01 * rng.standard_normal(n)).astype(np.float32) for c in range(nch)])
        d_out = torch.zeros(nch, n + 1, device="cuda")
        pkg.fmpll(d_out, torch.from_numpy(x).cuda(), freq, 240000.0, d_st, nco, 0.0, bw)
        out = d_out.cpu().numpy()
        got = pkg.pll_state_from_tensor(d_st)
        for c in range(nch):
            oracle.fmpll(x[c], freq, 240000.0, out_ref[c], refs[c], nco, 0.0, bw)
            assert np.array_equal(_u32(out[c]), _u32(out_ref[c])), f"toff {toffs[c]:g} block {blk}"
            for f in ("feedbackI", "feedbackQ", "integrator", "phaseEst", "trigOffset", "lastCarrier"):
                assert getattr(got[c], f) == getattr(refs[c], f), f"toff {toffs[c]:g} block {blk} {f}"


def test_fmpll_long_stream_shared_offset(pkg, oracle, torch_cuda):
    """64 channels sharing trigOffset just below and just above the trigArg-table bound of the
    114 kHz PLL (the context path of a long-running receiver): bit-exact against the oracle."""
    torch = torch_cuda
    n, freq, nco, bw = 7350, 114e3, 0.5, 0.001
    w = 2 * np.pi * np.float32(freq / 240000.0)
    bound = 1.375 * 2.0 ** 29   # PLL_TAB_WT_MAX
    for toff in (float(int(bound / w) - n - 2), float(int(bound / w) + 5)):
        nch = 64
        d_st = pkg.pll_state_tensor(nch)
        arr = (pkg.PllState * nch)()
        refs = []
        for i in range(nch):
            arr[i] = pkg.PllState(1.0, 0.0, 0.0, 0.0, toff, 1.0)
            refs.append(oracle.PllState(1.0, 0.0, 0.0, 0.0, toff, 1.0))
        d_st = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).cuda()
        rng = np.random.default_rng(3)
        t = np.arange(n) / 240000.0
        x = np.stack([(0.05 * np.cos(2 * np.pi * freq * t + 0.1 * c) + 0.02 * rng.standard_normal(n))
                      .astype(np.float32) for c in range(nch)])
        d_out = torch.zeros(nch, n + 1, device="cuda")
        pkg.fmpll(d_out, torch.from_numpy(x).cuda(), freq, 240000.0, d_st, nco, 0.0, bw)
        out = d_out.cpu().numpy()
        for c in range(nch):
            o = np.zeros(n + 1, np.float32)
            o[-1] = 1.0
            oracle.fmpll(x[c], freq, 240000.0, o, refs[c], nco, 0.0, bw)
            assert np.array_equal(_u32(out[c]), _u32(o)), f"toff {toff:g} ch {c}"


@pytest.mark.parametrize("nbytes", [16, 4096 + 48, 3 * (1 << 20) + 16 * 7])
def test_hbm_copy(pkg, torch_cuda, nbytes):
    """The bandwidth-calibration copy (sdr_hbm_copy) copies every byte, ragged tails included, and
    rejects misaligned sizes."""
    torch = torch_cuda
    g = torch.Generator(device="cuda").manual_seed(nbytes)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    dst = torch.zeros_like(src)
    pkg.hbm_copy(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    with pytest.raises(pkg.SdrError):
        pkg.hbm_copy(dst[:nbytes - 8], src[:nbytes - 8])
