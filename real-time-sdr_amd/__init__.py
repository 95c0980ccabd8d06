"""real-time-sdr_amd -- MI355X-native FM/RDS DSP hot path of TheZxc07/real-time-SDR.

Python binding (ctypes) of the C ABI in include/sdr_amd.h, implemented by libsdr_amd.so
(hand-written HIP kernels for gfx950). PyTorch is used only as device-memory / stream plumbing:
every call takes device pointers, and the torch helpers here just pass `tensor.data_ptr()` and
the current HIP stream. There is no CPU fallback: if the library cannot be loaded, every entry
point raises.

Reference interface mirrored (file:line in TheZxc07/real-time-SDR):
  convolveFIR (decimating)      src/filter.cpp:106-121   -> convolve_fir
  convolveFIR (resampling)      src/filter.cpp:123-147   -> convolve_fir_resample
  fmDemodNoArctan               src/demod.cpp:3-24       -> fm_demod
  fmpll / pllblock_args         src/pll.cpp:4-61         -> fmpll / PllState
  cdr                           src/rds_utilities.cpp:4-21 -> cdr
  RF_frontend / mono / stereo / rds stage bodies         -> Pipeline
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ["SDR_AMD_LIB"]) if os.environ.get("SDR_AMD_LIB") else HERE / "libsdr_amd.so"  # override: A/B experiments (tools/)

SDR_OK = 0
SDR_E_TIMEOUT = -5           # a parity-release wait gave up: outputs poisoned until reset (include/sdr_amd.h)
SDR_MAX_SYMS = 256
SDR_MAX_BITS = 256
SDR_PCM_POISON = -32768      # audio of a block whose persistent PLL or release wait timed out (include/sdr_amd.h)
SDR_NBITS_POISONED = -2      # nbits of such a block (its rds_clean rows are NaN)
FLAG_FAST_FRONTEND = 0x1
FLAG_PLL_LIBM = 0x2
FLAG_KEEP_INTERMEDIATES = 0x4

_lib = None


class SdrError(RuntimeError):
    def __init__(self, msg: str, code: int | None = None):
        super().__init__(msg)
        self.code = code


class PllState(C.Structure):
    """pllblock_args (include/pll.h:10-17); lastCarrier doubles as pllOut[last] (pll.cpp:18)."""
    _fields_ = [("feedbackI", C.c_float), ("feedbackQ", C.c_float), ("integrator", C.c_float),
                ("phaseEst", C.c_float), ("trigOffset", C.c_double), ("lastCarrier", C.c_float)]


class Info(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("nch", "mode", "rds_on", "rf_Fs", "rf_decim", "if_Fs", "audio_upsample",
                                        "audio_decim", "symbol_Fs", "rf_taps", "block_iq", "block_if", "n_audio",
                                        "n_rds", "history")]


def lib() -> C.CDLL:
    """Load libsdr_amd.so (built in-tree by __graft_entry__.build() / `make`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise SdrError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(os.fspath(LIB_PATH))
    vp, sz, i32, f32 = C.c_void_p, C.c_size_t, C.c_int, C.c_float
    sigs = {
        "sdr_last_error": ([], C.c_char_p),
        "sdr_version": ([], i32),
        "sdr_impulse_response_lpf": ([f32, f32, C.c_ushort, vp], i32),
        "sdr_impulse_response_lpf_gain": ([f32, f32, C.c_ushort, i32, vp], i32),
        "sdr_impulse_response_bpf": ([f32, vp, C.c_ushort, vp], i32),
        "sdr_impulse_response_apf": ([f32, C.c_ushort, vp], i32),
        "sdr_impulse_response_rrc": ([f32, C.c_ushort, vp], i32),
        "sdr_convolve_fir": ([vp, sz, vp, sz, i32, i32, vp, i32, vp, i32, i32, vp], i32),
        "sdr_convolve_fir_resample": ([vp, sz, vp, sz, i32, i32, vp, i32, vp, i32, i32, i32, vp], i32),
        "sdr_fm_demod": ([vp, sz, vp, vp, sz, i32, i32, vp, vp], i32),
        "sdr_fmpll": ([vp, sz, vp, sz, i32, i32, f32, f32, vp, f32, f32, f32, vp], i32),
        "sdr_cdr": ([vp, vp, sz, i32, i32, i32, vp], i32),
        "sdr_ctx_create": ([C.POINTER(vp), i32, i32, i32, i32, i32], i32),
        "sdr_ctx_destroy": ([vp], i32),
        "sdr_ctx_reset": ([vp, vp], i32),
        "sdr_ctx_info": ([vp, C.POINTER(Info)], i32),
        "sdr_frontend": ([vp, vp, sz, vp], i32),
        "sdr_frontend_release_wait": ([vp, vp], i32),
        "sdr_frontend_timing": ([vp, i32], i32),
        "sdr_frontend_times": ([vp, C.POINTER(C.c_double), i32, C.POINTER(i32)], i32),
        "sdr_frontend_stamps": ([vp, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong), i32, C.POINTER(i32)], i32),
        "sdr_mono": ([vp, vp, sz, vp], i32),
        "sdr_stereo": ([vp, vp, sz, vp], i32),
        "sdr_rds_dsp": ([vp, vp, sz, vp], i32),
        "sdr_rds_bits": ([vp, vp, vp, vp, sz, vp, vp, sz, vp], i32),
        "sdr_get_fm_demod": ([vp, vp, sz, vp], i32),
        "sdr_push_fm_demod": ([vp, vp, sz, vp], i32),
        "sdr_stereo_pre": ([vp, vp], i32),
        "sdr_stereo_pll": ([vp, vp], i32),
        "sdr_stereo_post": ([vp, vp, sz, vp], i32),
        "sdr_rds_pre": ([vp, vp], i32),
        "sdr_pre": ([vp, vp], i32),
        "sdr_rds_pll": ([vp, vp], i32),
        "sdr_plls": ([vp, vp], i32),
        "sdr_plls_launch": ([vp, i32, vp], i32),
        "sdr_plls_prepare": ([vp, i32, vp], i32),
        "sdr_plls_fits": ([vp, i32, i32, i32, C.POINTER(i32), C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)], i32),
        "sdr_plls_launch_sel": ([vp, i32, i32, vp], i32),
        "sdr_plls_signal": ([vp, vp], i32),
        "sdr_frontend_pre_parts": ([vp, vp, sz, i32, vp], i32),
        "sdr_plls_wait": ([vp, vp], i32),
        "sdr_plls_report": ([vp, C.POINTER(C.c_double), i32, C.POINTER(i32), vp], i32),
        "sdr_plls_cycles": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_double), vp], i32),
        "sdr_plls_block_cycles": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_double), i32, C.POINTER(C.c_int), vp], i32),
        "sdr_plls_timeline": ([vp, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong), i32, C.POINTER(i32), vp], i32),
        "sdr_rds_post": ([vp, vp, sz, vp], i32),
        "sdr_ctx_buffer": ([vp, C.c_char_p, C.POINTER(vp), C.POINTER(sz), C.POINTER(i32)], i32),
        "sdr_hbm_copy": ([vp, vp, sz, vp], i32),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != SDR_OK:
        msg = lib().sdr_last_error().decode(errors="replace")
        raise SdrError(f"{what} failed ({rc}): {msg}", rc)


def hbm_copy(dst, src, stream=None) -> None:
    """dst <- src (same byte size, 16-byte aligned device tensors) with the calibration copy kernel
    (sdr_hbm_copy): the HBM rate a plain stream reaches, for the benchmark's roofline context."""
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != nbytes:
        raise SdrError("hbm_copy: size mismatch")
    check(lib().sdr_hbm_copy(_ptr(dst), _ptr(src), nbytes, _stream(stream)), "sdr_hbm_copy")


# ------------------------------------------------------------------ torch plumbing helpers
def _ptr(t) -> int | None:
    if t is None:
        return None
    return int(t.data_ptr())


def _stream(stream=None) -> int | None:
    if stream is not None:
        return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)
    import torch
    return int(torch.cuda.current_stream().cuda_stream) or None


def _row_stride(t) -> int:
    """Elements between consecutive channels of a 2-D [nch][len] tensor (last dim contiguous)."""
    assert t.dim() == 2 and t.stride(1) == 1, "expected a [nch][len] tensor with a contiguous last dim"
    return int(t.stride(0))


# ------------------------------------------------------------------ tap design (host)
def _taps(fn, n, *args):
    import numpy as np
    h = np.zeros(n, np.float32)
    check(fn(*args, h.ctypes.data_as(C.c_void_p)), fn.__name__)
    return h


def impulse_response_lpf(Fs, Fc, num_taps, u=None):
    """impulseResponseLPF, src/filter.cpp:13-29 (u=None) or :33-50 (integer gain u)."""
    if u is None:
        return _taps(lib().sdr_impulse_response_lpf, num_taps, Fs, Fc, num_taps)
    return _taps(lib().sdr_impulse_response_lpf_gain, num_taps, Fs, Fc, num_taps, u)


def impulse_response_bpf(Fs, f0, f1, num_taps):
    """impulseResponseBPF, src/filter.cpp:55-71."""
    import numpy as np
    fb = np.array([f0, f1], np.float32)
    return _taps(lib().sdr_impulse_response_bpf, num_taps, Fs, fb.ctypes.data_as(C.c_void_p), num_taps)


def impulse_response_apf(gain, num_taps):
    """impulseResponseAPF, src/filter.cpp:73-78."""
    return _taps(lib().sdr_impulse_response_apf, num_taps, gain, num_taps)


def impulse_response_rrc(Fs, num_taps):
    """impulseResponseRRC, src/filter.cpp:80-102."""
    return _taps(lib().sdr_impulse_response_rrc, num_taps, Fs, num_taps)


# ------------------------------------------------------------------ batched primitives (torch tensors)
def convolve_fir(y, x, h, state, D: int, stream=None):
    """convolveFIR(y, x, h, state, D) for every row: y[nch][nx/D], x[nch][nx], state[nch][>=ntaps-1]."""
    nch, nx = x.shape
    check(lib().sdr_convolve_fir(_ptr(y), _row_stride(y), _ptr(x), _row_stride(x), nch, nx, _ptr(h), h.numel(),
                                 _ptr(state), state.shape[1], D, _stream(stream)), "convolve_fir")
    return y


def convolve_fir_resample(y, x, h, state, U: int, D: int, stream=None):
    """convolveFIR(y, x, h, state, U, D) for every row: y[nch][nx*U/D]."""
    nch, nx = x.shape
    check(lib().sdr_convolve_fir_resample(_ptr(y), _row_stride(y), _ptr(x), _row_stride(x), nch, nx, _ptr(h),
                                          h.numel(), _ptr(state), state.shape[1], U, D, _stream(stream)),
          "convolve_fir_resample")
    return y


def fm_demod(out, I, Q, prev, stream=None):
    """fmDemodNoArctan for every row; prev[nch][2] = (prev_I, prev_Q), updated in place."""
    nch, n = I.shape
    assert Q.stride(0) == I.stride(0)
    check(lib().sdr_fm_demod(_ptr(out), _row_stride(out), _ptr(I), _ptr(Q), _row_stride(I), nch, n, _ptr(prev),
                             _stream(stream)), "fm_demod")
    return out


def fmpll(out, x, freq, Fs, state, ncoScale=1.0, phaseAdjust=0.0, normBandwidth=0.01, stream=None):
    """fmpll for every row: out[nch][n+1]; state = uint8 tensor holding nch PllState records."""
    nch, n = x.shape
    check(lib().sdr_fmpll(_ptr(out), _row_stride(out), _ptr(x), _row_stride(x), nch, n, freq, Fs, _ptr(state),
                          ncoScale, phaseAdjust, normBandwidth, _stream(stream)), "fmpll")
    return out


def cdr(offset, x, sps: int, stream=None):
    nch, n = x.shape
    check(lib().sdr_cdr(_ptr(offset), _ptr(x), _row_stride(x), nch, n, sps, _stream(stream)), "cdr")
    return offset


def pll_state_tensor(nch: int, device="cuda", feedbackI=1.0, lastCarrier=1.0):
    """Device array of nch PllState records initialised like stereo.cpp:51-57."""
    import numpy as np
    import torch
    arr = (PllState * nch)()
    for i in range(nch):
        arr[i] = PllState(feedbackI, 0.0, 0.0, 0.0, 0.0, lastCarrier)
    raw = np.frombuffer(bytes(arr), dtype=np.uint8).copy()
    return torch.from_numpy(raw).to(device)


def pll_state_from_tensor(t) -> list:
    raw = t.cpu().numpy().tobytes()
    n = len(raw) // C.sizeof(PllState)
    arr = (PllState * n).from_buffer_copy(raw)
    return list(arr)


# ------------------------------------------------------------------ fused pipeline
class Pipeline:
    """A device context of `nch` channels: the reference's RF_frontend + mono + stereo + rds bodies.

    Per block: frontend(iq) then any of mono(), stereo(), rds() (each at most once per block).
    """

    def __init__(self, nch: int, mode: int = 0, rds_on: bool = True, device: int = 0, flags: int = 0):
        import torch
        self.device = device
        self.torch_device = torch.device("cuda", device)
        h = C.c_void_p()
        check(lib().sdr_ctx_create(C.byref(h), device, nch, mode, 1 if rds_on else 0, flags), "sdr_ctx_create")
        self._h = h
        info = Info()
        check(lib().sdr_ctx_info(self._h, C.byref(info)), "sdr_ctx_info")
        self.info = info
        self.nch = nch
        i32 = torch.int32
        dev = self.torch_device
        self.offset = torch.zeros(nch, dtype=i32, device=dev)
        self.nsym = torch.zeros(nch, dtype=i32, device=dev)
        self.nbits = torch.zeros(nch, dtype=i32, device=dev)
        self.symbols = torch.zeros(nch, SDR_MAX_SYMS, dtype=torch.uint8, device=dev)
        self.bits = torch.zeros(nch, SDR_MAX_BITS, dtype=torch.uint8, device=dev)

    def close(self):
        if getattr(self, "_h", None):
            lib().sdr_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, stream=None):
        check(lib().sdr_ctx_reset(self._h, _stream(stream)), "sdr_ctx_reset")

    def frontend(self, iq, stream=None):
        """iq: uint8 [nch][2*block_iq] (device)."""
        check(lib().sdr_frontend(self._h, _ptr(iq), _row_stride(iq), _stream(stream)), "sdr_frontend")

    def release_wait(self, stream=None):
        """The parity-release wait of the next frontend(), enqueued now on `stream` (that call then
        enqueues none there): the front-end kernel can be timed alone."""
        check(lib().sdr_frontend_release_wait(self._h, _stream(stream)), "sdr_frontend_release_wait")

    def frontend_timing(self, max_launches: int):
        """Record the dispatch start / end of the next max_launches frontend() kernels."""
        check(lib().sdr_frontend_timing(self._h, max_launches), "sdr_frontend_timing")

    def frontend_times(self, max_launches: int = 4096) -> list:
        """ms per timed frontend() kernel, in call order (synchronises with the last)."""
        arr = (C.c_double * max_launches)()
        n = C.c_int(0)
        check(lib().sdr_frontend_times(self._h, arr, max_launches, C.byref(n)), "sdr_frontend_times")
        return list(arr[:n.value])

    def frontend_stamps(self, max_launches: int = 4096) -> tuple[list, list]:
        """(start, end) of each timed frontend() kernel in 100 MHz device ticks (plls_timeline's clock)."""
        a, z = (C.c_ulonglong * max_launches)(), (C.c_ulonglong * max_launches)()
        n = C.c_int(0)
        check(lib().sdr_frontend_stamps(self._h, a, z, max_launches, C.byref(n)), "sdr_frontend_stamps")
        return list(a[:n.value]), list(z[:n.value])

    def fm_demod(self, out=None, stream=None):
        import torch
        if out is None:
            out = torch.empty(self.nch, self.info.block_if, dtype=torch.float32, device=self.torch_device)
        check(lib().sdr_get_fm_demod(self._h, _ptr(out), _row_stride(out), _stream(stream)), "sdr_get_fm_demod")
        return out

    def mono(self, out=None, stream=None):
        import torch
        if out is None:
            out = torch.empty(self.nch, self.info.n_audio, dtype=torch.int16, device=self.torch_device)
        check(lib().sdr_mono(self._h, _ptr(out), _row_stride(out), _stream(stream)), "sdr_mono")
        return out

    def stereo(self, out=None, stream=None):
        import torch
        if out is None:
            out = torch.empty(self.nch, 2 * self.info.n_audio, dtype=torch.int16, device=self.torch_device)
        check(lib().sdr_stereo(self._h, _ptr(out), _row_stride(out), _stream(stream)), "sdr_stereo")
        return out

    # the stereo / RDS bodies split at their PLL (include/sdr_amd.h): pre; pll; post per block
    def stereo_pre(self, stream=None):
        check(lib().sdr_stereo_pre(self._h, _stream(stream)), "sdr_stereo_pre")

    def stereo_pll(self, stream=None):
        check(lib().sdr_stereo_pll(self._h, _stream(stream)), "sdr_stereo_pll")

    def stereo_post(self, out, stream=None):
        check(lib().sdr_stereo_post(self._h, _ptr(out), _row_stride(out), _stream(stream)), "sdr_stereo_post")
        return out

    def rds_pre(self, stream=None):
        check(lib().sdr_rds_pre(self._h, _stream(stream)), "sdr_rds_pre")

    def pre(self, stream=None):
        """stereo_pre + rds_pre on one stream, the three fm_demod BPFs sharing one staged window."""
        check(lib().sdr_pre(self._h, _stream(stream)), "sdr_pre")

    def rds_pll(self, stream=None):
        check(lib().sdr_rds_pll(self._h, _stream(stream)), "sdr_rds_pll")

    def plls(self, stream=None):
        """stereo_pll + rds_pll in one dispatch."""
        check(lib().sdr_plls(self._h, _stream(stream)), "sdr_plls")

    # persistent PLLs (include/sdr_amd.h): one dispatch for many blocks
    def plls_launch(self, nblocks: int, stream=None, which: int = 3):
        """Persistent PLLs of the next nblocks blocks (which = 3: both; 1: stereo, 2: RDS only)."""
        check(lib().sdr_plls_launch_sel(self._h, nblocks, which, _stream(stream)), "sdr_plls_launch_sel")

    def plls_fits(self, n_cu: int, first_cu: int = 0, which: int = 3) -> dict:
        """Would plls_launch (which = 3: both PLLs; 1 stereo, 2 RDS: plls_launch_sel) accept a stream
        over CUs [first_cu, first_cu + n_cu)? The launch's waves, workgroups and how many of those the
        range keeps resident at once (sdr_plls_fits)."""
        w, g, r = C.c_int(), C.c_longlong(), C.c_longlong()
        check(lib().sdr_plls_fits(self._h, which, first_cu, n_cu, C.byref(w), C.byref(g), C.byref(r)),
              "sdr_plls_fits")
        return {"waves": w.value, "groups": g.value, "resident": r.value, "fits": g.value <= r.value}

    def plls_prepare(self, nblocks: int, stream=None):
        """The launch's bookkeeping ahead of plls_launch(nblocks) (allocation, stamp reset)."""
        check(lib().sdr_plls_prepare(self._h, nblocks, _stream(stream)), "sdr_plls_prepare")

    def plls_signal(self, stream=None):
        check(lib().sdr_plls_signal(self._h, _stream(stream)), "sdr_plls_signal")

    def frontend_pre_parts(self, iq, nparts: int, stream=None):
        """The first block of a pending persistent launch: frontend + pre + plls_signal in nparts
        sample ranges, each published to the PLLs as soon as it is ready (the pipeline fill)."""
        check(lib().sdr_frontend_pre_parts(self._h, _ptr(iq), _row_stride(iq), nparts, _stream(stream)),
              "sdr_frontend_pre_parts")

    def plls_wait(self, stream=None):
        check(lib().sdr_plls_wait(self._h, _stream(stream)), "sdr_plls_wait")

    def plls_report(self, max_blocks: int = 4096, stream=None) -> list:
        """Per-block PLL time (ms) of the last persistent launch; raises if a wait timed out."""
        arr = (C.c_double * max_blocks)()
        n = C.c_int(0)
        check(lib().sdr_plls_report(self._h, arr, max_blocks, C.byref(n), _stream(stream)), "sdr_plls_report")
        return list(arr[:n.value])

    def plls_timeline(self, max_blocks: int = 4096, stream=None) -> tuple[list, list]:
        """(t_start, t_end) per block of the last persistent launch, 100 MHz device ticks."""
        a, z = (C.c_ulonglong * max_blocks)(), (C.c_ulonglong * max_blocks)()
        n = C.c_int(0)
        check(lib().sdr_plls_timeline(self._h, a, z, max_blocks, C.byref(n), _stream(stream)), "sdr_plls_timeline")
        return list(a[:n.value]), list(z[:n.value])

    def plls_cycles(self, stream=None) -> tuple[float, float]:
        """(shader cycles per PLL step and wave, shader clock MHz) of the last persistent launch."""
        cyc, mhz = C.c_double(0.0), C.c_double(0.0)
        check(lib().sdr_plls_cycles(self._h, C.byref(cyc), C.byref(mhz), _stream(stream)), "sdr_plls_cycles")
        return cyc.value, mhz.value

    def plls_block_cycles(self, stream=None, max_blocks: int = 4096) -> tuple[list, list]:
        """Per block of the last persistent launch: (cycles per step and wave, shader clock MHz)."""
        cyc, mhz = (C.c_double * max_blocks)(), (C.c_double * max_blocks)()
        n = C.c_int(0)
        check(lib().sdr_plls_block_cycles(self._h, cyc, mhz, max_blocks, C.byref(n), _stream(stream)),
              "sdr_plls_block_cycles")
        k = min(n.value, max_blocks)
        return list(cyc[:k]), list(mhz[:k])

    def rds_post(self, out=None, bits=True, stream=None, bits_out=None):
        """bits_out: a [nch][SDR_MAX_BITS] u8 tensor the block's bits go to instead of self.bits."""
        check(lib().sdr_rds_post(self._h, _ptr(out), _row_stride(out) if out is not None else 0, _stream(stream)),
              "sdr_rds_post")
        if bits:
            self.rds_bits(stream, bits_out)
        return out

    def rds_bits(self, stream=None, bits_out=None):
        b = self.bits if bits_out is None else bits_out
        if tuple(b.shape) != (self.nch, SDR_MAX_BITS) or b.dtype != self.bits.dtype or not b.is_contiguous():
            raise ValueError(f"bits_out must be a contiguous [{self.nch}][{SDR_MAX_BITS}] uint8 tensor")
        check(lib().sdr_rds_bits(self._h, _ptr(self.offset), _ptr(self.nsym), _ptr(self.symbols), SDR_MAX_SYMS,
                                 _ptr(self.nbits), _ptr(b), SDR_MAX_BITS, _stream(stream)), "sdr_rds_bits")

    def push_fm_demod(self, fm, stream=None):
        """Make fm [nch][block_if] (device f32) the current block (the queue's consumer side)."""
        check(lib().sdr_push_fm_demod(self._h, _ptr(fm), _row_stride(fm), _stream(stream)), "sdr_push_fm_demod")

    def rds(self, out=None, bits=True, stream=None):
        """RDS DSP (+ symbol/bit recovery). Returns rds_clean [nch][n_rds]; bits in self.bits/nbits."""
        import torch
        if out is None:
            out = torch.empty(self.nch, self.info.n_rds, dtype=torch.float32, device=self.torch_device)
        check(lib().sdr_rds_dsp(self._h, _ptr(out), _row_stride(out), _stream(stream)), "sdr_rds_dsp")
        if bits:
            check(lib().sdr_rds_bits(self._h, _ptr(self.offset), _ptr(self.nsym), _ptr(self.symbols),
                                     SDR_MAX_SYMS, _ptr(self.nbits), _ptr(self.bits), SDR_MAX_BITS,
                                     _stream(stream)), "sdr_rds_bits")
        return out

    def buffer(self, name: str, stream=None):
        """Current-block intermediate copied into a new [nch][len] tensor (on `stream`, which is then
        synchronised; the default is the legacy null stream, which waits for every blocking stream
        -- never use it while a persistent PLL launch still waits for blocks)."""
        import torch
        p, s, n = C.c_void_p(), C.c_size_t(), C.c_int()
        check(lib().sdr_ctx_buffer(self._h, name.encode(), C.byref(p), C.byref(s), C.byref(n)), "sdr_ctx_buffer")
        full = torch.empty(0, dtype=torch.float32, device=self.torch_device)
        # wrap the device pointer through a DLPack-free path: copy rows with cudaMemcpy2D via torch
        out = torch.empty(self.nch, n.value, dtype=torch.float32, device=self.torch_device)
        import ctypes
        hip = _hip()
        st = _stream(stream) if stream is not None else None
        if st is None:
            rc = hip.hipMemcpy2D(ctypes.c_void_p(out.data_ptr()), ctypes.c_size_t(4 * n.value), p,
                                 ctypes.c_size_t(4 * s.value), ctypes.c_size_t(4 * n.value),
                                 ctypes.c_size_t(self.nch), ctypes.c_int(3))
        else:
            rc = hip.hipMemcpy2DAsync(ctypes.c_void_p(out.data_ptr()), ctypes.c_size_t(4 * n.value), p,
                                      ctypes.c_size_t(4 * s.value), ctypes.c_size_t(4 * n.value),
                                      ctypes.c_size_t(self.nch), ctypes.c_int(3), ctypes.c_void_p(st))
            if rc == 0:
                rc = hip.hipStreamSynchronize(ctypes.c_void_p(st))
        if rc != 0:
            raise SdrError(f"hipMemcpy2D failed ({rc})")
        del full
        return out


_hiplib = None


def _hip():
    global _hiplib
    if _hiplib is None:
        import ctypes.util
        for cand in ("libamdhip64.so", "libamdhip64.so.7", "/opt/rocm/lib/libamdhip64.so"):
            try:
                _hiplib = C.CDLL(cand)
                break
            except OSError:
                continue
        if _hiplib is None:
            raise SdrError("libamdhip64.so not found")
        _hiplib.hipMemcpy2D.restype = C.c_int
        _hiplib.hipMemcpy2DAsync.restype = C.c_int
        _hiplib.hipStreamSynchronize.restype = C.c_int
    return _hiplib
