"""ctypes wrapper over oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (oracle/sdr_oracle.c). Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the parity checker / CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
_LIB = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(dtype=np.int16, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


class PllState(C.Structure):
    """pllblock_args (include/pll.h:10-17)."""
    _fields_ = [("feedbackI", C.c_float), ("feedbackQ", C.c_float), ("integrator", C.c_float),
                ("phaseEst", C.c_float), ("trigOffset", C.c_double), ("lastCarrier", C.c_float)]


class _Chan(C.Structure):
    # layout of orc_chan (oracle/sdr_oracle.h); only scalar fields are read from Python
    _fields_ = ([(n, C.c_int) for n in ("rf_Fs", "rf_Fc", "rf_taps", "rf_decim", "audio_decim",
                                         "audio_upsample", "if_Fs", "audio_Fc", "symbol_Fs", "rds_on",
                                         "block_iq", "block_if", "n_audio", "n_rds")]
                + [(n, C.c_void_p) for n in ("rf_h", "audio_h", "pilot_h", "stereo_h", "apf_h", "rds_h",
                                             "rds_sq_h", "rds_bb_h", "rrc_h")]
                + [("audio_ntaps", C.c_int), ("rds_bb_ntaps", C.c_int)]
                + [("state_I", C.c_void_p), ("state_Q", C.c_void_p), ("prev_I", C.c_float), ("prev_Q", C.c_float)]
                + [("mono_state", C.c_void_p)]
                + [(n, C.c_void_p) for n in ("pilot_state", "band_state", "mdelay_state", "mfilt_state",
                                             "sfilt_state", "carrier")]
                + [("st_pll", PllState)]
                + [(n, C.c_void_p) for n in ("rband_state", "rsq_state", "rdelay_state", "rfilt_state",
                                             "rclean_state", "ipll")]
                + [("rds_pll", PllState)]
                + [(n, C.c_int) for n in ("rds_block_count", "half_symbol", "start", "last_bit", "sample_offset")]
                + [(n, C.c_void_p) for n in ("I", "Q", "Ids", "Qds", "t0", "t1", "t2", "t3", "t4", "t5")])


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = HERE / "liboracle.so"
        if not path.exists():
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(str(path))
        L.orc_lpf.argtypes = [C.c_float, C.c_float, C.c_ushort, _f32p]
        L.orc_lpf_gain.argtypes = [C.c_float, C.c_float, C.c_ushort, C.c_int, _f32p]
        L.orc_bpf.argtypes = [C.c_float, _f32p, C.c_ushort, _f32p]
        L.orc_apf.argtypes = [C.c_float, C.c_ushort, _f32p]
        L.orc_rrc.argtypes = [C.c_float, C.c_ushort, _f32p]
        L.orc_fir_decim.argtypes = [_f32p, _f32p, C.c_int, _f32p, C.c_int, _f32p, C.c_int, C.c_int]
        L.orc_fir_resample.argtypes = [_f32p, _f32p, C.c_int, _f32p, C.c_int, _f32p, C.c_int, C.c_int, C.c_int]
        L.orc_fm_demod.argtypes = [_f32p, _f32p, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), _f32p]
        L.orc_fmpll.argtypes = [_f32p, C.c_int, C.c_float, C.c_float, _f32p, C.POINTER(PllState),
                                C.c_float, C.c_float, C.c_float]
        L.orc_cdr.argtypes = [C.c_int, _f32p, C.c_int]
        L.orc_cdr.restype = C.c_int
        L.orc_slice.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, _i32p]
        L.orc_slice.restype = C.c_int
        L.orc_manchester.argtypes = [_i32p, _i32p, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_manchester.restype = C.c_int
        L.orc_differential.argtypes = [_i32p, _i32p, C.c_int, C.POINTER(C.c_int), C.c_int]
        L.orc_f32_to_i16.argtypes = [C.c_float]
        L.orc_f32_to_i16.restype = C.c_int16
        L.orc_chan_init.argtypes = [C.POINTER(_Chan), C.c_int, C.c_int]
        L.orc_chan_init.restype = C.c_int
        L.orc_chan_free.argtypes = [C.POINTER(_Chan)]
        L.orc_frontend_block.argtypes = [C.POINTER(_Chan), _u8p, _f32p]
        L.orc_mono_block.argtypes = [C.POINTER(_Chan), _f32p, _i16p]
        optf = C.c_void_p
        L.orc_stereo_block.argtypes = [C.POINTER(_Chan), _f32p, _i16p, optf, optf, optf, optf, optf]
        L.orc_rds_block.argtypes = [C.POINTER(_Chan), _f32p, _f32p, C.POINTER(C.c_int), _i32p,
                                    C.POINTER(C.c_int), _i32p, optf, optf, optf, optf, optf]
        L.orc_rds_block.restype = C.c_int
        _LIB = L
    return _LIB


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ---------------------------------------------------------------- taps
def lpf(Fs, Fc, ntaps, u=None):
    h = np.zeros(ntaps, np.float32)
    if u is None:
        lib().orc_lpf(Fs, Fc, ntaps, h)
    else:
        lib().orc_lpf_gain(Fs, Fc, ntaps, u, h)
    return h


def bpf(Fs, f0, f1, ntaps):
    h = np.zeros(ntaps, np.float32)
    lib().orc_bpf(Fs, np.array([f0, f1], np.float32), ntaps, h)
    return h


def apf(gain, ntaps):
    h = np.zeros(ntaps, np.float32)
    lib().orc_apf(gain, ntaps, h)
    return h


def rrc(Fs, ntaps):
    h = np.zeros(ntaps, np.float32)
    lib().orc_rrc(Fs, ntaps, h)
    return h


# ---------------------------------------------------------------- primitives
def fir_decim(x, h, state, D):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros(len(x) // D, np.float32)
    lib().orc_fir_decim(y, x, len(x), np.ascontiguousarray(h, np.float32), len(h), state, len(state), D)
    return y


def fir_resample(x, h, state, U, D):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros(len(x) * U // D, np.float32)
    lib().orc_fir_resample(y, x, len(x), np.ascontiguousarray(h, np.float32), len(h), state, len(state), U, D)
    return y


def fm_demod(I, Q, prev):
    """prev: length-2 float32 array [prev_I, prev_Q], updated in place."""
    I = np.ascontiguousarray(I, np.float32)
    Q = np.ascontiguousarray(Q, np.float32)
    out = np.zeros(len(I), np.float32)
    pi, pq = C.c_float(prev[0]), C.c_float(prev[1])
    lib().orc_fm_demod(I, Q, len(I), C.byref(pi), C.byref(pq), out)
    prev[0], prev[1] = pi.value, pq.value
    return out


def new_pll_state(feedbackI=1.0, lastCarrier=1.0):
    return PllState(feedbackI, 0.0, 0.0, 0.0, 0.0, lastCarrier)


def fmpll(x, freq, Fs, out, st, ncoScale=1.0, phaseAdjust=0.0, bw=0.01):
    """out: persistent float32 array of len(x)+1 (out[0] <- out[-1] on entry, pll.cpp:18)."""
    x = np.ascontiguousarray(x, np.float32)
    lib().orc_fmpll(x, len(x), freq, Fs, out, C.byref(st), ncoScale, phaseAdjust, bw)
    return out


def cdr(sps, x):
    x = np.ascontiguousarray(x, np.float32)
    return lib().orc_cdr(sps, x, len(x))


# ---------------------------------------------------------------- per-channel pipeline
class Channel:
    """One channel of the reference pipeline (RF_frontend + mono + stereo + rds), block by block."""

    def __init__(self, mode: int = 0, rds_on: bool = True):
        self._c = _Chan()
        if lib().orc_chan_init(C.byref(self._c), mode, 1 if rds_on else 0) != 0:
            raise ValueError(f"bad mode {mode}")
        c = self._c
        self.block_iq, self.block_if, self.n_audio, self.n_rds = c.block_iq, c.block_if, c.n_audio, c.n_rds
        self.symbol_Fs = c.symbol_Fs

    def __del__(self):
        try:
            lib().orc_chan_free(C.byref(self._c))
        except Exception:
            pass

    @property
    def state(self):
        return self._c

    def frontend(self, iq: np.ndarray) -> np.ndarray:
        out = np.zeros(self.block_if, np.float32)
        lib().orc_frontend_block(C.byref(self._c), np.ascontiguousarray(iq, np.uint8), out)
        return out

    def mono(self, fm: np.ndarray) -> np.ndarray:
        out = np.zeros(self.n_audio, np.int16)
        lib().orc_mono_block(C.byref(self._c), fm, out)
        return out

    def stereo(self, fm: np.ndarray, intermediates: bool = False):
        lr = np.zeros(2 * self.n_audio, np.int16)
        n = self.block_if
        if intermediates:
            d = {k: np.zeros(n + (1 if k == "carrier" else 0), np.float32)
                 for k in ("pilot", "carrier", "band", "stereo_dc", "mono_delay")}
            lib().orc_stereo_block(C.byref(self._c), fm, lr, _ptr(d["pilot"]), _ptr(d["carrier"]),
                                   _ptr(d["band"]), _ptr(d["stereo_dc"]), _ptr(d["mono_delay"]))
            return lr, d
        lib().orc_stereo_block(C.byref(self._c), fm, lr, None, None, None, None, None)
        return lr

    def rds(self, fm: np.ndarray, intermediates: bool = False):
        """Returns dict(rds_clean, offset, symbols or None, bits or None[, intermediates])."""
        n = self.block_if
        clean = np.zeros(self.n_rds, np.float32)
        off = C.c_int(0)
        nsym = C.c_int(0)
        sym = np.zeros(512, np.int32)
        bits = np.zeros(512, np.int32)
        d = None
        if intermediates:
            d = {"rds_band": np.zeros(n, np.float32), "gen_pilot": np.zeros(n, np.float32),
                 "ipll": np.zeros(n + 1, np.float32), "rds_dc": np.zeros(n, np.float32),
                 "rds_filt": np.zeros(self.n_rds, np.float32)}
            ptrs = [_ptr(d[k]) for k in ("rds_band", "gen_pilot", "ipll", "rds_dc", "rds_filt")]
        else:
            ptrs = [None] * 5
        nb = lib().orc_rds_block(C.byref(self._c), fm, clean, C.byref(off), sym, C.byref(nsym), bits, *ptrs)
        res = {"rds_clean": clean, "offset": off.value,
               "symbols": sym[:nsym.value].copy() if nb >= 0 else None,
               "bits": bits[:nb].copy() if nb >= 0 else None}
        if d is not None:
            res.update(d)
        return res


def run_channel(iq_blocks: np.ndarray, mode: int = 0, rds_on: bool = True, intermediates_at=()):
    """Run the full per-channel pipeline over iq_blocks[nblocks][2*block_iq]; returns dict of lists."""
    ch = Channel(mode, rds_on)
    out = {"fm_demod": [], "mono": [], "stereo": [], "rds_clean": [], "offset": [], "symbols": [], "bits": [],
           "intermediates": {}}
    for b, iq in enumerate(iq_blocks):
        fm = ch.frontend(iq)
        out["fm_demod"].append(fm)
        out["mono"].append(ch.mono(fm))
        want = b in intermediates_at
        st = ch.stereo(fm, intermediates=want)
        r = ch.rds(fm, intermediates=want)
        if want:
            lr, d = st
            d.update({k: r[k] for k in ("rds_band", "gen_pilot", "ipll", "rds_dc", "rds_filt")})
            out["intermediates"][b] = d
        else:
            lr = st
        out["stereo"].append(lr)
        out["rds_clean"].append(r["rds_clean"])
        out["offset"].append(r["offset"])
        out["symbols"].append(r["symbols"])
        out["bits"].append(r["bits"])
    return out


if __name__ == "__main__":  # pragma: no cover
    print(os.fspath(HERE / "liboracle.so"), lib())
