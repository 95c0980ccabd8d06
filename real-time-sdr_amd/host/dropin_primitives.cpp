// dropin_primitives.cpp -- the reference's per-vector DSP functions (include/dropin/{filter,demod,
// pll,rds_utilities}.h) executed by the MI355X kernels of libsdr_amd.so through its C ABI.
//
// Each call stages its single-channel std::vector arguments in device memory on the calling
// thread's stream, runs the batched kernel with nch = 1 and copies outputs and state back, so a
// caller written against the reference (src/filter.cpp, demod.cpp, pll.cpp, rds_utilities.cpp)
// links unchanged and gets bit-identical results. The batched, device-resident path for many
// channels is the sdr_ctx pipeline (include/sdr_amd.h); these wrappers are the compatibility layer.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <vector>

#include "demod.h"
#include "filter.h"
#include "hip_util.h"
#include "pll.h"
#include "rds_utilities.h"

using sdrhost::check_hip;
using sdrhost::check_sdr;
using sdrhost::DevBuf;
using sdrhost::thread_stream;

static_assert(sizeof(pllblock_args) == sizeof(sdr_pll_state), "pllblock_args must match sdr_pll_state");
static_assert(offsetof(pllblock_args, trigOffset) == offsetof(sdr_pll_state, trigOffset), "layout");
static_assert(offsetof(pllblock_args, lastCarrier) == offsetof(sdr_pll_state, lastCarrier), "layout");

namespace {

struct Workspace {
    DevBuf<float> a, b, c, d, e;
    DevBuf<uint8_t> u0, u1;
    DevBuf<int32_t> i0, i1, i2;
    DevBuf<sdr_pll_state> pll;
};

Workspace& ws() {
    thread_local Workspace w;
    return w;
}

template <typename T>
void h2d(T* dst, const T* src, size_t n, hipStream_t s) {
    if (n) check_hip(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D");
}
template <typename T>
void d2h(T* dst, const T* src, size_t n, hipStream_t s) {
    if (n) check_hip(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
}
void sync(hipStream_t s) { check_hip(hipStreamSynchronize(s), "hipStreamSynchronize"); }

void taps(std::vector<float>& h, unsigned short n) {
    h.clear();
    h.resize(n, 0.0f);
}

}  // namespace

// ------------------------------------------------------------------ tap design (host, filter.cpp:13-102)
void impulseResponseLPF(float Fs, float Fc, unsigned short num_taps, std::vector<float>& h) {
    taps(h, num_taps);
    check_sdr(sdr_impulse_response_lpf(Fs, Fc, num_taps, h.data()), "impulseResponseLPF");
}

void impulseResponseLPF(float Fs, float Fc, unsigned short num_taps, std::vector<float>& h, int u) {
    taps(h, num_taps);
    check_sdr(sdr_impulse_response_lpf_gain(Fs, Fc, num_taps, u, h.data()), "impulseResponseLPF");
}

void impulseResponseBPF(float Fs, float* Fb, unsigned short num_taps, std::vector<float>& h) {
    taps(h, num_taps);
    check_sdr(sdr_impulse_response_bpf(Fs, Fb, num_taps, h.data()), "impulseResponseBPF");
}

void impulseResponseAPF(float gain, unsigned short num_taps, std::vector<float>& h) {
    taps(h, num_taps);
    check_sdr(sdr_impulse_response_apf(gain, num_taps, h.data()), "impulseResponseAPF");
}

void impulseResponseRRC(float Fs, unsigned short num_taps, std::vector<float>& h) {
    taps(h, num_taps);
    check_sdr(sdr_impulse_response_rrc(Fs, num_taps, h.data()), "impulseResponseRRC");
}

// ------------------------------------------------------------------ convolveFIR (filter.cpp:106-147)
void convolveFIR(std::vector<float>& y, const std::vector<float>& x, const std::vector<float>& h,
                 std::vector<float>& state, int D) {
    y.clear();
    y.resize(D > 0 ? x.size() / D : 0, 0.0f);
    if (x.empty() || h.empty()) return;
    if (state.size() + 1 < h.size()) sdrhost::die("convolveFIR: state shorter than h.size()-1");
    hipStream_t s = thread_stream();
    Workspace& w = ws();
    float* dx = w.a.get(x.size());
    float* dh = w.b.get(h.size());
    float* ds = w.c.get(state.size());
    float* dy = w.d.get(std::max<size_t>(y.size(), 1));
    h2d(dx, x.data(), x.size(), s);
    h2d(dh, h.data(), h.size(), s);
    h2d(ds, state.data(), state.size(), s);
    check_sdr(sdr_convolve_fir(dy, y.size(), dx, x.size(), 1, (int)x.size(), dh, (int)h.size(), ds,
                               (int)state.size(), D, s), "convolveFIR");
    d2h(y.data(), dy, y.size(), s);
    d2h(state.data(), ds, state.size(), s);
    sync(s);
}

void convolveFIR(std::vector<float>& y, const std::vector<float>& x, const std::vector<float>& h,
                 std::vector<float>& state, int U, int D) {
    y.clear();
    y.resize((U > 0 && D > 0) ? x.size() * U / D : 0, 0.0f);
    if (x.empty() || h.empty()) return;
    hipStream_t s = thread_stream();
    Workspace& w = ws();
    float* dx = w.a.get(x.size());
    float* dh = w.b.get(h.size());
    float* ds = w.c.get(state.size());
    float* dy = w.d.get(std::max<size_t>(y.size(), 1));
    h2d(dx, x.data(), x.size(), s);
    h2d(dh, h.data(), h.size(), s);
    h2d(ds, state.data(), state.size(), s);
    check_sdr(sdr_convolve_fir_resample(dy, y.size(), dx, x.size(), 1, (int)x.size(), dh, (int)h.size(), ds,
                                        (int)state.size(), U, D, s), "convolveFIR (resample)");
    d2h(y.data(), dy, y.size(), s);
    d2h(state.data(), ds, state.size(), s);
    sync(s);
}

// ------------------------------------------------------------------ fmDemodNoArctan (demod.cpp:3-24)
void fmDemodNoArctan(const std::vector<float>& I, const std::vector<float>& Q, float& prev_I, float& prev_Q,
                     std::vector<float>& fm_demod) {
    fm_demod.clear();
    fm_demod.resize(I.size(), 0.0f);
    if (I.empty()) return;
    if (Q.size() < I.size()) sdrhost::die("fmDemodNoArctan: Q shorter than I");
    hipStream_t s = thread_stream();
    Workspace& w = ws();
    const size_t n = I.size();
    float* dI = w.a.get(n);
    float* dQ = w.b.get(n);
    float* dp = w.c.get(2);
    float* dout = w.d.get(n);
    const float prev[2] = {prev_I, prev_Q};
    h2d(dI, I.data(), n, s);
    h2d(dQ, Q.data(), n, s);
    h2d(dp, prev, 2, s);
    // I and Q are separate allocations: pass them as rows of one [2][...] view is not possible,
    // so the row stride is irrelevant for nch = 1
    check_sdr(sdr_fm_demod(dout, n, dI, dQ, n, 1, (int)n, dp, s), "fmDemodNoArctan");
    float pv[2];
    d2h(fm_demod.data(), dout, n, s);
    d2h(pv, dp, 2, s);
    sync(s);
    prev_I = pv[0];
    prev_Q = pv[1];
}

// ------------------------------------------------------------------ fmpll (pll.cpp:4-61)
void fmpll(const std::vector<float>& pllIn, float freq, float Fs, std::vector<float>& pllOut, pllblock_args& block,
           float ncoScale, float phaseAdjust, float normBandwidth) {
    const size_t n = pllIn.size();
    if (pllOut.size() != n + 1) sdrhost::die("fmpll: pllOut must hold pllIn.size()+1 samples (pll.cpp:18)");
    hipStream_t s = thread_stream();
    Workspace& w = ws();
    sdr_pll_state st;
    std::memcpy(&st, &block, sizeof(st));
    st.lastCarrier = pllOut[n];   // pllOut[0] <- pllOut[last] (pll.cpp:18)
    float* din = w.a.get(std::max<size_t>(n, 1));
    float* dout = w.b.get(n + 1);
    sdr_pll_state* dst = w.pll.get(1);
    h2d(din, pllIn.data(), n, s);
    h2d(dst, &st, 1, s);
    check_sdr(sdr_fmpll(dout, n + 1, din, std::max<size_t>(n, 1), 1, (int)n, freq, Fs, dst, ncoScale, phaseAdjust,
                        normBandwidth, s), "fmpll");
    d2h(pllOut.data(), dout, n + 1, s);
    d2h(&st, dst, 1, s);
    sync(s);
    std::memcpy(&block, &st, sizeof(st));
}

// ------------------------------------------------------------------ RDS symbol/bit recovery
int cdr(int sps, const std::vector<float>& signal) {
    if (signal.empty() || sps <= 0) return 0;
    hipStream_t s = thread_stream();
    Workspace& w = ws();
    float* dx = w.a.get(signal.size());
    int32_t* doff = w.i0.get(1);
    h2d(dx, signal.data(), signal.size(), s);
    check_sdr(sdr_cdr(doff, dx, signal.size(), 1, (int)signal.size(), sps, s), "cdr");
    int32_t off = 0;
    d2h(&off, doff, 1, s);
    sync(s);
    return off;
}

void manchester_decode(std::vector<int>& bits, const std::vector<int>& symbols, int& block_count, int& half_symbol,
                       int& start) {
    hipStream_t s = thread_stream();
    Workspace& w = ws();
    const size_t m = symbols.size();
    std::vector<uint8_t> sym8(m);
    for (size_t i = 0; i < m; i++) sym8[i] = (uint8_t)symbols[i];
    uint8_t* dsym = w.u0.get(std::max<size_t>(m, 1));
    uint8_t* dbits = w.u1.get(m / 2 + 2);
    int32_t* dn = w.i0.get(1);
    int32_t* dnsym = w.i1.get(1);
    int32_t* dstate = w.i2.get(2);
    const int32_t nsym = (int32_t)m, state[2] = {half_symbol, start};
    h2d(dsym, sym8.data(), m, s);
    h2d(dnsym, &nsym, 1, s);
    h2d(dstate, state, 2, s);
    check_sdr(sdr_manchester_decode(dbits, m / 2 + 2, dn, dsym, std::max<size_t>(m, 1), dnsym, 1, block_count, dstate,
                                    s), "manchester_decode");
    int32_t nb = 0, st2[2];
    d2h(&nb, dn, 1, s);
    d2h(st2, dstate, 2, s);
    sync(s);
    std::vector<uint8_t> b8(nb);
    d2h(b8.data(), dbits, nb, s);
    sync(s);
    bits.assign(b8.begin(), b8.end());
    half_symbol = st2[0];
    start = st2[1];
}

void differential_decode(std::vector<int>& decoded_bits, const std::vector<int>& bits, int& last_bit, int& block_num) {
    decoded_bits.clear();
    decoded_bits.resize(bits.size(), 0);
    if (bits.empty()) return;
    hipStream_t s = thread_stream();
    Workspace& w = ws();
    const size_t n = bits.size();
    std::vector<uint8_t> b8(n);
    for (size_t i = 0; i < n; i++) b8[i] = (uint8_t)bits[i];
    uint8_t* din = w.u0.get(n);
    uint8_t* dout = w.u1.get(n);
    int32_t* dn = w.i0.get(1);
    int32_t* dlast = w.i1.get(1);
    const int32_t nb = (int32_t)n, lb = last_bit;
    h2d(din, b8.data(), n, s);
    h2d(dn, &nb, 1, s);
    h2d(dlast, &lb, 1, s);
    check_sdr(sdr_differential_decode(dout, n, din, n, dn, 1, block_num, dlast, s), "differential_decode");
    int32_t lb2 = 0;
    d2h(b8.data(), dout, n, s);
    d2h(&lb2, dlast, 1, s);
    sync(s);
    for (size_t i = 0; i < n; i++) decoded_bits[i] = b8[i];
    last_bit = lb2;
}
