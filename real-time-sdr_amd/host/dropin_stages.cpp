// dropin_stages.cpp -- the reference's stage threads (include/dropin/{rffrontend,mono,stereo,rds}.h)
// with their per-block DSP on the MI355X kernels, behind the unchanged ThreadSafeQueue protocol.
//
//   RF_frontend  rffrontend.cpp:45-76  stdin u8 I/Q -> sdr_frontend -> fm_demod vector -> push
//   mono         mono.cpp:29-49        pop(0) -> sdr_mono -> int16 -> stdout
//   stereo       stereo.cpp:69-114     pop(0) -> sdr_stereo -> interleaved L/R int16 -> stdout
//   rds          rds.cpp:95-192        pop(1) -> sdr_rds_dsp + sdr_rds_bits -> frame sync (host)
//
// Each thread owns a one-channel sdr_ctx on its own HIP stream. The queue payload stays the
// reference's heap std::vector<float>* fm_demod block (deleted by the next push), so the
// reference's project.cpp links against these entry points unchanged; a consumer copies the block
// to the device and releases it (prepare) before computing.
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <iostream>
#include <string>
#include <vector>

#include "args.h"
#include "hip_util.h"
#include "mono.h"
#include "rds.h"
#include "rds_utilities.h"
#include "rffrontend.h"
#include "stereo.h"

using sdrhost::check_hip;
using sdrhost::check_sdr;
using sdrhost::die;

namespace {

// project.cpp:67-108 mode table -> mode index
int mode_of(const args* p) {
    const int U = (int)p->audio_upsample, D = (int)p->audio_decim;
    struct M { int rf_Fs, rf_decim, audio_decim, U, if_Fs; } modes[4] = {
        {2400000, 10, 5, 1, 240000}, {1440000, 4, 9, 1, 360000}, {2400000, 10, 800, 147, 240000},
        {1152000, 3, 1280, 147, 384000}};
    for (int m = 0; m < 4; m++)
        if (modes[m].rf_Fs == p->rf_Fs && modes[m].rf_decim == p->rf_decim && modes[m].audio_decim == D &&
            modes[m].U == U && modes[m].if_Fs == p->if_Fs && p->rf_taps == 101)
            return m;
    die("arguments do not match a mode of project.cpp:67-108");
}

int env_flags() {
    int f = 0;
    const char* e = std::getenv("SDR_FAST_FRONTEND");
    if (e && std::strcmp(e, "1") == 0) f |= SDR_FLAG_FAST_FRONTEND;
    return f;
}

struct Stage {
    sdr_ctx* ctx = nullptr;
    sdr_info info{};
    hipStream_t s = nullptr;
    float* d_fm = nullptr;
    Stage(const args* p, int rds_on) {
        check_hip(hipSetDevice(p->device), "hipSetDevice");
        check_sdr(sdr_ctx_create(&ctx, p->device, 1, mode_of(p), rds_on, env_flags()), "sdr_ctx_create");
        check_sdr(sdr_ctx_info(ctx, &info), "sdr_ctx_info");
        s = sdrhost::thread_stream();
        check_hip(hipMalloc(reinterpret_cast<void**>(&d_fm), info.block_if * sizeof(float)), "hipMalloc");
    }
    ~Stage() {
        (void)hipFree(d_fm);
        sdr_ctx_destroy(ctx);
    }
    // wait_and_pop + H2D + prepare: the payload is released as soon as it is on the device
    void pop(ThreadSafeQueue<std::vector<float>*>& q, int indicator) {
        std::vector<float>* fm = nullptr;
        q.wait_and_pop(fm, indicator);
        check_hip(hipMemcpyAsync(d_fm, fm->data(), info.block_if * sizeof(float), hipMemcpyHostToDevice, s),
                  "hipMemcpyAsync");
        check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
        q.prepare(indicator);
        check_sdr(sdr_push_fm_demod(ctx, d_fm, info.block_if, s), "sdr_push_fm_demod");
    }
};

}  // namespace

void RF_frontend(args* p) {
    Stage st(p, 0);
    const size_t nbytes = 2 * (size_t)st.info.block_iq;
    uint8_t* host = nullptr;
    uint8_t* d_iq = nullptr;
    check_hip(hipHostMalloc(reinterpret_cast<void**>(&host), nbytes, hipHostMallocDefault), "hipHostMalloc");
    check_hip(hipMalloc(reinterpret_cast<void**>(&d_iq), nbytes), "hipMalloc");
    while (true) {
        std::cin.read(reinterpret_cast<char*>(host), (std::streamsize)nbytes);
        if (std::cin.eof()) {                // rffrontend.cpp:50-52: the program ends with status 1
            // flush like exit(1) would, but skip static destructors: the consumer threads may still
            // be inside HIP calls and the runtime must not be torn down under them
            std::fflush(stdout);
            std::fflush(stderr);
            std::_Exit(1);
        }
        check_hip(hipMemcpyAsync(d_iq, host, nbytes, hipMemcpyHostToDevice, st.s), "hipMemcpyAsync");
        check_sdr(sdr_frontend(st.ctx, d_iq, nbytes, st.s), "sdr_frontend");
        auto* fm = new std::vector<float>(st.info.block_if);
        check_sdr(sdr_get_fm_demod(st.ctx, st.d_fm, st.info.block_if, st.s), "sdr_get_fm_demod");
        check_hip(hipMemcpyAsync(fm->data(), st.d_fm, st.info.block_if * sizeof(float), hipMemcpyDeviceToHost, st.s),
                  "hipMemcpyAsync");
        check_hip(hipStreamSynchronize(st.s), "hipStreamSynchronize");
        p->queue.push(fm);                   // rffrontend.cpp:74
    }
}

void mono(args* p) {
    Stage st(p, 0);
    const int n = st.info.n_audio;
    std::vector<short> audio(n);
    int16_t* d_audio = nullptr;
    check_hip(hipMalloc(reinterpret_cast<void**>(&d_audio), n * sizeof(int16_t)), "hipMalloc");
    while (true) {
        st.pop(p->queue, 0);
        check_sdr(sdr_mono(st.ctx, d_audio, n, st.s), "sdr_mono");
        check_hip(hipMemcpyAsync(audio.data(), d_audio, n * sizeof(int16_t), hipMemcpyDeviceToHost, st.s),
                  "hipMemcpyAsync");
        check_hip(hipStreamSynchronize(st.s), "hipStreamSynchronize");
        std::fwrite(audio.data(), sizeof(short), audio.size(), stdout);   // mono.cpp:45
    }
}

void stereo(args* p) {
    Stage st(p, 0);
    const int n = 2 * st.info.n_audio;
    std::vector<short> lr(n);
    int16_t* d_lr = nullptr;
    check_hip(hipMalloc(reinterpret_cast<void**>(&d_lr), n * sizeof(int16_t)), "hipMalloc");
    while (true) {
        st.pop(p->queue, 0);
        check_sdr(sdr_stereo(st.ctx, d_lr, n, st.s), "sdr_stereo");
        check_hip(hipMemcpyAsync(lr.data(), d_lr, n * sizeof(int16_t), hipMemcpyDeviceToHost, st.s),
                  "hipMemcpyAsync");
        check_hip(hipStreamSynchronize(st.s), "hipStreamSynchronize");
        std::fwrite(lr.data(), sizeof(short), lr.size(), stdout);         // stereo.cpp:111
    }
}

void rds(args* p) {
    Stage st(p, p->rds_on ? 1 : 0);
    int32_t* d_nbits = nullptr;
    uint8_t* d_bits = nullptr;
    check_hip(hipMalloc(reinterpret_cast<void**>(&d_nbits), sizeof(int32_t)), "hipMalloc");
    check_hip(hipMalloc(reinterpret_cast<void**>(&d_bits), SDR_MAX_BITS), "hipMalloc");
    uint8_t bits[SDR_MAX_BITS];
    // frame layer state (rds.cpp:67-92)
    uint64_t reg = 0, chars = 0, output = 0;
    bool first_time = true;
    int decoder_cont = 0;
    unsigned int idx = 0;
    std::deque<std::string> window;
    std::vector<int> stream, stream_state;
    while (true) {
        st.pop(p->queue, 1);
        check_sdr(sdr_rds_dsp(st.ctx, nullptr, 0, st.s), "sdr_rds_dsp");
        check_sdr(sdr_rds_bits(st.ctx, nullptr, nullptr, nullptr, 0, d_nbits, d_bits, SDR_MAX_BITS, st.s),
                  "sdr_rds_bits");
        int32_t nb = -1;
        check_hip(hipMemcpyAsync(&nb, d_nbits, sizeof(int32_t), hipMemcpyDeviceToHost, st.s), "hipMemcpyAsync");
        check_hip(hipMemcpyAsync(bits, d_bits, SDR_MAX_BITS, hipMemcpyDeviceToHost, st.s), "hipMemcpyAsync");
        check_hip(hipStreamSynchronize(st.s), "hipStreamSynchronize");
        if (nb < 0) continue;                // block_count <= 5 or !rds_on (rds.cpp:135)
        decoder_cont++;                      // rds.cpp:181-189
        stream.insert(stream.end(), bits, bits + nb);
        if (decoder_cont == 15) {
            start_frame_sync(idx, stream, stream_state, reg, chars, output, first_time, window);
            decoder_cont = 0;
            idx = 0;
            stream.clear();
        }
    }
}
