// sdr_multi.cpp -- multi-channel receiver: the reference program's three stage threads
// (project.cpp:134-136: RF front end, audio, RDS) over nch channels at once, on the C ABI of
// libsdr_amd.so, with the queue payload on the device (include/dropin/fm_batch.h) and the I/O
// overlapped with the GPU work.
//
//   sdr_multi NCH [--mode 0-3] [--in FILE|-] [--out PREFIX] [--fast] [--cus N]
//
// Input: u8 I/Q, block after block, each block NCH rows of 2*block_iq bytes (channel after
// channel: the [block][channel][bytes] layout of bench.py). Output: PREFIX.pcm -- per block NCH
// rows of 2*n_audio int16 (L/R interleaved per channel, stereo.cpp:100-111) -- and PREFIX.rds, the
// RDS text of every channel ("ch <c>: " + parse()'s lines, rds_utilities.cpp:172-199). A summary
// line goes to stderr.
//
// Threads and streams (per block b):
//   reader  stdin/file -> pinned ring slot (3 slots)
//   RF      slot -H2D (copy stream)-> d_iq[b%2]; sdr_frontend (RF stream); fm_demod -> a recycled
//           FmBatch (device), event, push                              rffrontend.cpp:45-76
//   audio   pop(0); sdr_push_fm_demod; stereo_pre / stereo_pll (its own stream, CU-masked to the
//           first N CUs) / stereo_post; L/R -D2H-> pinned[b%2]; the write of block b-1 overlaps
//           the GPU work of block b                                       stereo.cpp:69-114
//   rds     pop(1); sdr_push_fm_demod; rds_pre / rds_pll / rds_post / rds_bits; bits -D2H-> host;
//           frame sync per channel every 15 decoding blocks (host)       rds.cpp:95-192
// The two consumers own their contexts (the reference's threads own their state); every device
// hand-off is a HIP event, so no thread synchronises with another's GPU work except through the
// queue's prepare() ordering.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <iostream>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>

#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "fm_batch.h"
#include "hip_util.h"
#include "rds_utilities.h"
#include "sdr_amd.h"

using sdrhost::check_hip;
using sdrhost::check_sdr;
using sdrhost::die;

namespace {

struct Opts {
    int nch = 0, mode = 0, flags = 0, cus = 64, device = 0;
    std::string in = "-", out = "sdr_multi";
};

// stream on CUs [0, n) (or all CUs when n == 0): the serial PLLs' own CUs
hipStream_t pll_stream(int device, int n_cu) {
    void* s = nullptr;
    if (n_cu > 0 && sdr_stream_create_cu_range(&s, device, 0, n_cu, 0) == SDR_OK) return (hipStream_t)s;
    hipStream_t h = nullptr;
    check_hip(hipStreamCreateWithFlags(&h, hipStreamNonBlocking), "hipStreamCreate");
    return h;
}

hipStream_t plain_stream() {
    hipStream_t h = nullptr;
    check_hip(hipStreamCreateWithFlags(&h, hipStreamNonBlocking), "hipStreamCreate");
    return h;
}

hipEvent_t new_event() {
    hipEvent_t e = nullptr;
    check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
}

// ------------------------------------------------------------------ reader: input -> pinned ring
struct Reader {
    static constexpr int SLOTS = 4;   // pinned input slots: the read of block b+2..b+3 rides out host jitter
    FILE* f = nullptr;
    size_t bytes = 0;
    uint8_t* slot[SLOTS] = {};
    hipEvent_t consumed[SLOTS] = {};    // the H2D copy out of the slot has completed
    bool armed[SLOTS] = {};
    std::mutex m;
    std::condition_variable cv;
    std::deque<int> filled, empty;
    bool eof = false;
    double read_s = 0.0;                // time spent reading (the input side of the I/O)
    int readers = 8;                    // pread threads per block (regular files; SDR_MULTI_READERS)
    long long file_size = 0, offset = 0;
    std::thread th;

    Reader(const std::string& path, size_t block_bytes) : bytes(block_bytes) {
        f = path == "-" ? stdin : std::fopen(path.c_str(), "rb");
        if (!f) die("cannot open " + path);
        if (f != stdin) {   // a regular file is read by several threads at once (pread of a block's parts)
            struct stat sb;
            if (fstat(fileno(f), &sb) == 0 && S_ISREG(sb.st_mode)) {
                file_size = (long long)sb.st_size;
                if (const char* e = std::getenv("SDR_MULTI_READERS")) readers = std::max(1, std::atoi(e));
            } else {
                readers = 1;
            }
        } else {
            readers = 1;
        }
        for (int i = 0; i < SLOTS; i++) {
            check_hip(hipHostMalloc(reinterpret_cast<void**>(&slot[i]), bytes, hipHostMallocDefault), "hipHostMalloc");
            consumed[i] = new_event();
            empty.push_back(i);
        }
        th = std::thread([this] { run(); });
    }
    void run() {
        for (;;) {
            int i;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [this] { return !empty.empty(); });
                i = empty.front();
                empty.pop_front();
            }
            if (armed[i]) check_hip(hipEventSynchronize(consumed[i]), "hipEventSynchronize");
            const auto r0 = std::chrono::steady_clock::now();
            const size_t got = readers > 1 ? pread_block(slot[i]) : std::fread(slot[i], 1, bytes, f);
            read_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - r0).count();
            std::lock_guard<std::mutex> lk(m);
            if (got < bytes) {             // a partial block ends the stream (rffrontend.cpp:50-52)
                eof = true;
                cv.notify_all();
                return;
            }
            filled.push_back(i);
            cv.notify_all();
        }
    }
    // one block by `readers` threads, each a contiguous part (pread at the block's file offset)
    size_t pread_block(uint8_t* dst) {
        if (offset + (long long)bytes > file_size) return 0;   // a partial block ends the stream
        const size_t part = (bytes / readers + 4095) / 4096 * 4096;
        std::vector<std::thread> th_;
        std::vector<size_t> got_(readers, 0);
        for (int r = 0; r < readers; r++) {
            const size_t lo = std::min(bytes, part * r), hi = std::min(bytes, part * (r + 1));
            th_.emplace_back([&, r, lo, hi] {
                size_t done = 0;
                while (lo + done < hi) {
                    const ssize_t k = ::pread(fileno(f), dst + lo + done, hi - lo - done, offset + (long long)(lo + done));
                    if (k <= 0) break;
                    done += (size_t)k;
                }
                got_[r] = done;
            });
        }
        size_t got = 0;
        for (int r = 0; r < readers; r++) {
            th_[r].join();
            got += got_[r];
        }
        offset += (long long)got;
        return got;
    }
    int next() {   // a filled slot, or -1 at the end of the input
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [this] { return !filled.empty() || eof; });
        if (filled.empty()) return -1;
        const int i = filled.front();
        filled.pop_front();
        return i;
    }
    void release(int i, hipStream_t copy_stream) {   // after the H2D copy of slot i is enqueued
        check_hip(hipEventRecord(consumed[i], copy_stream), "hipEventRecord");
        std::lock_guard<std::mutex> lk(m);
        armed[i] = true;
        empty.push_back(i);
        cv.notify_all();
    }
    ~Reader() {
        if (th.joinable()) th.join();
        for (int i = 0; i < SLOTS; i++) (void)hipHostFree(slot[i]);
        if (f && f != stdin) std::fclose(f);
    }
};

struct Shared {
    Opts o;
    sdr_info info{};
    ThreadSafeQueue<FmBatch*> q;
    long long blocks = 0;
    std::chrono::steady_clock::time_point t_first{};   // block 0's front end enqueued (steady-state clock start)
    double read_s = 0.0, h2d_ms = 0.0, d2h_ms = 0.0;   // input reads; GPU time of the H2D / L+R D2H copies
};

hipEvent_t timing_event() {
    hipEvent_t e = nullptr;
    check_hip(hipEventCreate(&e), "hipEventCreate");
    return e;
}
float elapsed_ms(hipEvent_t a, hipEvent_t b) {
    check_hip(hipEventSynchronize(b), "hipEventSynchronize");
    float ms = 0.0f;
    check_hip(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime");
    return ms;
}

// ------------------------------------------------------------------ RF front end (producer)
void rf_thread(Shared* sh) {
    const Opts& o = sh->o;
    check_hip(hipSetDevice(o.device), "hipSetDevice");
    sdr_ctx* ctx = nullptr;
    check_sdr(sdr_ctx_create(&ctx, o.device, o.nch, o.mode, 0, o.flags), "sdr_ctx_create");
    const sdr_info& in = sh->info;
    const size_t row = 2 * (size_t)in.block_iq, bytes = row * o.nch;
    hipStream_t s = plain_stream(), s_copy = plain_stream();
    uint8_t* d_iq[2] = {};
    hipEvent_t h2d[2] = {new_event(), new_event()}, fe_done[2] = {new_event(), new_event()};
    // copy timing: a ring of event pairs, read without blocking the producer (a pair is waited for
    // only when the ring wraps onto a copy that has not finished)
    constexpr int TR = 8;
    hipEvent_t c0[TR], c1[TR];
    for (int i = 0; i < TR; i++) { c0[i] = timing_event(); c1[i] = timing_event(); }
    long long timed = 0;                                    // blocks whose copy time is in h2d_ms
    auto harvest = [&](long long upto, bool wait) {
        for (; timed < upto; timed++) {
            const int t = (int)(timed % TR);
            if (!wait && hipEventQuery(c1[t]) == hipErrorNotReady) break;
            sh->h2d_ms += elapsed_ms(c0[t], c1[t]);
        }
    };
    for (auto& p : d_iq) check_hip(hipMalloc(reinterpret_cast<void**>(&p), bytes), "hipMalloc");
    Reader rd(o.in, bytes);
    for (long long b = 0;; b++) {
        const int slot = rd.next();
        if (slot < 0) break;
        const int k = (int)(b & 1);
        if (b >= 2) check_hip(hipStreamWaitEvent(s_copy, fe_done[k], 0), "hipStreamWaitEvent");
        harvest(b - TR + 1, true);                          // the ring slot this block reuses
        harvest(b, false);
        const int t = (int)(b % TR);
        check_hip(hipEventRecord(c0[t], s_copy), "hipEventRecord");
        check_hip(hipMemcpyAsync(d_iq[k], rd.slot[slot], bytes, hipMemcpyHostToDevice, s_copy), "hipMemcpyAsync");
        check_hip(hipEventRecord(c1[t], s_copy), "hipEventRecord");
        check_hip(hipEventRecord(h2d[k], s_copy), "hipEventRecord");
        rd.release(slot, s_copy);
        check_hip(hipStreamWaitEvent(s, h2d[k], 0), "hipStreamWaitEvent");
        check_sdr(sdr_frontend(ctx, d_iq[k], row, s), "sdr_frontend");
        check_hip(hipEventRecord(fe_done[k], s), "hipEventRecord");
        FmBatch* fb = sh->q.acquire();
        for (auto& e : fb->released) check_hip(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent");
        check_sdr(sdr_get_fm_demod(ctx, fb->d_fm, fb->stride, s), "sdr_get_fm_demod");
        check_hip(hipEventRecord(fb->ready, s), "hipEventRecord");
        fb->block = b;
        sh->q.push(fb);                                     // rffrontend.cpp:74
        sh->blocks = b + 1;
        if (b == 0) sh->t_first = std::chrono::steady_clock::now();
    }
    sh->q.push(nullptr);                                    // end of stream
    check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
    harvest(sh->blocks, true);
    sh->read_s = rd.read_s;
    for (auto& p : d_iq) (void)hipFree(p);
    sdr_ctx_destroy(ctx);
}

// consumer prologue: the batch into this thread's context (wait_and_pop + prepare, async)
bool consume(Shared* sh, sdr_ctx* ctx, hipStream_t s, int indicator) {
    FmBatch* fb = nullptr;
    sh->q.wait_and_pop(fb, indicator);
    if (!fb) return false;
    check_hip(hipStreamWaitEvent(s, fb->ready, 0), "hipStreamWaitEvent");
    check_sdr(sdr_push_fm_demod(ctx, fb->d_fm, fb->stride, s), "sdr_push_fm_demod");
    check_hip(hipEventRecord(fb->released[indicator], s), "hipEventRecord");
    sh->q.prepare(indicator);
    return true;
}

// ------------------------------------------------------------------ audio (consumer 0)
void audio_thread(Shared* sh) {
    const Opts& o = sh->o;
    check_hip(hipSetDevice(o.device), "hipSetDevice");
    sdr_ctx* ctx = nullptr;
    check_sdr(sdr_ctx_create(&ctx, o.device, o.nch, o.mode, 0, o.flags), "sdr_ctx_create");
    const size_t n = 2 * (size_t)sh->info.n_audio, bytes = n * o.nch * sizeof(int16_t);
    hipStream_t s = plain_stream(), s_pll = pll_stream(o.device, o.cus);
    hipEvent_t pre = new_event(), pll = new_event(), out_ready[2] = {new_event(), new_event()};
    hipEvent_t d0[2] = {timing_event(), timing_event()}, d1[2] = {timing_event(), timing_event()};
    int16_t *d_lr[2] = {}, *h_lr[2] = {};
    for (int k = 0; k < 2; k++) {
        check_hip(hipMalloc(reinterpret_cast<void**>(&d_lr[k]), bytes), "hipMalloc");
        check_hip(hipHostMalloc(reinterpret_cast<void**>(&h_lr[k]), bytes, hipHostMallocDefault), "hipHostMalloc");
    }
    FILE* f = std::fopen((o.out + ".pcm").c_str(), "wb");
    if (!f) die("cannot write " + o.out + ".pcm");
    long long b = 0;
    auto write_block = [&](long long blk) {   // stereo.cpp:111, for every channel
        const int k = (int)(blk & 1);
        check_hip(hipEventSynchronize(out_ready[k]), "hipEventSynchronize");
        sh->d2h_ms += elapsed_ms(d0[k], d1[k]);
        std::fwrite(h_lr[k], 1, bytes, f);
    };
    while (consume(sh, ctx, s, 0)) {
        const int k = (int)(b & 1);
        check_sdr(sdr_stereo_pre(ctx, s), "sdr_stereo_pre");
        check_hip(hipEventRecord(pre, s), "hipEventRecord");
        check_hip(hipStreamWaitEvent(s_pll, pre, 0), "hipStreamWaitEvent");
        check_sdr(sdr_stereo_pll(ctx, s_pll), "sdr_stereo_pll");
        check_hip(hipEventRecord(pll, s_pll), "hipEventRecord");
        check_hip(hipStreamWaitEvent(s, pll, 0), "hipStreamWaitEvent");
        check_sdr(sdr_stereo_post(ctx, d_lr[k], n, s), "sdr_stereo_post");
        check_hip(hipEventRecord(d0[k], s), "hipEventRecord");
        check_hip(hipMemcpyAsync(h_lr[k], d_lr[k], bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
        check_hip(hipEventRecord(d1[k], s), "hipEventRecord");
        check_hip(hipEventRecord(out_ready[k], s), "hipEventRecord");
        if (b >= 1) write_block(b - 1);                     // overlaps block b's GPU work
        b++;
    }
    if (b >= 1) write_block(b - 1);
    std::fclose(f);
    check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
    sdr_ctx_destroy(ctx);
}

// ------------------------------------------------------------------ RDS (consumer 1)
struct FrameState {   // rds.cpp:67-92, per channel
    uint64_t reg = 0, chars = 0, output = 0;
    bool first_time = true;
    int decoder_cont = 0;
    unsigned int idx = 0;
    std::deque<std::string> window;
    std::vector<int> stream, stream_state;
    std::string text;
};

void rds_thread(Shared* sh) {
    const Opts& o = sh->o;
    check_hip(hipSetDevice(o.device), "hipSetDevice");
    sdr_ctx* ctx = nullptr;
    check_sdr(sdr_ctx_create(&ctx, o.device, o.nch, o.mode, 1, o.flags), "sdr_ctx_create");
    hipStream_t s = plain_stream(), s_pll = pll_stream(o.device, o.cus);
    hipEvent_t pre = new_event(), pll = new_event(), out_ready[2] = {new_event(), new_event()};
    int32_t *d_nbits = nullptr, *h_nbits[2] = {};
    uint8_t *d_bits = nullptr, *h_bits[2] = {};
    check_hip(hipMalloc(reinterpret_cast<void**>(&d_nbits), o.nch * sizeof(int32_t)), "hipMalloc");
    check_hip(hipMalloc(reinterpret_cast<void**>(&d_bits), (size_t)o.nch * SDR_MAX_BITS), "hipMalloc");
    for (int k = 0; k < 2; k++) {
        check_hip(hipHostMalloc(reinterpret_cast<void**>(&h_nbits[k]), o.nch * sizeof(int32_t), hipHostMallocDefault),
                  "hipHostMalloc");
        check_hip(hipHostMalloc(reinterpret_cast<void**>(&h_bits[k]), (size_t)o.nch * SDR_MAX_BITS,
                                hipHostMallocDefault), "hipHostMalloc");
    }
    std::vector<FrameState> fs((size_t)o.nch);
    auto frame_layer = [&](long long blk) {   // rds.cpp:181-189 per channel; parse() prints to cerr
        const int k = (int)(blk & 1);
        check_hip(hipEventSynchronize(out_ready[k]), "hipEventSynchronize");
        std::streambuf* saved = std::cerr.rdbuf();
        for (int c = 0; c < o.nch; c++) {
            const int nb = h_nbits[k][c];
            if (nb < 0) continue;                       // block_count <= 5 (rds.cpp:135)
            FrameState& st = fs[(size_t)c];
            const uint8_t* bits = h_bits[k] + (size_t)c * SDR_MAX_BITS;
            st.decoder_cont++;
            st.stream.insert(st.stream.end(), bits, bits + nb);
            if (st.decoder_cont == 15) {
                std::ostringstream text;
                std::cerr.rdbuf(text.rdbuf());
                start_frame_sync(st.idx, st.stream, st.stream_state, st.reg, st.chars, st.output, st.first_time,
                                 st.window);
                std::cerr.rdbuf(saved);
                st.text += text.str();
                st.decoder_cont = 0;
                st.idx = 0;
                st.stream.clear();
            }
        }
    };
    long long b = 0;
    while (consume(sh, ctx, s, 1)) {
        const int k = (int)(b & 1);
        check_sdr(sdr_rds_pre(ctx, s), "sdr_rds_pre");
        check_hip(hipEventRecord(pre, s), "hipEventRecord");
        check_hip(hipStreamWaitEvent(s_pll, pre, 0), "hipStreamWaitEvent");
        check_sdr(sdr_rds_pll(ctx, s_pll), "sdr_rds_pll");
        check_hip(hipEventRecord(pll, s_pll), "hipEventRecord");
        check_hip(hipStreamWaitEvent(s, pll, 0), "hipStreamWaitEvent");
        check_sdr(sdr_rds_post(ctx, nullptr, 0, s), "sdr_rds_post");
        check_sdr(sdr_rds_bits(ctx, nullptr, nullptr, nullptr, 0, d_nbits, d_bits, SDR_MAX_BITS, s), "sdr_rds_bits");
        check_hip(hipMemcpyAsync(h_nbits[k], d_nbits, o.nch * sizeof(int32_t), hipMemcpyDeviceToHost, s),
                  "hipMemcpyAsync");
        check_hip(hipMemcpyAsync(h_bits[k], d_bits, (size_t)o.nch * SDR_MAX_BITS, hipMemcpyDeviceToHost, s),
                  "hipMemcpyAsync");
        check_hip(hipEventRecord(out_ready[k], s), "hipEventRecord");
        if (b >= 1) frame_layer(b - 1);
        b++;
    }
    if (b >= 1) frame_layer(b - 1);
    FILE* f = std::fopen((o.out + ".rds").c_str(), "w");
    if (!f) die("cannot write " + o.out + ".rds");
    for (int c = 0; c < o.nch; c++) {
        std::istringstream lines(fs[(size_t)c].text);
        for (std::string line; std::getline(lines, line);) std::fprintf(f, "ch %d: %s\n", c, line.c_str());
    }
    std::fclose(f);
    check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
    sdr_ctx_destroy(ctx);
}

[[noreturn]] void usage() {
    std::fprintf(stderr, "usage: sdr_multi NCH [--mode 0-3] [--in FILE|-] [--out PREFIX] [--fast] [--cus N]\n");
    std::exit(1);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) usage();
    Shared sh;
    Opts& o = sh.o;
    o.nch = std::atoi(argv[1]);
    if (o.nch <= 0) usage();
    for (int i = 2; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--mode" && i + 1 < argc) o.mode = std::atoi(argv[++i]);
        else if (a == "--in" && i + 1 < argc) o.in = argv[++i];
        else if (a == "--out" && i + 1 < argc) o.out = argv[++i];
        else if (a == "--cus" && i + 1 < argc) o.cus = std::atoi(argv[++i]);
        else if (a == "--fast") o.flags |= SDR_FLAG_FAST_FRONTEND;
        else usage();
    }
    if (const char* dev = std::getenv("SDR_DEVICE")) o.device = std::atoi(dev);
    check_hip(hipSetDevice(o.device), "hipSetDevice");
    {
        sdr_ctx* probe = nullptr;   // sizes of the mode
        check_sdr(sdr_ctx_create(&probe, o.device, 1, o.mode, 0, 0), "sdr_ctx_create");
        check_sdr(sdr_ctx_info(probe, &sh.info), "sdr_ctx_info");
        sdr_ctx_destroy(probe);
    }
    // two recycled device batches of fm_demod [nch][block_if] (threadsafequeue.h's one slot, plus
    // the one the producer fills meanwhile)
    std::vector<FmBatch> batches(2);
    for (auto& fb : batches) {
        fb.nch = o.nch;
        fb.n = sh.info.block_if;
        fb.stride = (size_t)(fb.n + 63) / 64 * 64;
        check_hip(hipMalloc(reinterpret_cast<void**>(&fb.d_fm), fb.stride * o.nch * sizeof(float)), "hipMalloc");
        fb.ready = new_event();
        for (auto& e : fb.released) {
            e = new_event();
            check_hip(hipEventRecord(e, nullptr), "hipEventRecord");   // trivially complete
        }
        sh.q.add_free(&fb);
    }
    check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
    const auto t0 = std::chrono::steady_clock::now();
    std::thread t_rds(rds_thread, &sh);      // project.cpp:134-136
    std::thread t_audio(audio_thread, &sh);
    std::thread t_rf(rf_thread, &sh);
    t_rf.join();
    t_audio.join();
    t_rds.join();
    const auto t_end = std::chrono::steady_clock::now();
    const double sec = std::chrono::duration<double>(t_end - t0).count();
    const double steady = std::chrono::duration<double>(t_end - sh.t_first).count();
    const double samples = (double)sh.blocks * o.nch * sh.info.block_iq;
    const double signal_s = (double)sh.blocks * sh.info.block_iq / (double)sh.info.rf_Fs;
    const double in_gb = (double)sh.blocks * o.nch * 2.0 * sh.info.block_iq / 1e9;
    const double steady_samples = (double)(sh.blocks - 1) * o.nch * sh.info.block_iq;
    char after0[128] = "after block 0 n/a (fewer than 2 blocks)";
    if (sh.blocks >= 2 && steady > 0)
        std::snprintf(after0, sizeof(after0), "after block 0 %.1f MS/s (%.1fx real time)", steady_samples / steady / 1e6,
                      (double)(sh.blocks - 1) * sh.info.block_iq / (double)sh.info.rf_Fs / steady);
    std::fprintf(stderr,
                 "sdr_multi: %d channels x %lld blocks in %.3f s: %.1f MS/s I/Q, %.1fx real time; %s; "
                 "input read %.3f s (%.1f GB/s), H2D %.3f s GPU time (%.1f GB/s), L/R D2H %.3f s\n",
                 o.nch, sh.blocks, sec, sec > 0 ? samples / sec / 1e6 : 0.0, sec > 0 ? signal_s / sec : 0.0, after0,
                 sh.read_s, sh.read_s > 0 ? in_gb / sh.read_s : 0.0, sh.h2d_ms / 1e3,
                 sh.h2d_ms > 0 ? in_gb / (sh.h2d_ms / 1e3) : 0.0, sh.d2h_ms / 1e3);
    for (auto& fb : batches) (void)hipFree(fb.d_fm);
    return 0;
}
