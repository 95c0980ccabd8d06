// sdr_multi.cpp -- multi-channel receiver CLI over the engine of include/sdr_multi.h (the reference
// program's three stage threads over nch channels, project.cpp:134-136).
//
//   sdr_multi NCH [--mode 0-3] [--in FILE|-] [--out PREFIX] [--fast] [--cus N]
//
// Input: u8 I/Q, block after block, each block NCH rows of 2*block_iq bytes (channel after
// channel: the [block][channel][bytes] layout of bench.py). Output: PREFIX.pcm -- per block NCH
// rows of 2*n_audio int16 (L/R interleaved per channel, stereo.cpp:100-111) -- and PREFIX.rds, the
// RDS text of every channel ("ch <c>: " + parse()'s lines, rds_utilities.cpp:172-199). --cus N: the
// two consumers' PLLs on CUs [0, N) (persistent launches when the input is a regular file), 0: no
// CU masks. A summary line goes to stderr.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "sdr_amd.h"
#include "sdr_multi.h"

namespace {
[[noreturn]] void usage() {
    std::fprintf(stderr, "usage: sdr_multi NCH [--mode 0-3] [--in FILE|-] [--out PREFIX] [--fast] [--cus N]\n");
    std::exit(1);
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) usage();
    sdr_multi_opts o{};
    o.nch = std::atoi(argv[1]);
    o.pll_cus = 64;
    std::string in = "-", out = "sdr_multi";
    if (o.nch <= 0) usage();
    for (int i = 2; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--mode" && i + 1 < argc) o.mode = std::atoi(argv[++i]);
        else if (a == "--in" && i + 1 < argc) in = argv[++i];
        else if (a == "--out" && i + 1 < argc) out = argv[++i];
        else if (a == "--cus" && i + 1 < argc) o.pll_cus = std::atoi(argv[++i]);
        else if (a == "--fast") o.flags |= SDR_FLAG_FAST_FRONTEND;
        else usage();
    }
    if (const char* dev = std::getenv("SDR_DEVICE")) o.device = std::atoi(dev);
    o.in_path = in.c_str();
    o.out_prefix = out.c_str();
    sdr_multi_stats st{};
    const int rc = sdr_multi_run(&o, &st);
    if (rc != SDR_OK) {
        std::fprintf(stderr, "sdr_multi: %d %s\n", rc, sdr_last_error());
        return 1;
    }
    sdr_ctx* probe = nullptr;   // sizes of the mode
    sdr_info info{};
    if (sdr_ctx_create(&probe, o.device, 1, o.mode, 0, 0) != SDR_OK || sdr_ctx_info(probe, &info) != SDR_OK) return 1;
    sdr_ctx_destroy(probe);
    const double samples = (double)st.blocks * o.nch * info.block_iq;
    const double signal_s = (double)st.blocks * info.block_iq / (double)info.rf_Fs;
    const double in_gb = (double)st.blocks * o.nch * 2.0 * info.block_iq / 1e9;
    char after0[128] = "after block 0 n/a (fewer than 2 blocks)";
    if (st.blocks >= 2 && st.steady_seconds > 0)
        std::snprintf(after0, sizeof(after0), "after block 0 %.1f MS/s (%.1fx real time)",
                      (double)(st.blocks - 1) * o.nch * info.block_iq / st.steady_seconds / 1e6,
                      (double)(st.blocks - 1) * info.block_iq / (double)info.rf_Fs / st.steady_seconds);
    std::fprintf(stderr,
                 "sdr_multi: %d channels x %lld blocks in %.3f s: %.1f MS/s I/Q, %.1fx real time; %s; PLLs %s "
                 "(%.4f ms per block); input read %.3f s (%.1f GB/s), H2D %.3f s GPU time (%.1f GB/s), "
                 "L/R D2H %.3f s\n",
                 o.nch, st.blocks, st.seconds, st.seconds > 0 ? samples / st.seconds / 1e6 : 0.0,
                 st.seconds > 0 ? signal_s / st.seconds : 0.0, after0, st.persistent ? "persistent" : "per-block dispatch",
                 st.pll_period_ms, st.read_s, st.read_s > 0 ? in_gb / st.read_s : 0.0, st.h2d_ms / 1e3,
                 st.h2d_ms > 0 ? in_gb / (st.h2d_ms / 1e3) : 0.0, st.d2h_ms / 1e3);
    return 0;
}
