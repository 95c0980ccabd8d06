// sdr_project.cpp -- command-line receiver with the reference program's interface
// (src/project.cpp): `sdr_project [mode 0-3] [m|s|r] < iq.u8 > audio.s16` reads RTL-SDR style
// interleaved u8 I/Q from stdin, writes int16 PCM (mono, or L/R interleaved) to stdout and RDS
// text to stderr, with three threads (RF front end, audio, RDS) joined by the one-slot queue. All
// per-block DSP runs on the MI355X (device: env SDR_DEVICE, default 0).
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <thread>
#include <vector>

#include "args.h"
#include "mono.h"
#include "rds.h"
#include "rffrontend.h"
#include "stereo.h"

namespace {
[[noreturn]] void usage() {
    std::cerr << "usage: sdr_project [mode 0-3] [m|s|r] < iq.u8 > audio.s16\n"
                 "  modes: 0 (2.4 MS/s), 1 (1.44 MS/s), 2 (2.4 MS/s, 147/800), 3 (1.152 MS/s, 147/1280)\n"
                 "  types: m mono, s stereo, r stereo + RDS\n";
    std::exit(1);
}
}  // namespace

int main(int argc, char** argv) {
    ThreadSafeQueue<std::vector<float>*> queue;
    args a = {queue, 2400000, 100000, 101, 10, 5, 1, 240000, 16000, 48000, 39, false};
    if (const char* dev = std::getenv("SDR_DEVICE")) a.device = std::atoi(dev);
    void (*audio)(args*) = &mono;
    if (argc >= 3) {
        switch (std::atoi(argv[1])) {
            case 0: break;
            case 1: a.rf_Fs = 1440000; a.rf_decim = 4; a.audio_decim = 9; a.if_Fs = 360000; break;
            case 2: a.audio_decim = 800; a.audio_upsample = 147; a.symbol_Fs = 20; break;
            case 3: a.rf_Fs = 1152000; a.rf_decim = 3; a.audio_decim = 1280; a.if_Fs = 384000;
                    a.audio_upsample = 147; a.symbol_Fs = 20; break;
            default: usage();
        }
        switch (argv[2][0]) {
            case 'm': audio = &mono; break;
            case 's': audio = &stereo; break;
            case 'r': audio = &stereo; a.rds_on = true; break;
            default: usage();
        }
    }
    std::thread t_rds(rds, &a);
    std::thread t_audio(audio, &a);
    std::thread t_rf(RF_frontend, &a);
    t_rds.join();
    t_audio.join();
    t_rf.join();
    return 0;
}
