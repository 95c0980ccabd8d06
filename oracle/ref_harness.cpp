// ref_harness.cpp -- golden-vector generator over the UNMODIFIED reference DSP primitives.
// TEST INFRASTRUCTURE ONLY: built into oracle/_ref/ by oracle/Makefile from the reference's own
// src/filter.cpp, src/demod.cpp, src/pll.cpp and src/rds_utilities.cpp (never copied).
//
// It replays the per-block bodies of the reference stage threads on one channel of u8 I/Q read
// from a file, calling the reference functions exactly as the stage loops do:
//   RF_frontend  src/rffrontend.cpp:58-71      mono    src/mono.cpp:34-42
//   stereo       src/stereo.cpp:74-107         rds     src/rds.cpp:105-189
// and dumps every per-block output (plus full intermediates for chosen blocks) as raw files.
// The stage glue here is cross-checked against the real `project` binary (oracle/_ref/project)
// by tests/golden/make_golden.py: its stdout PCM must equal the mono/stereo audio written here.
//
// usage: ref_harness <iq.u8> <nblocks> <mode> <rds_on 0|1> <out_prefix> [dump_block ...]
#include "demod.h"
#include "dy4.h"
#include "filter.h"
#include "pll.h"
#include "rds_utilities.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <fstream>
#include <set>
#include <string>
#include <vector>

namespace {

template <typename T>
void put(const std::string& path, const std::vector<T>& v, bool append = true) {
    FILE* f = std::fopen(path.c_str(), append ? "ab" : "wb");
    if (!f) { std::perror(path.c_str()); std::exit(2); }
    if (!v.empty()) std::fwrite(v.data(), sizeof(T), v.size(), f);
    std::fclose(f);
}

void fresh(const std::string& path) { FILE* f = std::fopen(path.c_str(), "wb"); if (f) std::fclose(f); }

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s iq.u8 nblocks mode rds_on out_prefix [dump_block ...]\n", argv[0]);
        return 2;
    }
    const char* in_path = argv[1];
    const int nblocks = std::atoi(argv[2]);
    const int mode = std::atoi(argv[3]);
    const bool rds_on = std::atoi(argv[4]) != 0;
    const std::string pre = argv[5];
    std::set<int> dump;
    for (int i = 6; i < argc; i++) dump.insert(std::atoi(argv[i]));

    // args as project.cpp:31-108
    int rf_Fs = 2400000, rf_Fc = 100000, rf_decim = 10, if_Fs = 240000, audio_Fc = 16000, symbol_Fs = 39;
    unsigned short rf_taps = 101;
    float audio_decim = 5, audio_upsample = 1;
    switch (mode) {
        case 0: rf_Fs = 2.4e6; rf_decim = 10; audio_decim = 5; if_Fs = 240e3; break;
        case 1: rf_Fs = 1.44e6; rf_decim = 4; audio_decim = 9; if_Fs = 360e3; break;
        case 2: rf_Fs = 2.4e6; rf_decim = 10; audio_decim = 800; if_Fs = 240e3; audio_upsample = 147; symbol_Fs = 20; break;
        case 3: rf_Fs = 1.152e6; rf_decim = 3; audio_decim = 1280; if_Fs = 384e3; audio_upsample = 147; symbol_Fs = 20; break;
        default: return 2;
    }
    const int U = audio_upsample, D = audio_decim;
    const int block_iq = (1470 * rf_decim * D) / U;     // rffrontend.cpp:21
    const int block_if = (1470 * D) / U;                // mono.cpp:17 / stereo.cpp:12 / rds.cpp:24

    // ---- prologues: taps and state exactly as the stage functions set them up ----
    std::vector<float> rf_h;
    impulseResponseLPF(rf_Fs, rf_Fc, rf_taps, rf_h);                                  // rffrontend.cpp:24
    std::vector<float> state_I(rf_h.size() - 1, 0.0), state_Q(rf_h.size() - 1, 0.0);   // :36-39
    float prev_I = 0, prev_Q = 0;

    std::vector<float> audio_h_m;
    impulseResponseLPF(if_Fs * U, audio_Fc, rf_taps * U, audio_h_m, U);               // mono.cpp:22
    std::vector<float> state_audio(audio_h_m.size() - 1);                             // mono.cpp:27

    std::vector<float> mono_delay_h, audio_h, pilot_h, stereo_h, carrier_h;
    float fb_pilot[] = {18.5e3, 19.5e3}, fb_carrier[] = {37.5e3, 38.5e3}, fb_stereo[] = {22e3, 54e3};
    impulseResponseAPF(1, rf_taps, mono_delay_h);                                      // stereo.cpp:63
    impulseResponseLPF(if_Fs * audio_upsample, audio_Fc, rf_taps * audio_upsample, audio_h, audio_upsample); // :64
    impulseResponseBPF(rf_Fs / rf_decim, fb_pilot, rf_taps, pilot_h);                 // :65
    impulseResponseBPF(rf_Fs / rf_decim, fb_carrier, rf_taps, carrier_h);             // :66 (unused)
    impulseResponseBPF(rf_Fs / rf_decim, fb_stereo, rf_taps, stereo_h);               // :67
    std::vector<float> carrier(block_if + 1, 0.0);
    carrier[carrier.size() - 1] = 1.0;                                                 // stereo.cpp:45
    std::vector<float> extracted_pilot(block_if, 0.0), extracted_pilot_state(rf_taps - 1, 0.0);
    std::vector<float> band, band_state(rf_taps - 1, 0.0), stereo_dc(block_if, 0.0);
    std::vector<float> mono_delay(block_if, 0.0), mono_delay_state(rf_taps - 1, 0.0);
    std::vector<float> mono_filt, mono_state(rf_taps - 1, 0.0), stereo_filt, stereo_state(rf_taps - 1, 0.0);
    pllblock_args st_args;
    st_args.feedbackI = 1.0; st_args.feedbackQ = 0.0; st_args.integrator = 0.0;
    st_args.phaseEst = 0.0; st_args.trigOffset = 0.0; st_args.lastCarrier = 1.0;       // stereo.cpp:51-57

    std::vector<float> rds_h, rds_delay_h, rds_baseband_h, rds_pilot_h, rrc_h;
    float fb_rds[] = {54e3, 60e3}, fb_rds_squared[] = {113.5e3, 114.5e3};
    impulseResponseLPF(if_Fs * 247, 3e3, rf_taps * 247, rds_baseband_h, 247);         // rds.cpp:61
    impulseResponseBPF(if_Fs, fb_rds, rf_taps, rds_h);                                // :62
    impulseResponseBPF(if_Fs, fb_rds_squared, rf_taps, rds_pilot_h);                  // :63
    impulseResponseAPF(1, rf_taps, rds_delay_h);                                      // :64
    impulseResponseRRC(2375 * symbol_Fs, rf_taps, rrc_h);                             // :65
    int block_count = 0, half_symbol = 0, start = 0, last_bit = 0, sample_offset = 0;
    std::vector<float> rds_band, rds_band_squared(block_if, 0.0), rds_band_state(rf_taps - 1, 0.0);
    std::vector<float> gen_pilot, gen_pilot_state(rf_taps - 1, 0.0);
    std::vector<float> IPLL(block_if + 1, 0.0);
    IPLL[IPLL.size() - 1] = 1;                                                         // rds.cpp:38
    std::vector<float> rds_band_delay, rds_band_delay_state(rf_taps - 1, 0.0), rds_dc(block_if, 0.0);
    std::vector<float> rds_filt, rds_filt_state(rf_taps - 1, 0.0), rds_clean, rds_clean_state(rf_taps - 1, 0.0);
    std::vector<int> symbols, bits, decoded_bits;
    symbols.reserve(100); bits.reserve(100);
    pllblock_args rds_args;
    rds_args.feedbackI = 1.0; rds_args.feedbackQ = 0.0; rds_args.integrator = 0.0;
    rds_args.phaseEst = 0.0; rds_args.trigOffset = 0.0; rds_args.lastCarrier = 0.0;   // rds.cpp:51-56
    uint64_t reg = 0, chars = 0, output = 0;
    bool first_time = true;
    int decoder_cont = 0;
    unsigned int idx = 0;
    std::deque<std::string> window;
    std::vector<int> decoded_bits_stream, decoded_bits_stream_state;

    // RDS text (parse() prints to std::cerr) goes to <pre>rds_text.txt
    std::ofstream text_out(pre + "rds_text.txt");
    std::streambuf* old_cerr = std::cerr.rdbuf(text_out.rdbuf());

    // taps
    put(pre + "taps_rf.f32", rf_h, false);
    put(pre + "taps_audio.f32", audio_h, false);
    put(pre + "taps_pilot.f32", pilot_h, false);
    put(pre + "taps_stereo.f32", stereo_h, false);
    put(pre + "taps_carrier.f32", carrier_h, false);
    put(pre + "taps_apf.f32", mono_delay_h, false);
    put(pre + "taps_rds.f32", rds_h, false);
    put(pre + "taps_rds_sq.f32", rds_pilot_h, false);
    put(pre + "taps_rds_bb.f32", rds_baseband_h, false);
    put(pre + "taps_rrc.f32", rrc_h, false);
    for (const char* s : {"fm_demod.f32", "mono.i16", "stereo.i16", "rds_clean.f32", "bits.txt"}) fresh(pre + s);

    FILE* fin = std::fopen(in_path, "rb");
    if (!fin) { std::perror(in_path); return 2; }
    std::vector<uint8_t> IQ_buf(2 * block_iq);
    std::vector<float> I(block_iq), Q(block_iq), I_ds, Q_ds;
    std::vector<float>* IQ[] = {&I, &Q};
    FILE* fbits = std::fopen((pre + "bits.txt").c_str(), "w");

    for (int b = 0; b < nblocks; b++) {
        if (std::fread(IQ_buf.data(), 1, IQ_buf.size(), fin) != IQ_buf.size()) break;
        // ---- RF_frontend body (rffrontend.cpp:55-71)
        std::vector<float> fm_demod(block_if);
        for (int s = 0; s < 2 * block_iq; s++)
            (*IQ[s & 0x01])[s >> 1] = float(((unsigned char)IQ_buf[s] - 128.0) / 128.0);
        convolveFIR(I_ds, I, rf_h, state_I, rf_decim);
        convolveFIR(Q_ds, Q, rf_h, state_Q, rf_decim);
        fmDemodNoArctan(I_ds, Q_ds, prev_I, prev_Q, fm_demod);
        put(pre + "fm_demod.f32", fm_demod);

        // ---- mono body (mono.cpp:34-42)
        std::vector<float> audio_filt;
        std::vector<short> audio(block_if * U / D);
        convolveFIR(audio_filt, fm_demod, audio_h_m, state_audio, U, D);
        for (unsigned int i = 0; i < audio.size(); i++) audio[i] = static_cast<short int>(16384 * audio_filt[i]);
        put(pre + "mono.i16", audio);

        // ---- stereo body (stereo.cpp:74-107)
        convolveFIR(extracted_pilot, fm_demod, pilot_h, extracted_pilot_state, 1);
        fmpll(extracted_pilot, 19e3, rf_Fs / rf_decim, carrier, st_args, 2.0, 0, 0.01);
        convolveFIR(band, fm_demod, stereo_h, band_state, 1);
        for (unsigned int i = 0; i < band.size(); i++) stereo_dc[i] = 2.0 * band[i] * carrier[i];
        convolveFIR(mono_delay, fm_demod, mono_delay_h, mono_delay_state, 1);
        if (dump.count(b)) {
            std::string p = pre + "b" + std::to_string(b) + "_";
            put(p + "pilot.f32", extracted_pilot, false);
            put(p + "carrier.f32", carrier, false);
            put(p + "band.f32", band, false);
            put(p + "stereo_dc.f32", stereo_dc, false);
            put(p + "mono_delay.f32", mono_delay, false);
            put(p + "I_ds.f32", I_ds, false);
            put(p + "Q_ds.f32", Q_ds, false);
        }
        convolveFIR(mono_filt, mono_delay, audio_h, mono_state, audio_upsample, audio_decim);
        convolveFIR(stereo_filt, stereo_dc, audio_h, stereo_state, audio_upsample, audio_decim);
        std::vector<short> stereo(2 * ((int)(block_if * audio_upsample) / (int)audio_decim));
        for (int s = 0; s < (int)stereo.size(); s++) {
            short right = static_cast<short int>(16384 * (mono_filt[s >> 1] - stereo_filt[s >> 1]));
            short left = static_cast<short int>(16384 * (mono_filt[s >> 1] + stereo_filt[s >> 1]));
            stereo[s] = ((left) & ((s & 0x01) - 1)) | ((right) & ~((s & 0x01) - 1));
        }
        put(pre + "stereo.i16", stereo);

        // ---- rds body (rds.cpp:105-189)
        convolveFIR(rds_band, fm_demod, rds_h, rds_band_state, 1);
        for (int i = 0; i < block_if; i++) rds_band_squared[i] = rds_band[i] * rds_band[i];
        convolveFIR(gen_pilot, rds_band_squared, rds_pilot_h, gen_pilot_state, 1);
        fmpll(gen_pilot, 114e3, if_Fs, IPLL, rds_args, 0.5, 0, 0.001);
        convolveFIR(rds_band_delay, rds_band, rds_delay_h, rds_band_delay_state, 1);
        for (int i = 0; i < block_if; i++) rds_dc[i] = 2 * rds_band_delay[i] * IPLL[i];
        convolveFIR(rds_filt, rds_dc, rds_baseband_h, rds_filt_state, 247, 640);
        convolveFIR(rds_clean, rds_filt, rrc_h, rds_clean_state, 1);
        put(pre + "rds_clean.f32", rds_clean);
        if (dump.count(b)) {
            std::string p = pre + "b" + std::to_string(b) + "_";
            put(p + "rds_band.f32", rds_band, false);
            put(p + "gen_pilot.f32", gen_pilot, false);
            put(p + "ipll.f32", IPLL, false);
            put(p + "rds_dc.f32", rds_dc, false);
            put(p + "rds_filt.f32", rds_filt, false);
        }
        std::fprintf(fbits, "%d", b);
        if (block_count > 5 && rds_on) {
            sample_offset = cdr(symbol_Fs, rds_clean);
            symbols.clear();
            for (int i = 0; sample_offset + i * symbol_Fs < (int)rds_clean.size(); i++)
                symbols.push_back(rds_clean[sample_offset + i * symbol_Fs] > 0);
            manchester_decode(bits, symbols, block_count, half_symbol, start);
            differential_decode(decoded_bits, bits, last_bit, block_count);
            std::fprintf(fbits, " %d ", sample_offset);
            for (int s : symbols) std::fputc('0' + s, fbits);
            std::fputc(' ', fbits);
            for (int d : decoded_bits) std::fputc('0' + d, fbits);
            decoder_cont++;
            decoded_bits_stream.insert(decoded_bits_stream.end(), decoded_bits.begin(), decoded_bits.end());
            if (decoder_cont == 15) {
                start_frame_sync(idx, decoded_bits_stream, decoded_bits_stream_state, reg, chars, output,
                                 first_time, window);
                decoder_cont = 0;
                idx = 0;
                decoded_bits_stream.clear();
            }
        }
        std::fputc('\n', fbits);
        block_count++;
    }
    std::fclose(fbits);
    std::fclose(fin);
    std::cerr.rdbuf(old_cerr);
    return 0;
}
