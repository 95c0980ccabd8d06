// args.h (drop-in) -- the stage-thread argument block of the reference (include/args.h:6-19); same
// leading fields in the same order, so `args a = {queue, 2400000, 100000, 101, ...}` initialises it
// unchanged. Trailing fields (defaulted) select the GPU.
#ifndef SDR_DROPIN_ARGS_H
#define SDR_DROPIN_ARGS_H

#include <vector>

#include "threadsafequeue.h"

struct args {
    ThreadSafeQueue<std::vector<float> *> &queue;
    int rf_Fs;
    int rf_Fc;
    unsigned short int rf_taps;
    int rf_decim;
    float audio_decim;
    float audio_upsample;
    int if_Fs;
    int audio_Fc;
    int audio_Fs;
    int symbol_Fs;
    bool rds_on;
    int device = 0;   // HIP device the stage contexts run on
};

#endif
