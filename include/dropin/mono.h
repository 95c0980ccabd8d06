// mono.h (drop-in) -- stage thread entry point of the reference (include/mono.h), running its per-block
// DSP on the MI355X kernels of libsdr_amd.so.
#ifndef SDR_DROPIN_MONO_H
#define SDR_DROPIN_MONO_H

#include <iostream>
#include <vector>

#include "args.h"

void mono(args *p);

#endif
