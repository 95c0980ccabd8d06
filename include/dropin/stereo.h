// stereo.h (drop-in) -- stage thread entry point of the reference (include/stereo.h), running its per-block
// DSP on the MI355X kernels of libsdr_amd.so.
#ifndef SDR_DROPIN_STEREO_H
#define SDR_DROPIN_STEREO_H

#include <iostream>
#include <vector>

#include "args.h"

void stereo(args *p);

#endif
