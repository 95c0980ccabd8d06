// rffrontend.h (drop-in) -- stage thread entry point of the reference (include/rffrontend.h), running its per-block
// DSP on the MI355X kernels of libsdr_amd.so.
#ifndef SDR_DROPIN_RFFRONTEND_H
#define SDR_DROPIN_RFFRONTEND_H

#include <iostream>
#include <vector>

#include "args.h"

void RF_frontend(args *p);

#endif
