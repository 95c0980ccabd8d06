// rds.h (drop-in) -- stage thread entry point of the reference (include/rds.h), running its per-block
// DSP on the MI355X kernels of libsdr_amd.so.
#ifndef SDR_DROPIN_RDS_H
#define SDR_DROPIN_RDS_H

#include <iostream>
#include <vector>

#include "args.h"

void rds(args *p);

#endif
