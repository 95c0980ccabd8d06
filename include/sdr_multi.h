/* sdr_multi.h -- the multi-channel receiver engine: the reference program's three stage threads
 * (/root/reference/src/project.cpp:134-136: RF front end, audio, RDS) over nch channels at once,
 * joined by the reference's queue protocol (ThreadSafeQueue push / wait_and_pop / prepare,
 * /root/reference/include/threadsafequeue.h:24-74) carrying device-resident fm_demod batches
 * (include/dropin/fm_batch.h), on the C ABI of libsdr_amd.so. Implemented in
 * real-time-sdr_amd/host/sdr_multi_engine.cpp (libsdr_host.so); the CLI real-time-sdr_amd/bin/sdr_multi
 * and bench.py's queue_plumbed leg call it.
 *
 * Input is either a byte stream (a file, or "-" for stdin: u8 I/Q, block after block, each block nch
 * rows of 2*block_iq bytes), uploaded through a pinned ring, or blocks already resident on the
 * device ([nblocks][nch] rows, row_stride bytes apart, block_stride bytes between blocks). Outputs:
 * PREFIX.pcm (per block nch rows of 2*n_audio int16, L/R interleaved, stereo.cpp:100-111) and
 * PREFIX.rds (each channel's RDS text, "ch <c>: " + parse()'s lines, rds_utilities.cpp:172-199),
 * and/or captured rows of a few channels for a checker. */
#ifndef SDR_MULTI_H
#define SDR_MULTI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sdr_multi_opts {
    int nch, mode, flags, device;
    /* CUs [0, pll_cus) carry the two consumers' PLLs (stereo on the first half, RDS on the second,
     * one persistent launch each, sdr_plls_launch_sel) and every other stream runs on the rest;
     * 0: no CU masks and per-block PLL dispatches. A byte stream of unknown length (a pipe) also
     * uses per-block dispatches (a persistent launch must know its block count). */
    int pll_cus;
    const char *in_path;          /* input file or "-"; NULL: device input below */
    const uint8_t *d_iq;          /* device input: block b, channel c at d_iq + b*block_stride + c*row_stride */
    size_t row_stride, block_stride;
    int nblocks;                  /* blocks of the device input */
    const char *out_prefix;       /* PREFIX.pcm and PREFIX.rds; NULL: no files */
    /* optional captures for a checker (NULL: none), channel cap_ch[i] of every block b:
     * cap_lr[(b*ncap + i)*2*n_audio ..], cap_nbits[b*ncap + i] (-1: no RDS bits this block),
     * cap_bits[(b*ncap + i)*SDR_MAX_BITS ..]; room for cap_blocks blocks */
    int ncap, cap_blocks;
    const int *cap_ch;
    int16_t *cap_lr;
    int32_t *cap_nbits;
    uint8_t *cap_bits;
    /* optional (NULL: none), persistent mode: each consumer's PLL end stamp of every block (100 MHz
     * device clock), audio's at pll_end[b], RDS's at pll_end[stamp_blocks + b], b < stamp_blocks */
    int stamp_blocks;
    unsigned long long *pll_end;
} sdr_multi_opts;

typedef struct sdr_multi_stats {
    long long blocks;             /* blocks processed */
    double seconds;               /* wall time from the first block's input to the last outputs on the host */
    double steady_seconds;        /* the same from block 1's front end on (block 0's fill excluded) */
    double pll_period_ms;         /* persistent mode: device-clock period per block of the slower
                                     consumer's PLL launch, blocks 1 .. last (0 in dispatch mode) */
    double pll_span_ms;           /* persistent mode: block 0's PLL start to the last block's end */
    double read_s, h2d_ms, d2h_ms;   /* byte-stream input: read time, GPU time of the uploads; L/R D2H */
    int persistent;               /* 1: persistent PLL launches, 0: per-block dispatches */
} sdr_multi_stats;

/* Runs the receiver to the end of the input and returns 0; SDR_E_INVALID for invalid options (nothing
 * started). Once its threads run, a failure -- an unreadable input or output file, a library or HIP
 * runtime error, a persistent PLL launch that timed out -- prints "sdr: <what>" on stderr and ends the
 * process with exit(1), as the reference program does (rffrontend.cpp:50-52, utilities.h:7-10): the
 * three stage threads cannot be unwound from each other's queue waits. The run's contexts, CU-masked
 * streams and pinned output buffers are kept for the process's later runs (a run reuses idle ones of
 * the same shape, contexts through sdr_ctx_reset; SDR_MULTI_CTX_CACHE=0 / SDR_MULTI_STREAM_CACHE=0 /
 * SDR_MULTI_PIN_CACHE=0: made and freed per run). */
int sdr_multi_run(const sdr_multi_opts *opts, sdr_multi_stats *stats);

#ifdef __cplusplus
}
#endif

#endif
