/*
 * sdr_oracle.c -- CPU restatement of the reference FM/RDS DSP hot path (TEST INFRASTRUCTURE).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this file, as the
 * checker / CPU baseline. The shipped product (real-time-sdr_amd/csrc, libsdr_amd.so) never
 * links it. Parity of this restatement is pinned by tests/golden/ (outputs of the unmodified
 * reference sources built by oracle/Makefile into oracle/_ref/).
 *
 * Build: gcc -O2 -ffp-contract=off (no FMA contraction, no fast-math) so every float/double
 * rounding point matches g++ -O3 on x86-64 for the reference (scalar SSE, no FMA).
 * All references are to /root/reference (TheZxc07/real-time-SDR @ 2025-03-21).
 */
#include "sdr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define PI 3.14159265358979323846 /* include/dy4.h:13 */

/* ------------------------------------------------------------------ tap design */

/* impulseResponseLPF, 4-arg form: filter.cpp:13-29 */
void orc_lpf(float Fs, float Fc, unsigned short num_taps, float *h)
{
    float nc = Fc / (Fs / 2.0);                                   /* :18 */
    for (int i = 0; i < num_taps; i++) {
        float v;
        if (i == (num_taps - 1.0) / 2.0) {
            v = nc;                                               /* :23 */
        } else {
            double arg = PI * nc * (i - (num_taps - 1.0) / 2.0);  /* :25 */
            v = nc * sin(arg) / (PI * nc * (i - (num_taps - 1.0) / 2.0));
        }
        v = v * sin(i * PI / ((float)num_taps)) * sin(i * PI / ((float)num_taps)); /* :27 */
        h[i] = v;
    }
}

/* impulseResponseLPF, 5-arg form with integer interpolation gain u: filter.cpp:33-50 */
void orc_lpf_gain(float Fs, float Fc, unsigned short num_taps, int u, float *h)
{
    float nc = Fc / (Fs / 2.0);                                   /* :39 */
    for (int i = 0; i < num_taps; i++) {
        float v;
        if (i == (num_taps - 1.0) / 2.0) {
            v = u * nc;                                           /* :44 (float product) */
        } else {
            float unc = u * nc;                                   /* :46 u*nc is a float product */
            v = unc * sin(PI * nc * (i - (num_taps - 1.0) / 2.0)) / (PI * nc * (i - (num_taps - 1.0) / 2.0));
        }
        v = v * sin(i * PI / ((float)(num_taps))) * sin(i * PI / ((float)(num_taps))); /* :48 */
        h[i] = v;
    }
}

/* impulseResponseBPF: filter.cpp:55-71 (note the integer (num_taps-1)/2 at :66) */
void orc_bpf(float Fs, const float *Fb, unsigned short num_taps, float *h)
{
    float ncenter = ((Fb[1] + Fb[0]) / 2) / (Fs / 2);             /* :59 float */
    float npass = ((Fb[1] - Fb[0])) / (Fs / 2);                   /* :60 float */
    for (int i = 0; i < num_taps; i++) {
        float v;
        if (i == (num_taps - 1.0) / 2.0) {
            v = npass;                                            /* :64 */
        } else {
            int m = i - (num_taps - 1) / 2;                       /* :66 integer */
            v = npass * ((sin(PI * (npass / 2) * m)) / (PI * (npass / 2) * m));
        }
        v = v * cos(i * PI * ncenter);                            /* :68 */
        v = v * sin(i * PI / ((float)num_taps)) * sin(i * PI / ((float)num_taps)); /* :69 */
        h[i] = v;
    }
}

/* impulseResponseAPF: filter.cpp:73-78 */
void orc_apf(float gain, unsigned short num_taps, float *h)
{
    for (int i = 0; i < num_taps; i++) h[i] = 0.0f;
    h[(size_t)((num_taps - 1.0) / 2.0)] = gain;
}

/* impulseResponseRRC: filter.cpp:80-102 */
void orc_rrc(float Fs, unsigned short num_taps, float *h)
{
    float T_symbol = 1 / 2375.0;
    float beta = 0.90;
    float t;
    for (int i = 0; i < num_taps; i++) {
        t = (i - (float)num_taps / 2.0) / Fs;                     /* :90 */
        if (t == 0.0) {
            h[i] = 1.0 + beta * ((4.0 / PI) - 1);                 /* :92 */
        } else if ((t == (-T_symbol / (4.0 * beta))) | (t == (T_symbol / (4.0 * beta)))) {
            h[i] = (beta / sqrt(2.0)) * ((1 - 2.0 / PI) * (sin(PI / (4.0 * beta)))) +
                   ((1 - 2.0 / PI) * (cos(PI / (4 * beta))));     /* :95 */
        } else {
            h[i] = (sin(PI * t * (1 - beta) / T_symbol) + 4.0 * beta * (t / T_symbol) * cos(PI * t * (1 + beta) / T_symbol)) /
                   (PI * t * (1 - (4.0 * beta * t / T_symbol) * (4.0 * beta * t / T_symbol)) / T_symbol); /* :97 */
        }
    }
}

/* ------------------------------------------------------------------ primitives */

/* convolveFIR(y,x,h,state,D): filter.cpp:106-121. Accumulates from 0.0f in ascending k,
 * each term a rounded float product followed by a rounded float add (no FMA). */
void orc_fir_decim(float *y, const float *x, int nx, const float *h, int ntaps,
                   float *state, int nstate, int D)
{
    int ny = nx / D;
    for (int n = 0; n < nx && n / D < ny; n += D) {
        float acc = 0.0f;
        for (int k = 0; k < ntaps; k++) {
            float p = (n - k < 0) ? h[k] * state[n - k + nstate] : h[k] * x[n - k];
            acc = acc + p;
        }
        y[n / D] = acc;
    }
    /* :119 state = last (ntaps-1) inputs; we keep the last nstate (== ntaps-1 here) */
    if (nx >= nstate) {
        memcpy(state, x + nx - nstate, sizeof(float) * (size_t)nstate);
    } else {
        memmove(state, state + nx, sizeof(float) * (size_t)(nstate - nx));
        memcpy(state + nstate - nx, x, sizeof(float) * (size_t)nx);
    }
}

/* convolveFIR(y,x,h,state,U,D): filter.cpp:123-147. Output n uses taps k = phase, phase+U, ...
 * with phase = (n*D) % U and input index (n*D-k)/U; the phase restarts at 0 every block.
 * The reference's state update (:145) reads before x when ntaps-1 > nx (UB); the only state
 * entries ever read are the last <= 100 inputs, which is what nstate keeps here. */
void orc_fir_resample(float *y, const float *x, int nx, const float *h, int ntaps,
                      float *state, int nstate, int U, int D)
{
    int ny = nx * U / D;
    for (int n = 0; n < ny; n++) {
        float acc = 0.0f;
        int phase = (n * D) % U;
        for (int k = phase; k < ntaps; k += U) {
            int xi = (n * D - k) / U;
            float p = (xi < 0) ? h[k] * state[nstate + xi] : h[k] * x[xi];
            acc = acc + p;
        }
        y[n] = acc;
    }
    if (nx >= nstate) {
        memcpy(state, x + nx - nstate, sizeof(float) * (size_t)nstate);
    } else {
        memmove(state, state + nx, sizeof(float) * (size_t)(nstate - nx));
        memcpy(state + nstate - nx, x, sizeof(float) * (size_t)nx);
    }
}

/* fmDemodNoArctan: demod.cpp:3-24. Float numerator, double denominator and division. */
void orc_fm_demod(const float *I, const float *Q, int n, float *prev_I, float *prev_Q, float *out)
{
    float pI = *prev_I, pQ = *prev_Q;
    for (int i = 0; i < n; i++) {
        float ci = I[i], cq = Q[i];
        if ((ci == 0) & (cq == 0)) {
            out[i] = 0;
        } else {
            float num = ci * (cq - pQ) - cq * (ci - pI);
            double den = (double)ci * (double)ci + (double)cq * (double)cq; /* pow(x,2.0) -> mulsd */
            out[i] = (float)((double)num / den);
        }
        pI = ci;
        pQ = cq;
    }
    *prev_I = I[n - 1];
    *prev_Q = Q[n - 1];
}

/* fmpll: pll.cpp:4-61 */
void orc_fmpll(const float *in, int n, float freq, float Fs, float *out, orc_pll_state *st,
               float ncoScale, float phaseAdjust, float normBandwidth)
{
    float Cp = 2.666;
    float Ci = 3.555;
    float Kp = normBandwidth * Cp;
    float Ki = normBandwidth * normBandwidth * Ci;
    out[0] = out[n];                                              /* :18 */
    float trigArg;
    float errorI, errorQ, errorD;
    for (int i = 0; i < n; i++) {
        errorI = in[i] * (st->feedbackI);                         /* :36 */
        errorQ = in[i] * (-st->feedbackQ);                        /* :37 */
        errorD = atan2(errorQ, errorI);                           /* :39 double atan2 */
        st->integrator = st->integrator + Ki * errorD;            /* :41 */
        st->phaseEst = st->phaseEst + Kp * errorD + st->integrator; /* :42 */
        st->trigOffset += 1.0;                                    /* :46 */
        trigArg = 2 * PI * (freq / Fs) * (st->trigOffset) + st->phaseEst; /* :47 */
        st->feedbackI = cos(trigArg);                             /* :49 */
        st->feedbackQ = sin(trigArg);                             /* :50 */
        out[i + 1] = cos(trigArg * ncoScale + phaseAdjust);       /* :52 */
    }
    st->lastCarrier = out[n];                                     /* :58 */
}

/* cdr: rds_utilities.cpp:4-21 (abs of a float argument resolves to int abs: truncation) */
int orc_cdr(int sps, const float *x, int n)
{
    int maxi = 0, maxv = 0, sum = 0;
    for (int i = 0; i < sps; i++) {
        for (int k = 0; k < n / sps; k++) sum += abs((int)x[k * sps + i]);
        if (sum > maxv) {
            maxv = sum;
            maxi = i;
        }
        sum = 0;
    }
    return maxi;
}

/* symbol slicer: rds.cpp:157-161 */
int orc_slice(const float *x, int n, int offset, int sps, int *symbols)
{
    int m = 0;
    for (int i = 0; offset + i * sps < n; i++) symbols[m++] = x[offset + i * sps] > 0;
    return m;
}

/* manchester_decode: rds_utilities.cpp:34-68 */
int orc_manchester(int *bits, const int *symbols, int nsym, int block_count, int *half_symbol, int *start)
{
    int nb = 0;
    if (*start) bits[nb++] = *half_symbol;                        /* :38-40 */
    if (block_count == 0) {                                       /* :42-51 */
        int score = 0;
        for (int i = 0; i < nsym - 1; i += 2) score += symbols[i] ^ symbols[i + 1];
        for (int j = 1; j < nsym - 1; j += 2) score -= symbols[j] ^ symbols[j + 1];
        *start = score < 0;
    }
    for (int i = *start; i < nsym - 1; i += 2) bits[nb++] = symbols[i]; /* :55-59 */
    if (((nsym - *start) & 0x01) == 1) {                          /* :61-67 */
        *half_symbol = symbols[nsym - 1];
        *start = 1;
    } else {
        *start = 0;
    }
    return nb;
}

/* differential_decode: rds_utilities.cpp:70-88 */
void orc_differential(int *out, const int *bits, int nbits, int *last_bit, int block_num)
{
    if (nbits <= 0) return;
    out[0] = (block_num == 0) ? bits[0] : (bits[0] ^ *last_bit);
    for (int i = 1; i < nbits; i++) out[i] = bits[i] ^ bits[i - 1];
    *last_bit = bits[nbits - 1];
}

int16_t orc_f32_to_i16(float v)
{
    int32_t i;
    if (v >= -2147483648.0f && v < 2147483648.0f)
        i = (int32_t)v;
    else
        i = INT32_MIN;
    return (int16_t)(uint16_t)((uint32_t)i & 0xFFFFu);
}

/* ------------------------------------------------------------------ stages */

static float *fz(size_t n) { return (float *)calloc(n ? n : 1, sizeof(float)); }

int orc_chan_init(orc_chan *c, int mode, int rds_on)
{
    memset(c, 0, sizeof(*c));
    /* defaults: project.cpp:31-44 */
    c->rf_Fs = 2400000; c->rf_Fc = 100000; c->rf_taps = 101; c->rf_decim = 10;
    c->audio_decim = 5; c->audio_upsample = 1; c->if_Fs = 240000; c->audio_Fc = 16000;
    c->symbol_Fs = 39; c->rds_on = rds_on;
    switch (mode) {                                               /* project.cpp:67-108 */
    case 0: c->rf_Fs = 2400000; c->rf_decim = 10; c->audio_decim = 5; c->if_Fs = 240000; break;
    case 1: c->rf_Fs = 1440000; c->rf_decim = 4; c->audio_decim = 9; c->if_Fs = 360000; break;
    case 2: c->rf_Fs = 2400000; c->rf_decim = 10; c->audio_decim = 800; c->if_Fs = 240000;
            c->audio_upsample = 147; c->symbol_Fs = 20; break;
    case 3: c->rf_Fs = 1152000; c->rf_decim = 3; c->audio_decim = 1280; c->if_Fs = 384000;
            c->audio_upsample = 147; c->symbol_Fs = 20; break;
    default: return -1;
    }
    int U = c->audio_upsample, D = c->audio_decim, T = c->rf_taps;
    c->block_iq = (1470 * c->rf_decim * D) / U;                   /* rffrontend.cpp:21 */
    c->block_if = (1470 * D) / U;                                 /* mono.cpp:17 */
    c->n_audio = c->block_if * U / D;
    c->n_rds = c->block_if * 247 / 640;
    c->audio_ntaps = T * U;
    c->rds_bb_ntaps = T * 247;

    c->rf_h = fz(T); c->audio_h = fz(c->audio_ntaps); c->pilot_h = fz(T); c->stereo_h = fz(T);
    c->apf_h = fz(T); c->rds_h = fz(T); c->rds_sq_h = fz(T); c->rds_bb_h = fz(c->rds_bb_ntaps);
    c->rrc_h = fz(T);
    orc_lpf((float)c->rf_Fs, (float)c->rf_Fc, (unsigned short)T, c->rf_h);            /* rffrontend.cpp:24 */
    orc_lpf_gain((float)(c->if_Fs * U), (float)c->audio_Fc, (unsigned short)(T * U), U, c->audio_h); /* mono.cpp:22 */
    float fb_pilot[2] = {18.5e3f, 19.5e3f}, fb_stereo[2] = {22e3f, 54e3f};            /* stereo.cpp:59-61 */
    orc_bpf((float)(c->rf_Fs / c->rf_decim), fb_pilot, (unsigned short)T, c->pilot_h);  /* stereo.cpp:65 */
    orc_bpf((float)(c->rf_Fs / c->rf_decim), fb_stereo, (unsigned short)T, c->stereo_h);/* stereo.cpp:67 */
    orc_apf(1, (unsigned short)T, c->apf_h);                                           /* stereo.cpp:63 */
    float fb_rds[2] = {54e3f, 60e3f}, fb_rds_sq[2] = {113.5e3f, 114.5e3f};            /* rds.cpp:58-59 */
    orc_lpf_gain((float)(c->if_Fs * 247), 3e3f, (unsigned short)(T * 247), 247, c->rds_bb_h); /* rds.cpp:61 */
    orc_bpf((float)c->if_Fs, fb_rds, (unsigned short)T, c->rds_h);                   /* rds.cpp:62 */
    orc_bpf((float)c->if_Fs, fb_rds_sq, (unsigned short)T, c->rds_sq_h);             /* rds.cpp:63 */
    orc_rrc((float)(2375 * c->symbol_Fs), (unsigned short)T, c->rrc_h);              /* rds.cpp:65 */

    int S = T - 1;
    c->state_I = fz(S); c->state_Q = fz(S);
    c->mono_state = fz(S);
    c->pilot_state = fz(S); c->band_state = fz(S); c->mdelay_state = fz(S);
    c->mfilt_state = fz(S); c->sfilt_state = fz(S);
    c->carrier = fz(c->block_if + 1);
    c->carrier[c->block_if] = 1.0f;                               /* stereo.cpp:45 */
    c->st_pll.feedbackI = 1.0f; c->st_pll.lastCarrier = 1.0f;    /* stereo.cpp:51-57 */
    c->rband_state = fz(S); c->rsq_state = fz(S); c->rdelay_state = fz(S);
    c->rfilt_state = fz(S); c->rclean_state = fz(S);
    c->ipll = fz(c->block_if + 1);
    c->ipll[c->block_if] = 1.0f;                                  /* rds.cpp:38 */
    c->rds_pll.feedbackI = 1.0f;                                  /* rds.cpp:52-56 */

    size_t nb = (size_t)c->block_iq;
    c->I = fz(nb); c->Q = fz(nb); c->Ids = fz(c->block_if); c->Qds = fz(c->block_if);
    c->t0 = fz(c->block_if); c->t1 = fz(c->block_if); c->t2 = fz(c->block_if);
    c->t3 = fz(c->block_if); c->t4 = fz(c->block_if); c->t5 = fz(c->block_if);
    return 0;
}

void orc_chan_free(orc_chan *c)
{
    float **p[] = {&c->rf_h, &c->audio_h, &c->pilot_h, &c->stereo_h, &c->apf_h, &c->rds_h, &c->rds_sq_h,
                   &c->rds_bb_h, &c->rrc_h, &c->state_I, &c->state_Q, &c->mono_state, &c->pilot_state,
                   &c->band_state, &c->mdelay_state, &c->mfilt_state, &c->sfilt_state, &c->carrier,
                   &c->rband_state, &c->rsq_state, &c->rdelay_state, &c->rfilt_state, &c->rclean_state,
                   &c->ipll, &c->I, &c->Q, &c->Ids, &c->Qds, &c->t0, &c->t1, &c->t2, &c->t3, &c->t4, &c->t5};
    for (size_t i = 0; i < sizeof(p) / sizeof(p[0]); i++) {
        free(*p[i]);
        *p[i] = NULL;
    }
}

/* RF_frontend loop body: rffrontend.cpp:58-71 */
void orc_frontend_block(orc_chan *c, const uint8_t *iq, float *fm_demod)
{
    int n = c->block_iq, S = c->rf_taps - 1;
    for (int s = 0; s < 2 * n; s++) {                             /* :58-63 */
        float v = (float)(((unsigned char)iq[s] - 128.0) / 128.0);
        if (s & 1) c->Q[s >> 1] = v; else c->I[s >> 1] = v;
    }
    orc_fir_decim(c->Ids, c->I, n, c->rf_h, c->rf_taps, c->state_I, S, c->rf_decim); /* :67 */
    orc_fir_decim(c->Qds, c->Q, n, c->rf_h, c->rf_taps, c->state_Q, S, c->rf_decim); /* :68 */
    orc_fm_demod(c->Ids, c->Qds, c->block_if, &c->prev_I, &c->prev_Q, fm_demod);     /* :71 */
}

/* mono loop body: mono.cpp:34-42 */
void orc_mono_block(orc_chan *c, const float *fm_demod, int16_t *audio)
{
    float *filt = c->t0;
    orc_fir_resample(filt, fm_demod, c->block_if, c->audio_h, c->audio_ntaps, c->mono_state,
                     c->rf_taps - 1, c->audio_upsample, c->audio_decim);
    for (int i = 0; i < c->n_audio; i++) audio[i] = orc_f32_to_i16(16384 * filt[i]);
}

/* stereo loop body: stereo.cpp:74-107 */
void orc_stereo_block(orc_chan *c, const float *fm_demod, int16_t *lr,
                      float *pilot_o, float *carrier_o, float *band_o, float *sdc_o, float *mdelay_o)
{
    int n = c->block_if, S = c->rf_taps - 1, T = c->rf_taps;
    float *pilot = c->t0, *band = c->t1, *sdc = c->t2, *mdelay = c->t3, *mfilt = c->t4, *sfilt = c->t5;
    orc_fir_decim(pilot, fm_demod, n, c->pilot_h, T, c->pilot_state, S, 1);           /* :74 */
    orc_fmpll(pilot, n, 19e3f, (float)(c->rf_Fs / c->rf_decim), c->carrier, &c->st_pll, 2.0f, 0.0f, 0.01f); /* :77 */
    orc_fir_decim(band, fm_demod, n, c->stereo_h, T, c->band_state, S, 1);            /* :80 */
    for (int i = 0; i < n; i++) sdc[i] = (float)(2.0 * band[i] * c->carrier[i]);      /* :83-85 */
    orc_fir_decim(mdelay, fm_demod, n, c->apf_h, T, c->mdelay_state, S, 1);           /* :88 */
    if (pilot_o) memcpy(pilot_o, pilot, sizeof(float) * n);
    if (carrier_o) memcpy(carrier_o, c->carrier, sizeof(float) * (n + 1));
    if (band_o) memcpy(band_o, band, sizeof(float) * n);
    if (sdc_o) memcpy(sdc_o, sdc, sizeof(float) * n);
    if (mdelay_o) memcpy(mdelay_o, mdelay, sizeof(float) * n);
    orc_fir_resample(mfilt, mdelay, n, c->audio_h, c->audio_ntaps, c->mfilt_state, S, c->audio_upsample, c->audio_decim); /* :94 */
    orc_fir_resample(sfilt, sdc, n, c->audio_h, c->audio_ntaps, c->sfilt_state, S, c->audio_upsample, c->audio_decim);    /* :97 */
    for (int s = 0; s < 2 * c->n_audio; s++) {                    /* :100-107 */
        int16_t right = orc_f32_to_i16(16384 * (mfilt[s >> 1] - sfilt[s >> 1]));
        int16_t left = orc_f32_to_i16(16384 * (mfilt[s >> 1] + sfilt[s >> 1]));
        lr[s] = (s & 1) ? right : left;
    }
}

/* rds loop body: rds.cpp:105-182 (frame sync / parse excluded: SURVEY 8(f) f1) */
int orc_rds_block(orc_chan *c, const float *fm_demod, float *rds_clean, int *offset,
                  int *symbols, int *nsym, int *decoded_bits,
                  float *rband_o, float *gpilot_o, float *ipll_o, float *rdc_o, float *rfilt_o)
{
    int n = c->block_if, S = c->rf_taps - 1, T = c->rf_taps;
    float *rband = c->t0, *sq = c->t1, *gpilot = c->t2, *rdelay = c->t3, *rdc = c->t4, *rfilt = c->t5;
    orc_fir_decim(rband, fm_demod, n, c->rds_h, T, c->rband_state, S, 1);             /* :105 */
    for (int i = 0; i < n; i++) sq[i] = rband[i] * rband[i];                         /* :111-113 */
    orc_fir_decim(gpilot, sq, n, c->rds_sq_h, T, c->rsq_state, S, 1);                /* :116 */
    orc_fmpll(gpilot, n, 114e3f, (float)c->if_Fs, c->ipll, &c->rds_pll, 0.5f, 0.0f, 0.001f); /* :119 */
    orc_fir_decim(rdelay, rband, n, c->apf_h, T, c->rdelay_state, S, 1);             /* :122 */
    for (int i = 0; i < n; i++) rdc[i] = 2 * rdelay[i] * c->ipll[i];                 /* :125-127 */
    if (rband_o) memcpy(rband_o, rband, sizeof(float) * n);
    if (gpilot_o) memcpy(gpilot_o, gpilot, sizeof(float) * n);
    if (ipll_o) memcpy(ipll_o, c->ipll, sizeof(float) * (n + 1));
    if (rdc_o) memcpy(rdc_o, rdc, sizeof(float) * n);
    orc_fir_resample(rfilt, rdc, n, c->rds_bb_h, c->rds_bb_ntaps, c->rfilt_state, S, 247, 640); /* :130 */
    if (rfilt_o) memcpy(rfilt_o, rfilt, sizeof(float) * c->n_rds);
    /* RRC (:133): rds_clean_state is a 100-sample FIR state over the 2836-sample stream */
    orc_fir_decim(rds_clean, rfilt, c->n_rds, c->rrc_h, T, c->rclean_state, S, 1);
    int ret = -1;
    if (c->rds_block_count > 5 && c->rds_on) {                   /* :135 */
        c->sample_offset = orc_cdr(c->symbol_Fs, rds_clean, c->n_rds);                  /* :137 */
        int m = orc_slice(rds_clean, c->n_rds, c->sample_offset, c->symbol_Fs, symbols); /* :157-161 */
        int bits[512];
        int nb = orc_manchester(bits, symbols, m, c->rds_block_count, &c->half_symbol, &c->start); /* :164 */
        orc_differential(decoded_bits, bits, nb, &c->last_bit, c->rds_block_count);     /* :167 */
        if (nsym) *nsym = m;
        ret = nb;
    }
    if (offset) *offset = c->sample_offset;
    c->rds_block_count++;                                         /* :191 */
    return ret;
}
