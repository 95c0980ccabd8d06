// Microbenchmark: f32 VALU issue rate of scalar vs packed mul/add (no contraction),
// and the per-step latency of a serial PLL-like chain using f64 libm (OCML) calls.
// Used once to size the exact-mode FIR and the PLL kernel; not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

#pragma clang fp contract(off)

typedef float f2 __attribute__((ext_vector_type(2)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int ITERS>
__global__ void __launch_bounds__(256) scalar_muladd(float* out, float a, float b) {
  float acc[8];
  float x = threadIdx.x * 1e-3f;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      float p = acc[i] * a;
      acc[i] = p + b;
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ITERS>
__global__ void __launch_bounds__(256) packed_muladd(float* out, float a, float b) {
  f2 acc[8];
  float x = threadIdx.x * 1e-3f;
#pragma unroll
  for (int i = 0; i < 8; i++) { acc[i].x = x + i; acc[i].y = x - i; }
  f2 va = {a, a}, vb = {b, b};
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      f2 p = acc[i] * va;
      acc[i] = p + vb;
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Serial PLL-like chain per lane with double atan2 / sin / cos (OCML), like pll.cpp:34-53.
__global__ void pll_chain(float* out, const float* in, int nsteps) {
  float fbI = 1.f, fbQ = 0.f, integ = 0.f, ph = 0.f;
  double toff = 0.0;
  const float Kp = 0.01f * 2.666f, Ki = 0.01f * 0.01f * 3.555f;
  float acc = 0.f;
  int lane = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < nsteps; i++) {
    float x = in[(i & 1023)];
    float eI = x * fbI;
    float eQ = x * (-fbQ);
    float e = (float)atan2((double)eQ, (double)eI);
    integ = integ + Ki * e;
    ph = ph + Kp * e + integ;
    toff += 1.0;
    float t = (float)(2 * M_PI * (double)(19000.f / 240000.f) * toff + (double)ph);
    double s, c;
    sincos((double)t, &s, &c);
    fbI = (float)c;
    fbQ = (float)s;
    acc += (float)cos((double)(t * 2.0f));
  }
  out[lane] = acc + fbI;
}

int main() {
  float* d_out; float* d_in;
  const int nblk = 256 * 8 * 4, nthr = 256;
  CHECK(hipMalloc(&d_out, sizeof(float) * nblk * nthr));
  CHECK(hipMalloc(&d_in, sizeof(float) * 1024));
  float h_in[1024];
  for (int i = 0; i < 1024; i++) h_in[i] = (float)std::cos(2 * M_PI * 19000.0 / 240000.0 * i) * 0.1f;
  CHECK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int IT = 4096;
  for (int rep = 0; rep < 3; rep++) {
    float ms;
    hipLaunchKernelGGL(scalar_muladd<IT>, dim3(nblk), dim3(nthr), 0, 0, d_out, 0.999f, 1e-4f);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(scalar_muladd<IT>, dim3(nblk), dim3(nthr), 0, 0, d_out, 0.999f, 1e-4f);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    double ops = (double)nblk * nthr * IT * 8 * 2;  // lane-ops (mul + add)
    printf("scalar mul+add: %.3f ms, %.2f T lane-op/s\n", ms, ops / (ms * 1e-3) / 1e12);
    hipLaunchKernelGGL(packed_muladd<IT>, dim3(nblk), dim3(nthr), 0, 0, d_out, 0.999f, 1e-4f);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(packed_muladd<IT>, dim3(nblk), dim3(nthr), 0, 0, d_out, 0.999f, 1e-4f);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ops = (double)nblk * nthr * IT * 8 * 2 * 2;  // element-ops (2 per packed lane-op)
    printf("packed mul+add: %.3f ms, %.2f T element-op/s\n", ms, ops / (ms * 1e-3) / 1e12);
  }
  for (int waves : {1, 32, 1024, 4096}) {
    const int steps = 7350;
    float ms;
    hipLaunchKernelGGL(pll_chain, dim3(waves), dim3(64), 0, 0, d_out, d_in, 100);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(pll_chain, dim3(waves), dim3(64), 0, 0, d_out, d_in, steps);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("pll_chain f64 libm: %d waves x 64 lanes, %d steps: %.3f ms = %.1f ns/step\n", waves, steps, ms, ms * 1e6 / steps);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
