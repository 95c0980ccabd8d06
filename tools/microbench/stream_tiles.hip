// Read-bandwidth ceiling of the front end's access pattern: nch rows of `stride` bytes, each
// 64-lane workgroup reads one contiguous window of `win` bytes (16 B per lane per load, all loads
// issued before use) at tile offsets advancing by `adv` bytes, and reduces it to one word.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int PER>
__global__ __launch_bounds__(64) void k(const uint4* __restrict__ base, size_t stride16, int tiles, int adv16,
                                        unsigned* out) {
    const int ch = blockIdx.x / tiles, j = blockIdx.x % tiles;
    const uint4* p = base + ch * stride16 + (size_t)j * adv16;
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    u4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) v[i] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p) + threadIdx.x + 64 * i);
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    if (x == 0x12345678u) out[blockIdx.x] = x;
}

int main(int argc, char** argv) {
    const int nch = 1024;
    const size_t stride = 147008, rowb = 147000;
    uint8_t* d;
    hipMalloc(&d, nch * stride * 8 + (1 << 20));
    hipMemset(d, 1, nch * stride * 8);
    unsigned* o;
    hipMalloc(&o, 1 << 24);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, int per, const char* name) {
        const int win = per * 64 * 16, adv = win - 256;
        const int tiles = (int)((rowb - win) / adv) + 1;
        float best = 1e9;
        for (int it = 0; it < 20; it++) {
            const uint8_t* b = d + (size_t)(it % 8) * nch * stride;
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(nch * tiles), dim3(64), 0, 0, (const uint4*)b, stride / 16, tiles, adv / 16, o);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (it > 2 && ms < best) best = ms;
        }
        const double bytes = (double)nch * tiles * win;
        printf("%s win=%d B: %.4f ms, %.0f GB/s (window bytes), %.0f GB/s (row bytes)\n", name, win, best,
               bytes / best / 1e6, (double)nch * rowb / best / 1e6);
    };
    run(k<4>, 4, "per=4 ");
    run(k<8>, 8, "per=8 ");
    run(k<11>, 11, "per=11");
    run(k<16>, 16, "per=16");
    run(k<32>, 32, "per=32");
    return 0;
}
