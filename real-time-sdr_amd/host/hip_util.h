// hip_util.h -- small host helpers for the drop-in layer: error checks, growable device buffers
// and a per-thread HIP stream. Host code only (compiled with g++ against the HIP runtime).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "sdr_amd.h"

namespace sdrhost {

[[noreturn]] inline void die(const std::string& what) {
    std::fprintf(stderr, "sdr: %s\n", what.c_str());
    std::exit(1);   // the reference's failure behaviour (rffrontend.cpp:50-52, utilities.h:7-10)
}

inline void check_sdr(int rc, const char* what) {
    if (rc != SDR_OK) die(std::string(what) + ": " + sdr_last_error());
}

inline void check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) die(std::string(what) + ": " + hipGetErrorString(e));
}

// device buffer that only grows
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    T* get(size_t count) {
        if (count > n) {
            if (p) (void)hipFree(p);
            check_hip(hipMalloc(reinterpret_cast<void**>(&p), (count ? count : 1) * sizeof(T)), "hipMalloc");
            n = count;
        }
        return p;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// one non-blocking stream per host thread (the stage threads run concurrently, like the reference)
inline hipStream_t thread_stream() {
    thread_local struct S {
        hipStream_t s = nullptr;
        S() { check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate"); }
        ~S() {
            // sdr_stream_destroy also frees the per-stream sdr_fmpll scratch cached for this handle
            if (s) (void)sdr_stream_destroy(s);
        }
    } st;
    return st.s;
}

}  // namespace sdrhost
