// ref_newpad.cpp -- link-time allocation shim for building the UNMODIFIED reference sources.
// TEST INFRASTRUCTURE ONLY (oracle/_ref build, see oracle/Makefile).
//
// The reference's resampler state update `std::vector<float>(x.end()-h.size()+1, x.end())`
// (src/filter.cpp:145, called from src/rds.cpp:130 with len(h)=24947 > len(x)=7350) reads up to
// ~70 KB before x's first element (ASan: heap-buffer-overflow). The entries it copies
// from there are never read again (only the last 100 state entries are, filter.cpp:135), so all the
// shim must guarantee is that those bytes are mapped: every C++ allocation gets PAD bytes of slack
// in front of the pointer handed out. No reference source is changed.
#include <cstdlib>
#include <cstring>
#include <malloc.h>
#include <new>

namespace {
constexpr std::size_t PAD = 256 * 1024;

struct MallocTune {
    // keep the padded blocks on the heap (no mmap per allocation) so timing stays representative
    MallocTune() { mallopt(M_MMAP_THRESHOLD, 256 * 1024 * 1024); mallopt(M_TRIM_THRESHOLD, 512 * 1024 * 1024); }
} g_tune;

void* pad_alloc(std::size_t n) {
    char* p = static_cast<char*>(std::malloc(n + PAD));
    if (!p) throw std::bad_alloc();
    return p + PAD;
}
void pad_free(void* p) noexcept {
    if (p) std::free(static_cast<char*>(p) - PAD);
}
}  // namespace

void* operator new(std::size_t n) { return pad_alloc(n); }
void* operator new[](std::size_t n) { return pad_alloc(n); }
void* operator new(std::size_t n, const std::nothrow_t&) noexcept {
    try { return pad_alloc(n); } catch (...) { return nullptr; }
}
void* operator new[](std::size_t n, const std::nothrow_t&) noexcept {
    try { return pad_alloc(n); } catch (...) { return nullptr; }
}
void operator delete(void* p) noexcept { pad_free(p); }
void operator delete[](void* p) noexcept { pad_free(p); }
void operator delete(void* p, std::size_t) noexcept { pad_free(p); }
void operator delete[](void* p, std::size_t) noexcept { pad_free(p); }
