// Shared helpers for the gfx950 kernels of libdecagon_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "decagon_hip.h"

namespace dg {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Map a launch status to the ABI's return convention (0 or a positive hipError_t).
inline int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? DG_OK : static_cast<int>(e);
}

// The one piece of process state the library keeps: per kernel, the set of devices on which
// its dynamic-LDS opt-in (hipFuncSetAttribute, idempotent) has been applied — one bit per
// device id, so every device a process launches on is configured, and concurrent callers at
// worst set the attribute twice.
inline void lds_optin(const void* fn, int bytes, std::atomic<uint64_t>& done) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
        (void)hipGetLastError();  // not sticky: the launch after it reports its own status
        return;                   // (and a launch that needs the opt-in fails loudly)
    }
    done.fetch_or(bit, std::memory_order_acq_rel);
}

// Lanes that cooperate on one dense row of width d (d/4 float4 lanes, rounded up to a
// power of two so that a wave holds 64/LP rows or nonzeros side by side).
inline int lanes_per_row(int d) {
    int need = (d + 3) / 4;
    int lp = 1;
    while (lp < need) lp <<= 1;
    return lp;
}

__device__ __forceinline__ void fma4(float4& acc, float s, const float4& x) {
    acc.x = fmaf(s, x.x, acc.x);
    acc.y = fmaf(s, x.y, acc.y);
    acc.z = fmaf(s, x.z, acc.z);
    acc.w = fmaf(s, x.w, acc.w);
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
}

__device__ __forceinline__ float4 shfl4(const float4& v, int src) {
    return make_float4(__shfl(v.x, src), __shfl(v.y, src), __shfl(v.z, src), __shfl(v.w, src));
}

__device__ __forceinline__ float4 shfl_xor4(const float4& v, int m) {
    return make_float4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m),
                       __shfl_xor(v.w, m));
}

}  // namespace dg
