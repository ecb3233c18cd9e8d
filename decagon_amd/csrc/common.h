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

// An opaque copy of each component: the compiler cannot pair operations on them into packed
// fp32 instructions (tests/test_cpu_isa.py bans the op_sel:[0,1] form).
__device__ __forceinline__ void opaque4(float4& v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

// Σ partial[0 .. n) in block order, t = (((0 + p0) + p1) + ...) — the fp32 sum one lane gets
// reading them one by one — computed by one whole wave: lane l loads blocks l, l + 64, l + 128,
// l + 192 of each 256 at once (agent-scope loads: the partials were published from other XCDs),
// then the values are added in order through v_readlane.  One round trip per 256 partials
// instead of one per partial (a serial loop of sc1 loads waits ≈ 1 µs each).  Wave-uniform n.
__device__ __forceinline__ float block_order_sum(const float* partial, int n, int lane) {
    float t = 0.f;
#pragma unroll 1
    for (int b0 = 0; b0 < n; b0 += 4 * kWave) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int b = b0 + kWave * j + lane;
            v[j] = b < n ? __hip_atomic_load(partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (b0 + kWave * j >= n) break;  // wave-uniform
            const int m = n - (b0 + kWave * j) < kWave ? n - (b0 + kWave * j) : kWave;
#pragma unroll
            for (int l = 0; l < kWave; ++l) {
                if (l >= m) break;
                t += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[j]), l));
            }
        }
    }
    return t;
}

// Butterfly steps without an LDS round trip (ds_bpermute) where gfx950 allows: the value of
// lane ^ m from v_permlane32_swap / v_permlane16_swap (m = 32 / 16: lane halves / 16-lane rows
// exchanged between two copies of x) or DPP (m = 8: row_ror:8 within a row; m = 2 / 1:
// quad_perm [2,3,0,1] / [1,0,3,2]); m = 4 stays a ds_bpermute.  Exact partner values, and IEEE
// addition is commutative, so every step is bit for bit x + __shfl_xor(x, m).
template <int CTRL>
__device__ __forceinline__ float dpp_get(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int M>
__device__ __forceinline__ float xor_get(float x) {  // x of lane ^ M
    static_assert(M == 1 || M == 2 || M == 4 || M == 8 || M == 16 || M == 32, "xor_get: lane ^ 2^k");
    const int lane = threadIdx.x & 63;
    if constexpr (M == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        return __uint_as_float(lane < 32 ? r[1] : r[0]);
    } else if constexpr (M == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        return __uint_as_float((lane >> 4) & 1 ? r[0] : r[1]);
    } else if constexpr (M == 8) {
        return dpp_get<0x128>(x);  // row_ror:8
    } else if constexpr (M == 4) {
        return __shfl_xor(x, 4);
    } else if constexpr (M == 2) {
        return dpp_get<0x4E>(x);  // quad_perm [2,3,0,1]
    } else {
        return dpp_get<0xB1>(x);  // quad_perm [1,0,3,2]
    }
}
template <int M>
__device__ __forceinline__ float xor_add(float x) {  // x + x of lane ^ M
    // (own + partner in either order; the opaque copy keeps the compiler from pairing two such
    // adds into v_pk_add_f32 with op_sel:[0,1] — the form tests/test_cpu_isa.py bans)
    if constexpr (M == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        float a = __uint_as_float(r[0]);
        asm volatile("" : "+v"(a));
        return a + __uint_as_float(r[1]);
    } else if constexpr (M == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        float a = __uint_as_float(r[0]);
        asm volatile("" : "+v"(a));
        return a + __uint_as_float(r[1]);
    } else {
        return x + xor_get<M>(x);
    }
}
template <int M>
__device__ __forceinline__ float4 xor_add4(float4 v) {
    return make_float4(xor_add<M>(v.x), xor_add<M>(v.y), xor_add<M>(v.z), xor_add<M>(v.w));
}
// v summed over the butterfly m = M0, 2·M0, ..., 32 (the loop `for (m = M0; m < 64; m <<= 1)
// v += shfl_xor(v, m)`)
template <int M0>
__device__ __forceinline__ float4 xor_sum4_from(float4 v) {
    if constexpr (M0 >= 64) {
        return v;
    } else {
        return xor_sum4_from<M0 * 2>(xor_add4<M0>(v));
    }
}
template <int M0>
__device__ __forceinline__ float xor_sum_from(float v) {
    if constexpr (M0 >= 64) {
        return v;
    } else {
        return xor_sum_from<M0 * 2>(xor_add<M0>(v));
    }
}
// x summed over m = 1, 2, ..., P/2 (the loop `for (m = 1; m < P; m <<= 1) x += shfl_xor(x, m)`)
template <int P, int M = 1>
__device__ __forceinline__ float xor_sum_below(float x) {
    if constexpr (M >= P) {
        return x;
    } else {
        return xor_sum_below<P, M * 2>(xor_add<M>(x));
    }
}

}  // namespace dg
