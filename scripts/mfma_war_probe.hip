// MFMA SrcC write-after-read probe ("The MFMA SrcC hazard").
//
// Config 5's fused kernel, built without the opaque per-half copy, returned wrong half-0
// scores on ~2 % of tiles.  Its disassembly has, in the half-0 accumulator chain,
//     v_mfma_f32_16x16x32_bf16 v[90:93], A, B, v[148:151]   ; SrcC = the previous MFMA's result
//     s_nop 2
//     ds_read_b128 v[148:151], ...                          ; the next A fragment into that SrcC
// i.e. an LDS load overwriting the SrcC registers of an MFMA issued 3 wait states earlier, whose
// SrcC is itself being produced by the MFMA right before it.  This program runs exactly that
// sequence (and controls) under full occupancy and counts results that differ from the exact
// answer.  All-ones bf16 operands make every product exact: one MFMA gives 32 per element, the
// chain of three 96; an LDS value landing in SrcC before the MFMA read it gives 32 + 1e6.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/mfma_war_probe scripts/mfma_war_probe.hip
// Run:   scripts/mfma_war_probe [iters] [blocks]      (one JSON line per variant)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CHAIN2 "v_mfma_f32_16x16x32_bf16 v[100:103], %[a], %[b], 0\n v_mfma_f32_16x16x32_bf16 v[100:103], %[a], %[b], v[100:103]\n"
#define LAST "v_mfma_f32_16x16x32_bf16 v[104:107], %[a], %[b], v[100:103]\n"
#define TAIL "s_waitcnt lgkmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n v_mov_b32 %[r0], v104\n v_mov_b32 %[r1], v105\n v_mov_b32 %[r2], v106\n v_mov_b32 %[r3], v107\n"
#define OPS : [r0] "=v"(r0), [r1] "=v"(r1), [r2] "=v"(r2), [r3] "=v"(r3) : [a] "v"(a), [b] "v"(b), [l] "v"(laddr) \
    : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "memory"

// variant: 0 the failing shape: dependent chain, ds_read into the last MFMA's SrcC 3 wait states later
//          1 as 0 with 7 wait states (s_nop 6)
//          2 as 0 with 16 wait states
//          3 as 0 with the last MFMA's SrcC NOT produced by the MFMA right before it (an older result)
//          4 as 0 with a VALU write (v_mov) instead of the ds_read (what the compiler's rule covers)
//          5 as 0 with a global (vector memory) load instead of the ds_read
template <int V>
__device__ __forceinline__ void seq(bf16x8 a, bf16x8 b, uint32_t laddr, const float* gp, float& r0, float& r1,
                                    float& r2, float& r3) {
    if constexpr (V == 0) asm volatile(CHAIN2 LAST "s_nop 2\n ds_read_b128 v[100:103], %[l]\n" TAIL OPS);
    if constexpr (V == 1) asm volatile(CHAIN2 LAST "s_nop 6\n ds_read_b128 v[100:103], %[l]\n" TAIL OPS);
    if constexpr (V == 2) asm volatile(CHAIN2 LAST "s_nop 7\n s_nop 7\n ds_read_b128 v[100:103], %[l]\n" TAIL OPS);
    if constexpr (V == 3)
        asm volatile(CHAIN2 "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n" LAST "s_nop 2\n ds_read_b128 v[100:103], %[l]\n" TAIL OPS);
    if constexpr (V == 4) asm volatile(CHAIN2 LAST "s_nop 2\n v_mov_b32 v100, 0x49742400\n" TAIL OPS);
    if constexpr (V == 5) {
        asm volatile(CHAIN2 LAST "s_nop 2\n global_load_dwordx4 v[100:103], %[g], off\n s_waitcnt vmcnt(0)\n" TAIL
                     : [r0] "=v"(r0), [r1] "=v"(r1), [r2] "=v"(r2), [r3] "=v"(r3)
                     : [a] "v"(a), [b] "v"(b), [g] "v"(gp)
                     : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "memory");
    }
}

template <int V>
__global__ __launch_bounds__(768) void probe(const float* g, unsigned* bad, int iters, int noise) {
    __shared__ f4 lds[768];
    const int wave = threadIdx.x >> 6;
    lds[threadIdx.x] = f4{1e6f, 1e6f, 1e6f, 1e6f};
    __syncthreads();
    bf16x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (short)0x3f80;  // bf16 1.0
        b[i] = (short)0x3f80;
    }
    if (noise && (wave % 3 == 2)) {
        // noise waves: long dependent MFMA chains on the same SIMDs
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int it = 0; it < 4 * iters; ++it) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
        if (acc[0] == 12345.f) bad[64] = 1;
        return;
    }
    const uint32_t laddr = (uint32_t)(uintptr_t)(lds + threadIdx.x);  // LDS byte address
    const float* gp = g + 4 * (threadIdx.x & 255);
    unsigned nbad = 0;
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        float r0, r1, r2, r3;
        seq<V>(a, b, laddr, gp, r0, r1, r2, r3);
        nbad += (r0 != 96.f) + (r1 != 96.f) + (r2 != 96.f) + (r3 != 96.f);
    }
    if (nbad) atomicAdd(bad + V, nbad);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4096;
    const int blocks = argc > 2 ? atoi(argv[2]) : 1024;
    float* dg;
    unsigned* dbad;
    if (hipMalloc(&dg, 1024 * 4 * 4) != hipSuccess || hipMalloc(&dbad, 128 * 4) != hipSuccess) return 2;
    {
        float h[4096];
        for (int i = 0; i < 4096; ++i) h[i] = 1e6f;
        (void)hipMemcpy(dg, h, sizeof(h), hipMemcpyHostToDevice);
    }
    typedef void (*K)(const float*, unsigned*, int, int);
    const K ks[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>};
    const char* names[] = {"ds_read_into_srcC_3ws", "ds_read_into_srcC_7ws", "ds_read_into_srcC_16ws",
                           "ds_read_into_srcC_3ws_srcC_old", "valu_into_srcC_3ws", "global_load_into_srcC_3ws"};
    for (int noise = 0; noise < 2; ++noise) {
        for (int v = 0; v < 6; ++v) {
            (void)hipMemset(dbad, 0, 128 * 4);
            hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(768), 0, 0, dg, dbad, iters, noise);
            if (hipDeviceSynchronize() != hipSuccess) {
                printf("{\"variant\": \"%s\", \"error\": \"launch\"}\n", names[v]);
                return 3;
            }
            unsigned hb[128];
            (void)hipMemcpy(hb, dbad, 128 * 4, hipMemcpyDeviceToHost);
            const double seqs = (double)blocks * 768 * iters * (noise ? 2.0 / 3.0 : 1.0);
            printf("{\"variant\": \"%s\", \"noise\": %d, \"sequences\": %.0f, \"bad_elements\": %u}\n", names[v], noise,
                   seqs, hb[v]);
            fflush(stdout);
        }
    }
    (void)hipFree(dg);
    (void)hipFree(dbad);
    return 0;
}
