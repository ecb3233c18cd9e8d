// Packed-f32 forwarding probe ("The packed-f32 forwarding hazard").
//
// Config 5's fused kernel, built without the opaque per-half copy, returned a wrong low-half
// sum on ~2 % of tiles; its epilogue ran `v_mov_b32 vN, vM` immediately followed by a
// `v_pk_fma_f32 ..., v[N:N+1], ...` whose high half vN+1 was an MFMA result.  This program runs
// that two-instruction sequence and controlled variants of it, millions of times under full
// occupancy, and counts results that differ bit for bit from the expected fmaf.  It touches
// registers and vector memory only.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/pk_probe scripts/pk_probe.hip
// Run:   scripts/pk_probe [iters] [blocks]      (one JSON line per variant)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

#define MFMA_HI "v_mfma_f32_16x16x32_bf16 v[100:103], %[a], %[b8], 0\n s_nop 7\n s_nop 7\n s_nop 7\n"
#define VALU_HI "v_mov_b32 v103, %[y]\n s_nop 7\n s_nop 7\n"
#define OUT "v_mov_b32 %[r0], v104\n v_mov_b32 %[r1], v105\n v_mov_b32 %[m], v103\n"
#define CLOB "v100", "v101", "v102", "v103", "v104", "v105", "v108", "v109", "v110", "v111"

// variant: 0 the failing shape (MFMA-written hi, v_mov lo, src0, adjacent)
//          1 as 0 with one independent instruction (s_nop 0) between the v_mov and the v_pk_fma
//          2 as 0 with the high half written by a VALU instead of an MFMA
//          3 as 0 with the low half written by v_lshlrev_b32 instead of v_mov_b32
//          4 as 0 with the pair read as src1 instead of src0
//          5 as 0 with the v_pk_fma writing the register the v_mov read (index 1338's form)
//          6 as 0 with an independent MFMA issued right before the v_mov (in flight)
//          7 as 0 with v_pk_mul_f32 (no addend)
//          8 as 0 with the pair's low half broadcast (op_sel_hi:[0,1,1], colshared's form)
template <int V>
__device__ __forceinline__ void seq(float x, float y, f2 bb, f2 cc, bf16x8 a, bf16x8 b8, float& r0, float& r1,
                                    float& m) {
    if constexpr (V == 0)
        asm volatile(MFMA_HI "v_mov_b32 v102, %[x]\n v_pk_fma_f32 v[104:105], v[102:103], %[bb], %[cc]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 1)
        asm volatile(MFMA_HI "v_mov_b32 v102, %[x]\n s_nop 0\n v_pk_fma_f32 v[104:105], v[102:103], %[bb], %[cc]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 2)
        asm volatile(VALU_HI "v_mov_b32 v102, %[x]\n v_pk_fma_f32 v[104:105], v[102:103], %[bb], %[cc]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 3)
        asm volatile(MFMA_HI "v_lshlrev_b32 v102, 0, %[x]\n v_pk_fma_f32 v[104:105], v[102:103], %[bb], %[cc]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 4)
        asm volatile(MFMA_HI "v_mov_b32 v102, %[x]\n v_pk_fma_f32 v[104:105], %[bb], v[102:103], %[cc]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 5)
        asm volatile(MFMA_HI "v_mov_b32 v105, %[x]\n s_nop 7\n v_mov_b32 v102, v105\n"
                     " v_pk_fma_f32 v[104:105], v[102:103], %[bb], %[cc]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 6)
        asm volatile(MFMA_HI "v_mfma_f32_16x16x32_bf16 v[108:111], %[a], %[b8], 0\n"
                     " v_mov_b32 v102, %[x]\n v_pk_fma_f32 v[104:105], v[102:103], %[bb], %[cc]\n"
                     " s_nop 7\n s_nop 7\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 7)
        asm volatile(MFMA_HI "v_mov_b32 v102, %[x]\n v_pk_mul_f32 v[104:105], v[102:103], %[bb]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
    if constexpr (V == 8)
        asm volatile(MFMA_HI "v_mov_b32 v102, %[x]\n v_pk_fma_f32 v[104:105], v[102:103], %[bb], %[cc] op_sel_hi:[0,1,1]\n" OUT
                     : [r0] "=v"(r0), [r1] "=v"(r1), [m] "=v"(m)
                     : [x] "v"(x), [y] "v"(y), [bb] "v"(bb), [cc] "v"(cc), [a] "v"(a), [b8] "v"(b8)
                     : CLOB);
}

template <int V>
__global__ __launch_bounds__(768) void probe(const float* in, unsigned* bad, int iters, int noise) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int wave = threadIdx.x >> 6;
    float x = in[(t * 7) & 4095] + 1.0f, y = in[(t * 11 + 1) & 4095] + 2.0f;
    f2 bb = {in[(t * 13 + 2) & 4095] + 0.5f, in[(t * 17 + 3) & 4095] + 0.75f};
    f2 cc = {in[(t * 19 + 4) & 4095], in[(t * 23 + 5) & 4095]};
    bf16x8 a, b8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (short)(0x3f80 + ((t + i) & 15));   // bf16 values 1.0 .. 1.1
        b8[i] = (short)(0x3f00 + ((t * 3 + i) & 31));
    }
    unsigned bad_lo = 0, bad_hi = 0;
    if (noise && (wave & 1)) {
        // noise waves: a dependent MFMA chain plus VALU, for the same number of iterations
        typedef float f4 __attribute__((ext_vector_type(4)));
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int it = 0; it < iters; ++it) {
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b8, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b8, a, acc, 0, 0, 0);
            x = fmaf(x, 0.999f, acc[0] * 1e-30f);
        }
        if (x == 12345.f) bad[64] = 1;  // keep the chain
        return;
    }
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        float r0, r1, m;
        seq<V>(x, y, bb, cc, a, b8, r0, r1, m);
        const float e0 = V == 7 ? x * bb.x : fmaf(x, bb.x, cc.x);
        const float ehi_src = V == 8 ? x : m;
        const float e1 = V == 7 ? ehi_src * bb.y : fmaf(ehi_src, bb.y, cc.y);
        bad_lo += __float_as_uint(r0) != __float_as_uint(e0);
        bad_hi += __float_as_uint(r1) != __float_as_uint(e1);
        x = fmaf(x, 1.0001f, 1e-3f);
        if (x > 4.f) x -= 3.f;
        cc.x = fmaf(cc.x, 0.5f, 0.25f);
    }
    if (bad_lo) atomicAdd(bad + 2 * V, bad_lo);
    if (bad_hi) atomicAdd(bad + 2 * V + 1, bad_hi);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2048;
    const int blocks = argc > 2 ? atoi(argv[2]) : 1024;
    std::vector<float> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
    float* din;
    unsigned* dbad;
    if (hipMalloc(&din, 4096 * 4) != hipSuccess || hipMalloc(&dbad, 128 * 4) != hipSuccess) return 2;
    (void)hipMemcpy(din, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    typedef void (*K)(const float*, unsigned*, int, int);
    const K ks[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>, probe<8>};
    const char* names[] = {"mfma_hi_mov_src0",   "nop_between",      "valu_hi",
                           "lshlrev_producer",   "src1",             "dst_covers_mov_src",
                           "mfma_in_flight",     "pk_mul",           "lo_broadcast"};
    for (int noise = 0; noise < 2; ++noise) {
        for (int v = 0; v < 9; ++v) {
            (void)hipMemset(dbad, 0, 128 * 4);
            hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(768), 0, 0, din, dbad, iters, noise);
            if (hipDeviceSynchronize() != hipSuccess) {
                printf("{\"variant\": \"%s\", \"error\": \"launch\"}\n", names[v]);
                return 3;
            }
            unsigned hb[128];
            (void)hipMemcpy(hb, dbad, 128 * 4, hipMemcpyDeviceToHost);
            const double n = (double)blocks * 768 * iters / (noise ? 2 : 1);
            printf("{\"variant\": \"%s\", \"noise\": %d, \"sequences\": %.0f, \"bad_lo\": %u, \"bad_hi\": %u}\n",
                   names[v], noise, n, hb[2 * v], hb[2 * v + 1]);
            fflush(stdout);
        }
    }
    (void)hipFree(din);
    (void)hipFree(dbad);
    return 0;
}
