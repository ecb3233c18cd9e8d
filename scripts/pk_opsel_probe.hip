// Stand-alone reproduction attempt for config 5's wrong scores ("The config-5
// miscompile").  The failing build's score epilogue block (56 VALU instructions, copied from
// its assembly: the q loop's positive chain of both halves, packed by the compiler) runs on
// registers loaded from memory, then the same block with its four `v_pk_mul_f32 ...
// op_sel:[0,1]` as two scalar v_mul_f32 each — the edit that removed every failure in the
// full kernel (scripts/hazard_variants.py, unpack_sel01 / swap_sel01).  Every lane compares
// the two results bit for bit, for many inputs, with the other waves of each SIMD idle, running
// MFMA chains, or running MFMA chains with vector loads.  It touches registers and vector
// memory only (results through vector atomics).
//
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/pk_opsel_probe scripts/pk_opsel_probe.hip
// Run:   scripts/pk_opsel_probe [iters] [blocks]      (one JSON line per mode)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CLOB                                                                                          \
    "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", \
        "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v112", "v113", "v114", "v115", "v116", \
        "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v148", "v149", "v150", "v151", "v152", \
        "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", \
        "v165", "v166", "v167", "memory"

constexpr int kLive = 33;     // live-in registers of the block, loaded from memory
constexpr int kSets = 4096;   // input sets

#define DG_LOADS \
    "global_load_dword v74, %[p], off offset:0\n" \
    "global_load_dword v75, %[p], off offset:4\n" \
    "global_load_dword v76, %[p], off offset:8\n" \
    "global_load_dword v77, %[p], off offset:12\n" \
    "global_load_dword v78, %[p], off offset:16\n" \
    "global_load_dword v79, %[p], off offset:20\n" \
    "global_load_dword v80, %[p], off offset:24\n" \
    "global_load_dword v81, %[p], off offset:28\n" \
    "global_load_dword v82, %[p], off offset:32\n" \
    "global_load_dword v83, %[p], off offset:36\n" \
    "global_load_dword v84, %[p], off offset:40\n" \
    "global_load_dword v85, %[p], off offset:44\n" \
    "global_load_dword v86, %[p], off offset:48\n" \
    "global_load_dword v87, %[p], off offset:52\n" \
    "global_load_dword v88, %[p], off offset:56\n" \
    "global_load_dword v89, %[p], off offset:60\n" \
    "global_load_dword v90, %[p], off offset:64\n" \
    "global_load_dword v91, %[p], off offset:68\n" \
    "global_load_dword v92, %[p], off offset:72\n" \
    "global_load_dword v93, %[p], off offset:76\n" \
    "global_load_dword v95, %[p], off offset:80\n" \
    "global_load_dword v112, %[p], off offset:84\n" \
    "global_load_dword v113, %[p], off offset:88\n" \
    "global_load_dword v114, %[p], off offset:92\n" \
    "global_load_dword v115, %[p], off offset:96\n" \
    "global_load_dword v116, %[p], off offset:100\n" \
    "global_load_dword v117, %[p], off offset:104\n" \
    "global_load_dword v119, %[p], off offset:108\n" \
    "global_load_dword v123, %[p], off offset:112\n" \
    "global_load_dword v148, %[p], off offset:116\n" \
    "global_load_dword v149, %[p], off offset:120\n" \
    "global_load_dword v150, %[p], off offset:124\n" \
    "global_load_dword v151, %[p], off offset:128\n" \
    "s_waitcnt vmcnt(0)\n"

#define DG_BLOCK_PACKED \
    "v_lshlrev_b32_e32 v152, 16, v114\n" \
    "v_lshlrev_b32_e32 v153, 16, v82\n" \
    "v_and_b32_e32 v120, 0xffff0000, v82\n" \
    "v_and_b32_e32 v154, 0xffff0000, v114\n" \
    "v_lshlrev_b32_e32 v122, 16, v148\n" \
    "v_lshlrev_b32_e32 v156, 16, v115\n" \
    "v_and_b32_e32 v158, 0xffff0000, v115\n" \
    "v_lshlrev_b32_e32 v160, 16, v116\n" \
    "v_and_b32_e32 v162, 0xffff0000, v116\n" \
    "v_lshlrev_b32_e32 v164, 16, v117\n" \
    "v_and_b32_e32 v166, 0xffff0000, v117\n" \
    "v_and_b32_e32 v121, 0xffff0000, v148\n" \
    "v_lshlrev_b32_e32 v157, 16, v83\n" \
    "v_lshlrev_b32_e32 v118, 16, v149\n" \
    "v_and_b32_e32 v117, 0xffff0000, v149\n" \
    "v_and_b32_e32 v116, 0xffff0000, v83\n" \
    "v_lshlrev_b32_e32 v161, 16, v84\n" \
    "v_lshlrev_b32_e32 v94, 16, v150\n" \
    "v_and_b32_e32 v115, 0xffff0000, v150\n" \
    "v_and_b32_e32 v114, 0xffff0000, v84\n" \
    "v_lshlrev_b32_e32 v84, 16, v151\n" \
    "v_and_b32_e32 v83, 0xffff0000, v151\n" \
    "v_pk_mul_f32 v[148:149], v[152:153], v[122:123] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v150, v86\n" \
    "v_mov_b32_e32 v151, v74\n" \
    "v_mov_b32_e32 v155, v120\n" \
    "v_pk_fma_f32 v[112:113], v[150:151], v[148:149], v[112:113]\n" \
    "v_pk_mul_f32 v[148:149], v[154:155], v[120:121] op_sel:[0,1]\n" \
    "v_mov_b32_e32 v74, v87\n" \
    "v_pk_fma_f32 v[86:87], v[74:75], v[148:149], v[112:113]\n" \
    "v_pk_mul_f32 v[112:113], v[156:157], v[118:119] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v148, v88\n" \
    "v_mov_b32_e32 v149, v76\n" \
    "v_mov_b32_e32 v159, v116\n" \
    "v_pk_fma_f32 v[86:87], v[148:149], v[112:113], v[86:87]\n" \
    "v_pk_mul_f32 v[112:113], v[158:159], v[116:117] op_sel:[0,1]\n" \
    "v_mov_b32_e32 v76, v89\n" \
    "v_pk_fma_f32 v[86:87], v[76:77], v[112:113], v[86:87]\n" \
    "v_pk_mul_f32 v[88:89], v[160:161], v[94:95] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v152, v90\n" \
    "v_mov_b32_e32 v153, v78\n" \
    "v_mov_b32_e32 v163, v114\n" \
    "v_lshlrev_b32_e32 v165, 16, v85\n" \
    "v_and_b32_e32 v82, 0xffff0000, v85\n" \
    "v_pk_fma_f32 v[86:87], v[152:153], v[88:89], v[86:87]\n" \
    "v_pk_mul_f32 v[88:89], v[162:163], v[114:115] op_sel:[0,1]\n" \
    "v_mov_b32_e32 v78, v91\n" \
    "v_pk_fma_f32 v[86:87], v[78:79], v[88:89], v[86:87]\n" \
    "v_pk_mul_f32 v[88:89], v[164:165], v[84:85] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v90, v92\n" \
    "v_mov_b32_e32 v91, v80\n" \
    "v_mov_b32_e32 v167, v82\n" \
    "v_pk_fma_f32 v[86:87], v[90:91], v[88:89], v[86:87]\n" \
    "v_pk_mul_f32 v[88:89], v[166:167], v[82:83] op_sel:[0,1]\n" \
    "v_mov_b32_e32 v80, v93\n" \
    "v_pk_fma_f32 v[112:113], v[80:81], v[88:89], v[86:87]\n"

#define DG_BLOCK_SCALAR \
    "v_lshlrev_b32_e32 v152, 16, v114\n" \
    "v_lshlrev_b32_e32 v153, 16, v82\n" \
    "v_and_b32_e32 v120, 0xffff0000, v82\n" \
    "v_and_b32_e32 v154, 0xffff0000, v114\n" \
    "v_lshlrev_b32_e32 v122, 16, v148\n" \
    "v_lshlrev_b32_e32 v156, 16, v115\n" \
    "v_and_b32_e32 v158, 0xffff0000, v115\n" \
    "v_lshlrev_b32_e32 v160, 16, v116\n" \
    "v_and_b32_e32 v162, 0xffff0000, v116\n" \
    "v_lshlrev_b32_e32 v164, 16, v117\n" \
    "v_and_b32_e32 v166, 0xffff0000, v117\n" \
    "v_and_b32_e32 v121, 0xffff0000, v148\n" \
    "v_lshlrev_b32_e32 v157, 16, v83\n" \
    "v_lshlrev_b32_e32 v118, 16, v149\n" \
    "v_and_b32_e32 v117, 0xffff0000, v149\n" \
    "v_and_b32_e32 v116, 0xffff0000, v83\n" \
    "v_lshlrev_b32_e32 v161, 16, v84\n" \
    "v_lshlrev_b32_e32 v94, 16, v150\n" \
    "v_and_b32_e32 v115, 0xffff0000, v150\n" \
    "v_and_b32_e32 v114, 0xffff0000, v84\n" \
    "v_lshlrev_b32_e32 v84, 16, v151\n" \
    "v_and_b32_e32 v83, 0xffff0000, v151\n" \
    "v_pk_mul_f32 v[148:149], v[152:153], v[122:123] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v150, v86\n" \
    "v_mov_b32_e32 v151, v74\n" \
    "v_mov_b32_e32 v155, v120\n" \
    "v_pk_fma_f32 v[112:113], v[150:151], v[148:149], v[112:113]\n" \
    "v_mul_f32 v148, v154, v121\n" \
    "v_mul_f32 v149, v155, v121\n" \
    "v_mov_b32_e32 v74, v87\n" \
    "v_pk_fma_f32 v[86:87], v[74:75], v[148:149], v[112:113]\n" \
    "v_pk_mul_f32 v[112:113], v[156:157], v[118:119] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v148, v88\n" \
    "v_mov_b32_e32 v149, v76\n" \
    "v_mov_b32_e32 v159, v116\n" \
    "v_pk_fma_f32 v[86:87], v[148:149], v[112:113], v[86:87]\n" \
    "v_mul_f32 v112, v158, v117\n" \
    "v_mul_f32 v113, v159, v117\n" \
    "v_mov_b32_e32 v76, v89\n" \
    "v_pk_fma_f32 v[86:87], v[76:77], v[112:113], v[86:87]\n" \
    "v_pk_mul_f32 v[88:89], v[160:161], v[94:95] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v152, v90\n" \
    "v_mov_b32_e32 v153, v78\n" \
    "v_mov_b32_e32 v163, v114\n" \
    "v_lshlrev_b32_e32 v165, 16, v85\n" \
    "v_and_b32_e32 v82, 0xffff0000, v85\n" \
    "v_pk_fma_f32 v[86:87], v[152:153], v[88:89], v[86:87]\n" \
    "v_mul_f32 v88, v162, v115\n" \
    "v_mul_f32 v89, v163, v115\n" \
    "v_mov_b32_e32 v78, v91\n" \
    "v_pk_fma_f32 v[86:87], v[78:79], v[88:89], v[86:87]\n" \
    "v_pk_mul_f32 v[88:89], v[164:165], v[84:85] op_sel_hi:[1,0]\n" \
    "v_mov_b32_e32 v90, v92\n" \
    "v_mov_b32_e32 v91, v80\n" \
    "v_mov_b32_e32 v167, v82\n" \
    "v_pk_fma_f32 v[86:87], v[90:91], v[88:89], v[86:87]\n" \
    "v_mul_f32 v88, v166, v83\n" \
    "v_mul_f32 v89, v167, v83\n" \
    "v_mov_b32_e32 v80, v93\n" \
    "v_pk_fma_f32 v[112:113], v[80:81], v[88:89], v[86:87]\n"


// mode 0: every wave checks; 1: odd waves run a dependent MFMA chain; 2: odd waves run MFMAs
// and stream vector loads (the real kernel's neighbours on a SIMD)
__global__ __launch_bounds__(768) void probe(const float* in, unsigned* bad, int iters, int mode) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int wave = threadIdx.x >> 6;
    if (mode && (wave & 1)) {
        bf16x8 a, b;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            a[i] = (short)(0x3f80 + ((t + i) & 15));
            b[i] = (short)(0x3f00 + ((t * 3 + i) & 31));
        }
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        float s = 0.f;
        for (int it = 0; it < 3 * iters; ++it) {
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc, 0, 0, 0);
            if (mode == 2) s += in[((t * 131 + it * 4099) & (kSets * kLive - 1))];
        }
        if (acc[0] + s == 12345.f) bad[64] = 1;  // keep the chain
        return;
    }
    unsigned bad_lo = 0, bad_hi = 0;
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        const float* p = in + ((t + it * 977) & (kSets - 1)) * kLive;
        float r0, r1, s0, s1;
        asm volatile(DG_LOADS DG_BLOCK_PACKED "v_mov_b32 %[r0], v112\n v_mov_b32 %[r1], v113\n"
                     : [r0] "=v"(r0), [r1] "=v"(r1)
                     : [p] "v"(p)
                     : CLOB);
        asm volatile(DG_LOADS DG_BLOCK_SCALAR "v_mov_b32 %[r0], v112\n v_mov_b32 %[r1], v113\n"
                     : [r0] "=v"(s0), [r1] "=v"(s1)
                     : [p] "v"(p)
                     : CLOB);
        bad_lo += __float_as_uint(r0) != __float_as_uint(s0);
        bad_hi += __float_as_uint(r1) != __float_as_uint(s1);
    }
    if (bad_lo) atomicAdd(bad + 0, bad_lo);
    if (bad_hi) atomicAdd(bad + 1, bad_hi);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4096;
    const int blocks = argc > 2 ? atoi(argv[2]) : 1024;
    std::vector<float> h((size_t)kSets * kLive);
    unsigned s = 12345u;
    for (auto& x : h) {
        s = s * 1664525u + 1013904223u;
        x = (float)((int)(s >> 8) % 2001 - 1000) / 500.f;  // [-2, 2]
    }
    float* din;
    unsigned* dbad;
    if (hipMalloc(&din, h.size() * 4) != hipSuccess || hipMalloc(&dbad, 128 * 4) != hipSuccess) return 2;
    (void)hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 3; ++mode) {
        (void)hipMemset(dbad, 0, 128 * 4);
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(768), 0, 0, din, dbad, iters, mode);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("{\"mode\": %d, \"error\": \"launch\"}\n", mode);
            return 3;
        }
        unsigned hb[2];
        (void)hipMemcpy(hb, dbad, 8, hipMemcpyDeviceToHost);
        const double n = (double)blocks * 768 * iters / (mode ? 2 : 1);
        printf("{\"mode\": %d, \"lane_blocks\": %.0f, \"bad_lo\": %u, \"bad_hi\": %u}\n", mode, n, hb[0], hb[1]);
        fflush(stdout);
    }
    return 0;
}
