// One wave's 32-pair decoder tile and the counter-based unigram draw, shared by decoder.hip
// (the decoder launches) and slot_scorer.hip (config 5's draws).
//
// Replaces (paths relative to the reference root):
//   DecagonOptimizer.batch_predict + tf.diag_part     decagon/deep/optimizer.py:51-57, :63-85
//   tf.nn.fixed_unigram_candidate_sampler(0.75)        decagon/deep/optimizer.py:40-47
#pragma once
#include "common.h"

namespace dg {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Draw #idx of the counter-based unigram sampler from a Walker alias table: entry j holds
// {acceptance probability (float bits), alias index}.  One 64-bit hash gives the column j
// (high 32 bits, scaled by range) and the 24-bit acceptance uniform (low bits): one 8-byte
// load per draw, no search.
// The counter-based part of draw idx: alias slot j and its uniform u (no memory access).
__device__ __forceinline__ void unigram_pick(int range, uint64_t seed, uint64_t idx, int& j, float& u) {
    const uint64_t h = splitmix64(seed ^ splitmix64(idx));
    j = (int)(((h >> 32) * (uint64_t)range) >> 32);
    u = (float)(h & 0xFFFFFFu) * (1.0f / 16777216.0f);
}

// Draw idx given its slot's table entry e = table[j].
__device__ __forceinline__ int unigram_take(int j, float u, uint2 e) { return u < __uint_as_float(e.x) ? j : (int)e.y; }

__device__ __forceinline__ int unigram_draw(const uint2* table, int range, uint64_t seed,
                                            uint64_t idx) {
    int j;
    float u;
    unigram_pick(range, seed, idx, j, u);
    return unigram_take(j, u, table[j]);
}

struct DecTab {
    const float* row_table;
    const float* col_table;
    const float* G;
    const float* l;
    int64_t ld_row;
    int64_t ld_col;
    int32_t d;
    int32_t vec4;  // row_table, ld_row and l allow 16-byte loads
};

typedef __attribute__((address_space(1))) float gf32;

// A load of an embedding row element.  kSc1: a global `sc1` load (agent scope, bypasses this
// CU's L1) — the form that reads bytes another workgroup of the same launch stored `sc1`
// (MI355X_MICROARCH.md "Valid forms", first row; cdna_hip_programming.md Guideline 16).
template <bool kSc1>
__device__ __forceinline__ float ld_emb(const float* p) {
    if constexpr (kSc1)
        return __hip_atomic_load((gf32*)(const_cast<float*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        return *p;
}

template <bool kSc1>
__device__ __forceinline__ float4 ld_emb4(const float* p) {
    if constexpr (kSc1)
        return make_float4(ld_emb<true>(p), ld_emb<true>(p + 1), ld_emb<true>(p + 2), ld_emb<true>(p + 3));
    else
        return *reinterpret_cast<const float4*>(p);
}

// Scores of 32 pairs on one wave: lane i (both halves) names pair i by its row index
// `ridx` (into row_table) and column index `cidx` (into col_table); `valid` masks pairs
// past the end.  T = (U∘l)·G runs on v_mfma_f32_32x32x2_f32 in k-blocks of 32 whose A/B
// fragments are loaded up front (one memory round trip per block, not per k-step); then
// score[p] = Σ_j T[p][j]·l[j]·V[p][j] is folded over the 32 lanes of each half-wave.
// Returns the score of pair (r&3)+8(r>>2)+4h, r = (lane & 31) >> 1, in part[0] of lanes 2r and
// 2r+1 of each half (a reduce-scatter over the half's 32 lanes: 16 shuffles instead of a
// butterfly per score's 80).  kSc1: every load of
// row_table / col_table is an sc1 load (the tables were written in this launch).  kD: the width
// when known at compile time (only that path is compiled: fewer registers), else 0.
#ifdef DG_DEC_PROF
// Profiling build only (scripts/dec_prof.py): s_memrealtime stamps of the hinge decoder's
// phases per (block, wave).
constexpr int kDecProfSlots = 8;
__device__ unsigned long long g_dec_prof[256][2][kDecProfSlots];
#define DG_DEC_STAMP(i)                                                                                       \
    do {                                                                                                      \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                           \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 256)                                                      \
            dg::g_dec_prof[blockIdx.x][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memrealtime();                 \
    } while (0)
#else
#define DG_DEC_STAMP(i) ((void)0)
#endif

template <bool kSc1 = false, int kD = 0>
__device__ __forceinline__ void score_tile(const DecTab& t, int ridx, int cidx, bool valid,
                                           float (&part)[16]) {
    const int lane = threadIdx.x & 63;
    const int i = lane & 31;
    const int h = lane >> 5;
    const int d = kD ? kD : t.d;
    const float* u = t.row_table + (int64_t)ridx * t.ld_row;
#pragma unroll
    for (int r = 0; r < 16; ++r) part[r] = 0.f;
    if (d == 32) {
        // one k-block, one n-block: every load (G, l, U row, V rows) in flight together, then
        // the 16 MFMAs.  MFMA s takes k = 16h + s from lane half h (the contraction order is
        // free), so each lane's A operand is 16 contiguous floats of its U row: 4 float4 loads
        // the parameters (G, l) first, then the U and V rows: sc1 (atomic) loads keep their
        // source order, and a plain load or a use between them costs a memory round trip each
        float av[16], bv[16], v[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) bv[s] = t.G[(16 * h + s) * 32 + i];
        const float lj = t.l ? t.l[i] : 1.0f;
        float4 w4[4];
        if (t.vec4 && t.l) {
            const float4* l4 = reinterpret_cast<const float4*>(t.l + 16 * h);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) w4[s4] = l4[s4];
        }
        if (!t.vec4) {
#pragma unroll
            for (int s = 0; s < 16; ++s) av[s] = valid ? ld_emb<kSc1>(u + 16 * h + s) : 0.f;
        } else {
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const float4 a4 = valid ? ld_emb4<kSc1>(u + 16 * h + 4 * s4) : make_float4(0.f, 0.f, 0.f, 0.f);
                av[4 * s4] = a4.x;
                av[4 * s4 + 1] = a4.y;
                av[4 * s4 + 2] = a4.z;
                av[4 * s4 + 3] = a4.w;
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int prow = (r & 3) + 8 * (r >> 2) + 4 * h;
            v[r] = ld_emb<kSc1>(t.col_table + (int64_t)__shfl(cidx, prow) * t.ld_col + i);
        }
        if (t.l) {
            if (t.vec4) {
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4) {
                    av[4 * s4] *= w4[s4].x;
                    av[4 * s4 + 1] *= w4[s4].y;
                    av[4 * s4 + 2] *= w4[s4].z;
                    av[4 * s4 + 3] *= w4[s4].w;
                }
            } else {
#pragma unroll
                for (int s = 0; s < 16; ++s) av[s] *= t.l[16 * h + s];
            }
        }
        DG_DEC_STAMP(2);  // (profiling build: the tile's loads landed)
        f32x16 acc = {};
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) part[r] = fmaf(acc[r] * lj, v[r], 0.f);
        DG_DEC_STAMP(3);  // MFMA chain + epilogue products
    }
#pragma unroll 1
    for (int n0 = 0; d != 32 && n0 < d; n0 += 32) {
        f32x16 acc = {};
#pragma unroll 1
        for (int k0 = 0; k0 < d; k0 += 32) {
            float av[16], bv[16];
#pragma unroll
            for (int s = 0; s < 16; ++s) av[s] = valid ? ld_emb<kSc1>(u + k0 + 2 * s + h) : 0.f;
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const int kk = k0 + 2 * s + h;
                if (t.l) av[s] *= t.l[kk];
                bv[s] = t.G[(int64_t)kk * d + n0 + i];
            }
#pragma unroll
            for (int s = 0; s < 16; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc, 0, 0, 0);
        }
        const int j = n0 + i;
        const float lj = t.l ? t.l[j] : 1.0f;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int prow = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int c = __shfl(cidx, prow);  // lane prow names pair prow
            v[r] = ld_emb<kSc1>(t.col_table + (int64_t)c * t.ld_col + j);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) part[r] = fmaf(acc[r] * lj, v[r], part[r]);
    }
    // reduce-scatter over the half's 32 lanes: at each step a lane keeps the half of its
    // remaining scores that its lane bit selects and adds its partner's copy of them
    const int b4 = (i >> 4) & 1, b3 = (i >> 3) & 1, b2 = (i >> 2) & 1, b1 = (i >> 1) & 1;
    float v8[8], v4[4], v2[2];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        v8[j] = (b4 ? part[8 + j] : part[j]) + xor_get<16>(b4 ? part[j] : part[8 + j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) v4[j] = (b3 ? v8[4 + j] : v8[j]) + xor_get<8>(b3 ? v8[j] : v8[4 + j]);
#pragma unroll
    for (int j = 0; j < 2; ++j) v2[j] = (b2 ? v4[2 + j] : v4[j]) + __shfl_xor(b2 ? v4[j] : v4[2 + j], 4);
    float v1 = (b1 ? v2[1] : v2[0]) + xor_get<2>(b1 ? v2[0] : v2[1]);
    v1 = xor_add<1>(v1);
    part[0] = v1;  // score r = 8·b4 + 4·b3 + 2·b2 + b1 = (lane & 31) >> 1
    DG_DEC_STAMP(4);  // reduce-scatter
}

}  // namespace dg
