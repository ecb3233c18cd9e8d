// Batched strided fp32 GEMM on gfx950's f32-input MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces (paths relative to the reference root):
//   tf.matmul(x, weights_k), one per relation k          decagon/deep/layers.py:113
//   row·L·G·L·colᵀ (predictions)                         decagon/deep/optimizer.py:87-106
//
// v_mfma_f32_32x32x2_f32 is exact fp32: its result is bit-for-bit a k-ordered fmaf chain
// (cdna_hip_programming.md §3 'FP32-input MFMA'), so this path keeps the reference's fp32
// numerics while running on the matrix pipe.  One wave computes one 32x32 output tile:
//   A operand, lane l: A[m0 + (l&31)][k0 + (l>>5)]   (one f32 per lane per k-step of 2)
//   B operand, lane l: B[k0 + (l>>5)][n0 + (l&31)]
//   C/D, register r of lane l: C[m0 + (r&3) + 8(r>>2) + 4(l>>5)][n0 + (l&31)]
// For the relation-batched projection (m = N_j nodes, n = 32, k = 64, batch = K relations)
// each lane keeps its A fragment (the H_j rows) in registers across KB consecutive
// relations of the batch, so H_j is read once per KB relations; the B fragments (W_k, 8 KB)
// and the C stores (two 128-byte row segments per register) are coalesced.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct GemmOne {
    const float* a;
    const float* b;
    float* c;
    const float* sa;
    const float* sc;
    const int32_t* b_map;
    int64_t a_bs, a_sm, a_sk;
    int64_t b_bs, b_sk, b_sn;
    int64_t c_bs, c_sm, c_sn;
    int32_t m, n, k, batch;
    int32_t tiles_m, tiles_n, batch_per_wave;
    int32_t tile_blocks;   // blocks along the tile dimension (4 tiles each)
    int32_t block_begin;   // first block of this GEMM in the launch
    int32_t pad;
};

struct GemmArgs {
    GemmOne g[DG_MAX_GROUPS];
    int32_t n;
};

// One launch runs up to DG_MAX_GROUPS GEMMs: block b -> (GEMM, tile block, batch block).
__device__ __forceinline__ const GemmOne& pick(const GemmArgs& A, int b, int& tb, int& bb) {
    int i = 0;
#pragma unroll 1
    while (i + 1 < A.n && b >= A.g[i + 1].block_begin) ++i;
    const GemmOne& g = A.g[i];
    const int lb = b - g.block_begin;
    bb = lb / g.tile_blocks;
    tb = lb - bb * g.tile_blocks;
    return g;
}

// Generic path: any K, A fragment re-loaded per k-step (L1/L2 resident).
__global__ __launch_bounds__(256) void gemm_f32_generic(const GemmArgs args) {
    int tb, bblk;
    const GemmOne& g = pick(args, blockIdx.x, tb, bblk);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int tile = tb * 4 + wave;
    if (tile >= g.tiles_m * g.tiles_n) return;
    const int tm = tile / g.tiles_n;
    const int tn = tile - tm * g.tiles_n;
    const int i = lane & 31;
    const int h = lane >> 5;
    const int row = tm * 32 + i;
    const int col = tn * 32 + i;
    const bool row_ok = row < g.m;
    const bool col_ok = col < g.n;
    const int b0 = bblk * g.batch_per_wave;
    const int b1 = min(b0 + g.batch_per_wave, g.batch);
#pragma unroll 1
    for (int b = b0; b < b1; ++b) {
        const float* A = g.a + b * g.a_bs + (int64_t)row * g.a_sm;
        const int bb = g.b_map ? g.b_map[b] : b;
        const float* B = g.b + bb * g.b_bs + (int64_t)col * g.b_sn;
        f32x16 acc = {};
#pragma unroll 4
        for (int k0 = 0; k0 < g.k; k0 += 2) {
            const int kk = k0 + h;
            float av = 0.f, bv = 0.f;
            if (kk < g.k) {
                if (row_ok) {
                    av = A[kk * g.a_sk];
                    if (g.sa) av *= g.sa[kk];
                }
                if (col_ok) bv = B[kk * g.b_sk];
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
        if (col_ok) {
            const float s = g.sc ? g.sc[col] : 1.0f;
            float* C = g.c + bb * g.c_bs + (int64_t)col * g.c_sn;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int mrow = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (mrow < g.m) C[(int64_t)mrow * g.c_sm] = acc[r] * s;
            }
        }
    }
}

// Projection path: K == KD (compile-time), the A fragment (KD/2 values per lane) lives in
// registers for all relations the wave handles.
template <int KD>
__global__ __launch_bounds__(256) void gemm_f32_resident_a(const GemmArgs args) {
    constexpr int S = KD / 2;
    int tb, bblk;
    const GemmOne& g = pick(args, blockIdx.x, tb, bblk);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int tile = tb * 4 + wave;
    if (tile >= g.tiles_m * g.tiles_n) return;
    const int tm = tile / g.tiles_n;
    const int tn = tile - tm * g.tiles_n;
    const int i = lane & 31;
    const int h = lane >> 5;
    const int row = tm * 32 + i;
    const int col = tn * 32 + i;
    const bool row_ok = row < g.m;
    const bool col_ok = col < g.n;
    const int b0 = bblk * g.batch_per_wave;
    const int b1 = min(b0 + g.batch_per_wave, g.batch);
    if (b0 >= b1) return;

    // A does not depend on the batch index when a_bs == 0 (shared H_j): load it once.
    float afrag[S];
    const bool shared_a = g.a_bs == 0;
    auto load_a = [&](int b) {
        const float* A = g.a + b * g.a_bs + (int64_t)row * g.a_sm;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int kk = 2 * s + h;
            float av = row_ok ? A[kk * g.a_sk] : 0.f;
            if (g.sa) av *= g.sa[kk];
            afrag[s] = av;
        }
    };
    load_a(b0);
    const float s_col = (col_ok && g.sc) ? g.sc[col] : 1.0f;
#pragma unroll 1
    for (int b = b0; b < b1; ++b) {
        if (!shared_a && b != b0) load_a(b);
        const int bb = g.b_map ? g.b_map[b] : b;
        const float* B = g.b + bb * g.b_bs + (int64_t)col * g.b_sn;
        float bfrag[S];
#pragma unroll
        for (int s = 0; s < S; ++s) bfrag[s] = col_ok ? B[(2 * s + h) * g.b_sk] : 0.f;
        f32x16 acc = {};
#pragma unroll
        for (int s = 0; s < S; ++s)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(afrag[s], bfrag[s], acc, 0, 0, 0);
        if (col_ok) {
            float* C = g.c + bb * g.c_bs + (int64_t)col * g.c_sn;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int mrow = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (mrow < g.m) C[(int64_t)mrow * g.c_sm] = acc[r] * s_col;
            }
        }
    }
}

}  // namespace

extern "C" int dg_gemm_f32(const dg_gemm_desc* descs, int32_t n_desc, void* stream) {
    if (!descs || n_desc < 1) return DG_EINVAL;
    if (n_desc > DG_MAX_GROUPS) return DG_ETOOMANY;
    GemmArgs A{};
    int64_t blocks = 0;
    int kd = -1;
    for (int i = 0; i < n_desc; ++i) {
        const dg_gemm_desc* d = &descs[i];
        if (d->m < 0 || d->n < 0 || d->k < 0 || d->batch < 0) return DG_EINVAL;
        if (d->m == 0 || d->n == 0 || d->batch == 0) continue;
        if (!d->c) return DG_EINVAL;
        if (d->k > 0 && (!d->a || !d->b)) return DG_EINVAL;
        GemmOne& g = A.g[A.n++];
        g.a = d->a;
        g.b = d->b;
        g.c = d->c;
        g.sa = d->sa;
        g.sc = d->sc;
        g.b_map = d->b_map;
        g.a_bs = d->a_bs;
        g.a_sm = d->a_sm;
        g.a_sk = d->a_sk;
        g.b_bs = d->b_bs;
        g.b_sk = d->b_sk;
        g.b_sn = d->b_sn;
        g.c_bs = d->c_bs;
        g.c_sm = d->c_sm;
        g.c_sn = d->c_sn;
        g.m = d->m;
        g.n = d->n;
        g.k = d->k;
        g.batch = d->batch;
        g.tiles_m = dg::ceil_div(d->m, 32);
        g.tiles_n = dg::ceil_div(d->n, 32);
        g.tile_blocks = dg::ceil_div((int64_t)g.tiles_m * g.tiles_n, 4);
        // Relations per wave: enough waves to fill 256 CUs several times over, and each
        // wave amortises its A fragment over up to 16 relations.
        int bpw = 1;
        while (bpw < 16 && (int64_t)g.tile_blocks * 4 * dg::ceil_div(d->batch, bpw * 2) >= 8192) bpw *= 2;
        g.batch_per_wave = bpw;
        g.block_begin = static_cast<int32_t>(blocks);
        blocks += (int64_t)g.tile_blocks * dg::ceil_div(d->batch, bpw);
        if (blocks > 0x7fffffff) return DG_EINVAL;
        const int kk = (d->k == 64 || d->k == 32) ? d->k : 0;
        kd = (kd < 0 || kd == kk) ? kk : 0;
    }
    if (A.n == 0) return DG_OK;
    dim3 grid(static_cast<unsigned>(blocks)), block(256);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (kd == 64)
        hipLaunchKernelGGL(gemm_f32_resident_a<64>, grid, block, 0, st, A);
    else if (kd == 32)
        hipLaunchKernelGGL(gemm_f32_resident_a<32>, grid, block, 0, st, A);
    else
        hipLaunchKernelGGL(gemm_f32_generic, grid, block, 0, st, A);
    return dg::launch_status();
}
