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
#include <type_traits>

#include "common.h"
#include "dropout.h"

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
    int32_t reduce;        // batch-reduce mode: batches summed in runs of batch_per_wave
    const uint64_t* drop_state;  // batch-reduce only: batch products masked before the sum
    uint32_t drop_tag;
    float drop_keep;
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
    f32x16 acc = {};
    const bool drop = g.reduce && g.drop_state;  // masked batch-reduce (dropout backward)
    f32x16 dsum = {};
    const uint32_t dkey = drop ? dg::drop_key(g.drop_state, g.drop_tag) : 0u;
#pragma unroll 1
    for (int b = b0; b < b1; ++b) {
        const float* A = g.a + b * g.a_bs + (int64_t)row * g.a_sm;
        const int bb = g.b_map ? g.b_map[b] : b;
        const float* B = g.b + bb * g.b_bs + (int64_t)col * g.b_sn;
        if (!g.reduce || drop) acc = f32x16{};
        f32x16& t = acc;
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
            t = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, t, 0, 0, 0);
        }
        if (drop) {
            // Σ_b M_b∘(A_b·B_b): element (row, col) of batch b carries mask bit (bb·m + row)·n + col
            // (bb = b_map[b]: a relation shard's batch b is global relation bb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int mrow = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const uint32_t idx = static_cast<uint32_t>(((int64_t)bb * g.m + mrow) * g.n + col);
                dsum[r] += t[r] * dg::keep_scale(dkey, idx, g.drop_keep);
            }
        }
        if (g.reduce && b + 1 < b1) continue;  // batch-reduce: one store per run, at run index
        if (drop) acc = dsum;
        if (col_ok) {
            const float s = g.sc ? g.sc[col] : 1.0f;
            float* C = g.c + (g.reduce ? bblk : bb) * g.c_bs + (int64_t)col * g.c_sn;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int mrow = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (mrow < g.m) C[(int64_t)mrow * g.c_sm] = acc[r] * s;
            }
        }
    }
}

// Batch-reduce with K == 32 and both operands contiguous along k (A(m,k) = a[m*a_sm + k],
// B(k,n) = b[n*b_sn + k]): the backward's Σ_b dP_b·W2_bᵀ.  The 32 k-values are consumed in
// the order c = 16h + s (s = MFMA step, h = lane half) — a permutation of the same sum — so
// each lane reads 16 contiguous floats of its row (4 float4 loads) instead of 16 scattered
// ones.  A wave computes a 32-row tile against all n (≤ 64: NT tiles) for its run of batches;
// with a dropout descriptor each batch product is masked before it joins the run's sum.  With a
// batch map, batch b reads B_{map(b)} and carries mask bits of batch map(b) (A and the run
// index stay unmapped).
template <int NT>
__global__ __launch_bounds__(256) void gemm_f32_reduce_k32(const GemmArgs args) {
    int tb, bblk;
    const GemmOne& g = pick(args, blockIdx.x, tb, bblk);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int tm = tb * 4 + wave;
    if (tm >= g.tiles_m) return;
    const int i = lane & 31;
    const int h = lane >> 5;
    const int row = tm * 32 + i;
    const bool row_ok = row < g.m;
    const int b0 = bblk * g.batch_per_wave;
    const int b1 = min(b0 + g.batch_per_wave, g.batch);
    const bool drop = g.drop_state != nullptr;
    const uint32_t dkey = drop ? dg::drop_key(g.drop_state, g.drop_tag) : 0u;
    f32x16 sum[NT], acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) sum[t] = f32x16{};
    // the next batch's fragments are loaded while the current batch's MFMAs run
    float4 a4[4], b4[NT][4];
    auto load = [&](int b) {
        const int bb = g.b_map ? g.b_map[b] : b;
        const float* A = g.a + b * g.a_bs + (int64_t)(row_ok ? row : 0) * g.a_sm + 16 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            a4[q] = row_ok ? *reinterpret_cast<const float4*>(A + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int col = t * 32 + i;
            const float* B = g.b + bb * g.b_bs + (int64_t)(col < g.n ? col : 0) * g.b_sn + 16 * h;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                b4[t][q] = col < g.n ? *reinterpret_cast<const float4*>(B + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    if (b0 < b1) load(b0);
#pragma unroll 1
    for (int b = b0; b < b1; ++b) {
        float4 ca[4], cb[NT][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) ca[q] = a4[q];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) cb[t][q] = b4[t][q];
        if (b + 1 < b1) load(b + 1);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = drop ? f32x16{} : sum[t];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float av[4] = {ca[q].x, ca[q].y, ca[q].z, ca[q].w};
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float bv[4] = {cb[t][q].x, cb[t][q].y, cb[t][q].z, cb[t][q].w};
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc[t], 0, 0, 0);
            }
        }
        if (drop) {
            const int bb = g.b_map ? g.b_map[b] : b;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int mrow = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const uint32_t idx = static_cast<uint32_t>(((int64_t)bb * g.m + mrow) * g.n + t * 32 + i);
                    sum[t][r] += acc[t][r] * dg::keep_scale(dkey, idx, g.drop_keep);
                }
        } else {
#pragma unroll
            for (int t = 0; t < NT; ++t) sum[t] = acc[t];
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int col = t * 32 + i;
        if (col >= g.n) continue;
        float* C = g.c + bblk * g.c_bs + (int64_t)col * g.c_sn;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int mrow = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (mrow < g.m) C[(int64_t)mrow * g.c_sm] = sum[t][r];
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

// Relation-batched projection C_b = A · B_map(b) with A shared by every batch (H_j,
// a_bs == 0), n <= 32, K == KD, no scaling: the transposed product on the matrix pipe,
//   D[n][m] = sum_k B[k][n] * A[m][k] = C[m][n],
// so lane l ends with row m0 + (l&31) and columns 8q + 4(l>>5) .. +3 of it for q < 4: four
// 16-byte stores per lane.  One wave per 32-row tile of A (its fragment in registers for the
// block's run of batches); B_map(b) (KD×32 floats) is staged through LDS once per block and
// batch, double-buffered, in the fragment order [n][k / S][k % S] (rows padded by 4 floats),
// its float4 loads issued two batches ahead and before the previous batch's stores (vmcnt
// counts stores too: a wait for a load issued after a store would drain the store).
template <int KD>
__global__ __launch_bounds__(512) void gemm_f32_proj(const GemmArgs args) {
    constexpr int S = KD / 2;
    constexpr int LDW = S + 4;               // floats per (n, k&1) row of the staged B
    constexpr int WB = 32 * 2 * LDW;         // floats per staged B buffer
    constexpr int NF4 = KD * 8;              // float4s of one [KD][32] B
    __shared__ float wl[2 * WB];
    int tb, bblk;
    const GemmOne& g = pick(args, blockIdx.x, tb, bblk);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const int tm = tb * nw + wave;           // this wave's 32-row tile
    const int i = lane & 31;
    const int h = lane >> 5;
    const int b0 = bblk * g.batch_per_wave;
    const int b1 = min(b0 + g.batch_per_wave, g.batch);
    const int row = tm * 32 + i;
    const bool row_ok = tm < g.tiles_m && row < g.m;

    // k order: MFMA step s contracts k = s (lane half 0) and k = S + s (half 1), so each lane's
    // B operand is one contiguous half row of A — S/4 float4 loads (a permutation of the
    // k-sum; A contiguous along k, rows 16-byte aligned)
    float hf[S];  // B operand of the transposed product: A[row][S·h + s]
    {
        const float4* A = reinterpret_cast<const float4*>(g.a + (int64_t)(row_ok ? row : 0) * g.a_sm + S * h);
#pragma unroll
        for (int q = 0; q < S / 4; ++q) {
            const float4 v = row_ok ? A[q] : make_float4(0.f, 0.f, 0.f, 0.f);
            hf[4 * q] = v.x;
            hf[4 * q + 1] = v.y;
            hf[4 * q + 2] = v.z;
            hf[4 * q + 3] = v.w;
        }
    }
    // the block's batch map in one register (<= 64 batches): lane j holds map(b0 + j), read
    // with readlane — no vector load (and no vmcnt wait, which would also drain the stores)
    // inside the loop
    const int bm = b0 + lane < b1 ? (g.b_map ? g.b_map[b0 + lane] : b0 + lane) : 0;
    auto map_of = [&](int b) { return __builtin_amdgcn_readlane(bm, b - b0); };
    // B_map(b) in float4s of [KD][32]: thread t holds float4s t and t + blockDim, taken modulo
    // NF4 (a duplicate slot is written twice with the same value) and columns >= n read as
    // column 0 (they only feed output columns that are not stored) — so loads and LDS writes
    // are unconditional, and the compiler's waits stay counted: a branch around them made it
    // wait for vmcnt(0), i.e. for the previous batch's HBM stores, every batch
    float4 wr0 = make_float4(0.f, 0.f, 0.f, 0.f), wr1 = wr0;
    const int f0 = threadIdx.x & (NF4 - 1), f1 = (threadIdx.x + blockDim.x) & (NF4 - 1);
    const int c0 = 4 * (f0 & 7) < g.n ? 4 * (f0 & 7) : 0, c1 = 4 * (f1 & 7) < g.n ? 4 * (f1 & 7) : 0;
    auto load_b = [&](int b) {
        const float* B = g.b + map_of(b) * g.b_bs;
        wr0 = *reinterpret_cast<const float4*>(B + (f0 >> 3) * g.b_sk + c0);
        wr1 = *reinterpret_cast<const float4*>(B + (f1 >> 3) * g.b_sk + c1);
    };
    auto put_b = [&](int u) {
        float* w = wl + u * WB;
        auto put4 = [&](int f, float4 v) {
            const int k = f >> 3, n = 4 * (f & 7);
            float* d = w + (n * 2 + k / S) * LDW + (k % S);
            d[0] = v.x;
            d[2 * LDW] = v.y;
            d[4 * LDW] = v.z;
            d[6 * LDW] = v.w;
        };
        put4(f0, wr0);
        put4(f1, wr1);
    };
    if (b0 < b1) {
        load_b(b0);
        put_b(0);
        load_b(min(b0 + 1, b1 - 1));
    }
    // iteration b: barrier | MFMAs on buffer b | B(b+1) registers -> the other buffer (its loads
    // were issued before batch b-1's stores) | loads of B(b+2) | stores of batch b.
    // MODE 0: this wave stores nothing (no tile); 1: n == 32 — every lane stores all four
    // pieces unconditionally (a lane past the last row stores row m-1's values, shuffled in
    // from the lane that owns it: the same bytes) so the wave's VMEM count per iteration is
    // fixed and the waits before the LDS writes stay counted (vmcnt(4), not vmcnt(0): the
    // previous batch's stores keep draining under this batch's MFMAs); 2: general n.
    const bool last_tile = tm == g.tiles_m - 1;
    const int src = row_ok ? lane : (g.m - 1 - tm * 32) + 32 * h;
    auto body = [&](int b, auto mode_tag) {
        constexpr int MODE = decltype(mode_tag)::value;
        __syncthreads();  // buffer (b - b0) & 1 staged; the other one is free
        const float* w = wl + ((b - b0) & 1) * WB + (i * 2 + h) * LDW;
        f32x16 acc = {};
#pragma unroll
        for (int s4 = 0; s4 < S; s4 += 4) {
            const float4 af = *reinterpret_cast<const float4*>(w + s4);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.x, hf[s4 + 0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.y, hf[s4 + 1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.z, hf[s4 + 2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.w, hf[s4 + 3], acc, 0, 0, 0);
        }
        put_b((b + 1 - b0) & 1);          // past the run's end: a harmless rewrite of the free buffer
        load_b(min(b + 2, b1 - 1));
        if constexpr (MODE == 1) {
            if (last_tile) {
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = __shfl(acc[r], src);
            }
            float* C = g.c + map_of(b) * g.c_bs + (int64_t)(row_ok ? row : g.m - 1) * g.c_sm;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<float4*>(C + 8 * q + 4 * h) =
                    make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
        } else if constexpr (MODE == 2) {
            if (row_ok) {
                float* C = g.c + map_of(b) * g.c_bs + (int64_t)row * g.c_sm;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int n = 8 * q + 4 * h;
                    if (n < g.n)
                        *reinterpret_cast<float4*>(C + n) =
                            make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                }
            }
        }
    };
    using M0 = std::integral_constant<int, 0>;
    using M1 = std::integral_constant<int, 1>;
    using M2 = std::integral_constant<int, 2>;
    if (tm >= g.tiles_m) {
#pragma unroll 1
        for (int b = b0; b < b1; ++b) body(b, M0{});
    } else if (g.n == 32) {
#pragma unroll 1
        for (int b = b0; b < b1; ++b) body(b, M1{});
    } else {
#pragma unroll 1
        for (int b = b0; b < b1; ++b) body(b, M2{});
    }
}

// C_b = Aᵀ·B_b with A shared ([rows][M], row stride lda) and B_b = b + b*b_bs ([rows][N],
// row stride ldb): the weight gradient H_jᵀ·dP_k of the per-relation projections (the
// backward of layers.py:113).  The reduction runs over `rows` (up to the node count), so a
// workgroup takes one (batch, row split) and its 4 waves interleave the split's row pairs,
// each on MT×NT accumulators of v_mfma_f32_32x32x2_f32 (both operand fragments are rows of
// A / B read by 32 consecutive lanes: coalesced); the waves meet in LDS in a fixed order.
struct TnArgs {
    const float* a;
    const float* b;
    float* out;            // [batch][M][N], or the split partials [n_split][batch][M][N]
    int64_t lda, a_bs, ldb, b_bs;
    int32_t rows, M, N, batch;
    int32_t n_split, rows_per_split;
};

template <int MT, int NT>
__global__ __launch_bounds__(256) void gemm_tn_kernel(const TnArgs a) {
    __shared__ float red[2][MT * NT][16][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int i = lane & 31, h = lane >> 5;
    const int b = blockIdx.x / a.n_split;
    const int s = blockIdx.x - b * a.n_split;
    const int r_begin = s * a.rows_per_split;
    const int r_end = min(a.rows, r_begin + a.rows_per_split);
    const float* A = a.a + (int64_t)b * a.a_bs;
    const float* B = a.b + (int64_t)b * a.b_bs;
    f32x16 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x16{};
#pragma unroll 8
    for (int r0 = r_begin + 2 * w; r0 < r_end; r0 += 8) {
        const int r = r0 + h;
        const bool ok = r < r_end;
        float af[MT], bf[NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = ok ? A[(int64_t)r * a.lda + mt * 32 + i] : 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bf[nt] = ok ? B[(int64_t)r * a.ldb + nt * 32 + i] : 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mt], bf[nt], acc[mt][nt], 0, 0, 0);
    }
    // the 4 waves' sums meet in two LDS stages, (w0 + w2) + (w1 + w3): 16 KB per MT·NT pair
    if (w >= 2) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 16; ++r) red[w - 2][mt * NT + nt][r][lane] = acc[mt][nt][r];
    }
    __syncthreads();
    if (w < 2) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 16; ++r) red[w][mt * NT + nt][r][lane] += acc[mt][nt][r];
    }
    __syncthreads();
    float* out = a.out + ((int64_t)s * a.batch + b) * a.M * a.N;
    for (int e = threadIdx.x; e < MT * NT * 1024; e += 256) {
        const int q = e >> 10, r = (e >> 6) & 15, l = e & 63;
        const float v = red[0][q][r][l] + red[1][q][r][l];
        const int mt = q / NT, nt = q - mt * NT;
        const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        out[(int64_t)row * a.N + nt * 32 + (l & 31)] = v;
    }
}

}  // namespace

extern "C" int dg_gemm_tn_f32(const float* a, int64_t lda, int64_t a_bs, const float* b, int64_t ldb, int64_t b_bs, float* c,
                              int32_t rows, int32_t M, int32_t N, int32_t batch, int32_t n_split, float* partial,
                              void* stream) {
    if (rows < 0 || batch < 0 || n_split < 1) return DG_EINVAL;
    if (M < 32 || N < 32 || (M & 31) || (N & 31) || (M / 32) * (N / 32) > 4) return DG_EINVAL;
    if (lda < M || ldb < N) return DG_EINVAL;
    if (batch == 0) return DG_OK;
    if (!a || !b || !c || (n_split > 1 && !partial)) return DG_EINVAL;
    if (n_split > 1 && !dg::aligned16(partial)) return DG_EALIGN;
    TnArgs t{a, b, n_split > 1 ? partial : c, lda, a_bs, ldb, b_bs, rows, M, N, batch, n_split,
             2 * dg::ceil_div(dg::ceil_div(rows, n_split), 2)};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t blocks = (int64_t)batch * n_split;
    if (blocks > 0x7fffffff) return DG_EINVAL;
    dim3 grid(static_cast<unsigned>(blocks)), block(256);
    const int mt = M / 32, nt = N / 32;
    if (mt == 1 && nt == 1) hipLaunchKernelGGL((gemm_tn_kernel<1, 1>), grid, block, 0, st, t);
    else if (mt == 2 && nt == 1) hipLaunchKernelGGL((gemm_tn_kernel<2, 1>), grid, block, 0, st, t);
    else if (mt == 1 && nt == 2) hipLaunchKernelGGL((gemm_tn_kernel<1, 2>), grid, block, 0, st, t);
    else if (mt == 2 && nt == 2) hipLaunchKernelGGL((gemm_tn_kernel<2, 2>), grid, block, 0, st, t);
    else if (mt == 4 && nt == 1) hipLaunchKernelGGL((gemm_tn_kernel<4, 1>), grid, block, 0, st, t);
    else if (mt == 1 && nt == 4) hipLaunchKernelGGL((gemm_tn_kernel<1, 4>), grid, block, 0, st, t);
    else if (mt == 3 && nt == 1) hipLaunchKernelGGL((gemm_tn_kernel<3, 1>), grid, block, 0, st, t);
    else if (mt == 1 && nt == 3) hipLaunchKernelGGL((gemm_tn_kernel<1, 3>), grid, block, 0, st, t);
    else return DG_EINVAL;
    int rc = dg::launch_status();
    if (rc != DG_OK || n_split == 1) return rc;
    // the split partials, summed in split order (dg_gcn_epilogue_f32 without flags)
    if (!dg::aligned16(c)) return DG_EALIGN;
    dg_epi_group g{partial, nullptr, n_split, 0};
    return dg_gcn_epilogue_f32(&g, 1, c, batch * M, N, 0, stream);
}

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
        if (d->reduce < 0) return DG_EINVAL;
        if (d->drop_state && (d->reduce <= 0 || !(d->drop_keep > 0.f && d->drop_keep <= 1.f))) return DG_EINVAL;
        if (d->drop_state && !d->b_map && (int64_t)d->batch * d->m * d->n >= 0xFFFFFFFFLL) return DG_EINVAL;
        g.reduce = d->reduce > 0 ? 1 : 0;
        g.drop_state = d->drop_state;
        g.drop_tag = d->drop_tag;
        g.drop_keep = d->drop_keep;
        if (g.reduce) bpw = d->reduce;
        g.batch_per_wave = bpw;
        g.block_begin = static_cast<int32_t>(blocks);
        blocks += (int64_t)g.tile_blocks * dg::ceil_div(d->batch, bpw);
        if (blocks > 0x7fffffff) return DG_EINVAL;
        const int kk = (d->k == 64 || d->k == 32) && !g.reduce ? d->k : 0;  // reduce: generic path
        kd = (kd < 0 || kd == kk) ? kk : 0;
    }
    if (A.n == 0) return DG_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // batch-reduce, K = 32, both operands contiguous along k, n <= 64, no scaling / map
    bool rk32 = true;
    int nt_max = 1;
    for (int i = 0; i < A.n && rk32; ++i) {
        const GemmOne& g = A.g[i];
        rk32 = g.reduce && g.k == 32 && g.a_sk == 1 && g.b_sk == 1 && g.n <= 64 && !g.sa && !g.sc &&
               (g.a_sm & 3) == 0 && (g.a_bs & 3) == 0 && (g.b_sn & 3) == 0 && (g.b_bs & 3) == 0 &&
               dg::aligned16(g.a) && dg::aligned16(g.b);
        nt_max = g.tiles_n > nt_max ? g.tiles_n : nt_max;
    }
    if (rk32) {
        int64_t rblocks = 0;
        for (int i = 0; i < A.n; ++i) {
            GemmOne& g = A.g[i];
            g.tile_blocks = dg::ceil_div(g.tiles_m, 4);  // 4 waves = 4 row tiles per block
            g.block_begin = static_cast<int32_t>(rblocks);
            rblocks += (int64_t)g.tile_blocks * dg::ceil_div(g.batch, g.batch_per_wave);
        }
        if (rblocks > 0x7fffffff) return DG_EINVAL;
        dim3 rgrid(static_cast<unsigned>(rblocks)), rblock(256);
        if (nt_max == 1)
            hipLaunchKernelGGL(gemm_f32_reduce_k32<1>, rgrid, rblock, 0, st, A);
        else
            hipLaunchKernelGGL(gemm_f32_reduce_k32<2>, rgrid, rblock, 0, st, A);
        return dg::launch_status();
    }
    // the projection shape (every descriptor): shared A, n <= 32 (a multiple of 4), K in
    // {32, 64}, unscaled, C rows 16-byte aligned and contiguous
    bool proj = kd > 0;
    for (int i = 0; i < A.n && proj; ++i) {
        const GemmOne& g = A.g[i];
        proj = g.a_bs == 0 && g.a_sk == 1 && (g.a_sm & 3) == 0 && dg::aligned16(g.a) &&
               g.n <= 32 && (g.n & 3) == 0 && !g.sa && !g.sc && g.c_sn == 1 && (g.c_sm & 3) == 0 &&
               (g.c_bs & 3) == 0 && dg::aligned16(g.c) && g.b_sn == 1 && (g.b_sk & 3) == 0 && (g.b_bs & 3) == 0 &&
               dg::aligned16(g.b);
    }
    constexpr int proj_blocks = 512;  // grid target (sweep 256-4,096 at config P: 512 fastest)
    if (proj) {
        // waves per block: the m tiles split evenly over ceil(tiles/8) blocks (>= 4 waves)
        int tiles_m_max = 0;
        for (int i = 0; i < A.n; ++i) tiles_m_max = A.g[i].tiles_m > tiles_m_max ? A.g[i].tiles_m : tiles_m_max;
        const int nbm = dg::ceil_div(tiles_m_max, 8);
        const int wpb = dg::ceil_div(tiles_m_max, nbm) < 4 ? 4 : dg::ceil_div(tiles_m_max, nbm);
        int64_t pblocks = 0;
        for (int i = 0; i < A.n; ++i) {
            GemmOne& g = A.g[i];
            g.tile_blocks = dg::ceil_div(g.tiles_m, wpb);
            // batches per block: about 2 blocks per CU of 256, amortising each wave's A fragment
            int bpb = 1;
            while (bpb < 64 && (int64_t)g.tile_blocks * dg::ceil_div(g.batch, bpb * 2) >= proj_blocks) bpb *= 2;  // <= 64: one map register
            g.batch_per_wave = bpb;
            g.block_begin = static_cast<int32_t>(pblocks);
            pblocks += (int64_t)g.tile_blocks * dg::ceil_div(g.batch, bpb);
        }
        dim3 pgrid(static_cast<unsigned>(pblocks)), pblock(64 * wpb);
        if (kd == 64)
            hipLaunchKernelGGL(gemm_f32_proj<64>, pgrid, pblock, 0, st, A);
        else
            hipLaunchKernelGGL(gemm_f32_proj<32>, pgrid, pblock, 0, st, A);
        return dg::launch_status();
    }
    dim3 grid(static_cast<unsigned>(blocks)), block(256);
    if (kd == 64)
        hipLaunchKernelGGL(gemm_f32_resident_a<64>, grid, block, 0, st, A);
    else if (kd == 32)
        hipLaunchKernelGGL(gemm_f32_resident_a<32>, grid, block, 0, st, A);
    else
        hipLaunchKernelGGL(gemm_f32_generic, grid, block, 0, st, A);
    return dg::launch_status();
}
