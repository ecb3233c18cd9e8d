// Config 5 (BASELINE configs[4]) scorer: bf16 DEDICOM scores of every relation slot's
// positive batch and its degree^0.75 negatives, d = 256, on gfx950's bf16 MFMA.
//
// Replaces (paths relative to the reference root), for every DEDICOM relation slot at once:
//   tf.nn.fixed_unigram_candidate_sampler(..., unigrams=degrees[i][k])   decagon/deep/optimizer.py:38-47
//   batch_predict(row_inputs / neg_samples, col_inputs) with G = R (global interaction) and
//   L = D_k (the slot's local variation): diag(u·D_k·R·D_k·vᵀ)             optimizer.py:51-57, 63-85,
//                                                                          model.py:130-134
//
// Per slot s the score of a pair (u, v) is
//     score = Σ_n T_s[u][n] · D_s[n] · v[n],      T_s = E · (D_s ∘ R)   (rows of R scaled by D_s)
// T_s is computed ONCE per slot for every row of the row table — 32-row tiles on
// v_mfma_f32_32x32x16_bf16 — instead of once per pair: a slot's 2B pairs draw their rows from
// n_rows drugs (config 5: 1,024 pairs over 645 drugs, 672 rows padded), so this issues
// n_rows/2B of the per-pair contraction's MFMA work and reads E and R as contiguous tiles.
//
// Work unit = (slot s, row tile t), slot-major; a persistent workgroup (4 waves, two per CU)
// walks a contiguous range of units.  On entering a slot it
//   1. draws the slot's B negatives from the slot's own alias table (counter (slot0+s)·B + i, so
//      the draws do not depend on the sharding) and writes them out,
//   2. buckets the slot's 2B pairs by row tile in LDS (counting sort: LDS integer atomics; the
//      order inside a bucket is free — every pair's score is computed alone, in a fixed order),
//   3. builds its B operands: wave w owns output columns [64w, 64w+64) (two 32-column blocks),
//      lane (r, h) holds bf16(D_s[k]·R[k][n]) for k = 16σ + 8h + j, n = 64w + 32cb + r — 128
//      VGPRs, kept for every tile of the slot.
// Per unit: the E tile (32 rows) goes to LDS (16-byte pieces XOR-swizzled by row, so the A
// fragment reads are conflict-free), 2 × 16 MFMAs per wave, T'[m][n] = T[m][n]·D_s[n] to LDS,
// then 16-lane groups score the tile's bucket: lane q of a group dots T'[u][16q, 16q+16) with
// v[16q, 16q+16) (v loaded before the MFMAs), a 4-step DPP fold, lane 15 writes the score.
// Numerics: the products D_s[k]·R[k][n] are rounded to bf16 (the MFMA operand), everything
// after is fp32; tests/test_gpu_config5.py restates exactly that in float64.
#include "common.h"
#include "decoder_tile.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16v8 __attribute__((ext_vector_type(8)));

constexpr int kD = 256;           // embedding width (config 5)
constexpr int kThreads = 256;     // 4 waves: wave w owns T columns [64w, 64w + 64)
constexpr int kTile = 32;         // rows per tile (one MFMA M block)
constexpr int kMaxTiles = 32;     // n_rows <= 1024
constexpr int kTStride = kD + 4;  // T' row stride (floats): rows land 4 banks apart
constexpr int kPre = 3;           // rounds of v rows loaded before the MFMAs (16 pairs per round)

struct SlotArgs {
    const uint16_t* row_table;
    const uint16_t* col_table;
    const uint16_t* Rt;      // [d][d], Rt[n][k] = R[k][n]
    const uint16_t* D;       // [*][d] slot diagonals, indexed by GLOBAL slot id
    const int32_t* pos_rows; // [n_slots * B], local slots, slot-major
    const int32_t* pos_cols;
    const uint2* alias;      // slot (slot0 + s)'s table at alias + (slot0 + s) * alias_stride
    int32_t* neg_rows;       // [n_slots * B]
    float* out;              // [2 * n_slots * B]: positives, then negatives
    uint64_t seed;
    int64_t alias_stride;
    int64_t ld_row, ld_col;
    int32_t n_rows, range, batch, slot0, n_slots, n_tiles;
    int64_t n_units;
};

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// lane l += lane l - S of its 16-lane row (DPP row_shr:S, zero from outside the row)
template <int S>
__device__ __forceinline__ float row_shr_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x110 + S, 0xF, 0xF, true));
}

// dot of T'[ul][16q, 16q + 16) (LDS) with the bf16 v piece (two 16-B loads)
__device__ __forceinline__ float piece_dot(const float* trow, int q, const uint4& v0, const uint4& v1) {
    const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // rotate the four 16-B reads by q / 4 so the 16 lanes of a group hit 16 distinct bank sets
        const int c = (i + (q >> 2)) & 3;
        const float4 t = *reinterpret_cast<const float4*>(trow + 16 * q + 4 * c);
        s = fmaf(t.x, bf_lo(w[2 * c]), s);
        s = fmaf(t.y, bf_hi(w[2 * c]), s);
        s = fmaf(t.z, bf_lo(w[2 * c + 1]), s);
        s = fmaf(t.w, bf_hi(w[2 * c + 1]), s);
    }
    return s;
}

__global__ __launch_bounds__(kThreads, 2) void slot_scorer_kernel(const SlotArgs a) {
    __shared__ uint4 etile[kTile * kD / 8];         // 16 KB, piece q of row m at m*32 + (q ^ (m & 15))
    __shared__ float tt[kTile * kTStride];          // 33,280 B: T'
    __shared__ uint32_t ent[2048];                  // the slot's pairs, then bucketed
    __shared__ uint32_t srt[2048];
    __shared__ int cnt[kMaxTiles + 1];
    __shared__ int off[kMaxTiles + 1];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 31;
    const int h = lane >> 5;
    const int g = tid >> 4;  // pair group (16 lanes)
    const int q = tid & 15;
    const int B = a.batch;
    const int NT = a.n_tiles;
    const int64_t per = a.n_units / gridDim.x, extra = a.n_units % gridDim.x;
    const int64_t u0 = blockIdx.x * per + min<int64_t>(blockIdx.x, extra);
    const int64_t u1 = u0 + per + (blockIdx.x < extra ? 1 : 0);

    bf16x8 rs0[16], rs1[16];
    float dn0 = 0.f, dn1 = 0.f;
    int cur = -1;
    const uint16_t* dk = nullptr;
#pragma unroll 1
    for (int64_t unit = u0; unit < u1; ++unit) {
        const int s = (int)(unit / NT);
        const int t = (int)(unit - (int64_t)s * NT);
        if (s != cur) {  // block-uniform
            cur = s;
            const int sg = a.slot0 + s;
            dk = a.D + (int64_t)sg * kD;
            __syncthreads();  // the previous slot's buckets are no longer read
            if (tid <= kMaxTiles) cnt[tid] = 0;
            __syncthreads();
            const uint2* tab = a.alias + (int64_t)sg * a.alias_stride;
            for (int p = tid; p < 2 * B; p += kThreads) {
                const int i = p < B ? p : p - B;
                const int64_t pi = (int64_t)s * B + i;
                const int v = a.pos_cols[pi];
                int u;
                if (p < B) {
                    u = a.pos_rows[pi];
                } else {
                    u = dg::unigram_draw(tab, a.range, a.seed, (uint64_t)sg * B + i);
                    a.neg_rows[pi] = u;  // every block visiting the slot writes the same value
                }
                const int bin = u >> 5;
                atomicAdd(&cnt[bin], 1);
                ent[p] = (uint32_t)p | ((uint32_t)(u & 31) << 11) | ((uint32_t)v << 16);
                srt[p] = (uint32_t)bin;  // (scratch: the bin, read back below)
            }
            __syncthreads();
            if (tid == 0) {
                int acc = 0;
                for (int b = 0; b < NT; ++b) {
                    off[b] = acc;
                    acc += cnt[b];
                    cnt[b] = off[b];  // the scatter cursor
                }
                off[NT] = acc;
            }
            __syncthreads();
            uint32_t mine[8];  // (2B <= 2048: at most 8 pairs per thread)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int p = tid + kThreads * k;
                mine[k] = p < 2 * B ? srt[p] : 0u;
            }
            __syncthreads();  // the bins are read before srt is overwritten
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int p = tid + kThreads * k;
                if (p < 2 * B) srt[atomicAdd(&cnt[mine[k]], 1)] = ent[p];
            }
            // the slot's B operands: bf16(D_s[k] · R[k][n]), n = 64w + 32cb + r, k = 16σ + 8h + j
            // (32-bit byte offsets from the uniform bases: one VGPR per address, nothing hoisted)
            const char* rtb = reinterpret_cast<const char*>(a.Rt);
            const char* dkb = reinterpret_cast<const char*>(dk);
            uint32_t o0 = (uint32_t)((64 * wave + r) * kD) * 2u;
            asm volatile("" : "+v"(o0));  // opaque here: its addresses are not hoisted out of the unit loop
#pragma unroll
            for (int sg2 = 0; sg2 < 16; ++sg2) {
                const uint32_t k0 = (uint32_t)(16 * sg2 + 8 * h) * 2u;
                const uint4 dd = *reinterpret_cast<const uint4*>(dkb + k0);
                const uint4 x0 = *reinterpret_cast<const uint4*>(rtb + (o0 + k0));
                const uint4 x1 = *reinterpret_cast<const uint4*>(rtb + (o0 + 32u * kD * 2u + k0));
                const uint32_t dw[4] = {dd.x, dd.y, dd.z, dd.w};
                const uint32_t w0[4] = {x0.x, x0.y, x0.z, x0.w};
                const uint32_t w1[4] = {x1.x, x1.y, x1.z, x1.w};
                bf16v8 y0, y1;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    y0[2 * j] = (__bf16)(bf_lo(w0[j]) * bf_lo(dw[j]));
                    y0[2 * j + 1] = (__bf16)(bf_hi(w0[j]) * bf_hi(dw[j]));
                    y1[2 * j] = (__bf16)(bf_lo(w1[j]) * bf_lo(dw[j]));
                    y1[2 * j + 1] = (__bf16)(bf_hi(w1[j]) * bf_hi(dw[j]));
                }
                rs0[sg2] = __builtin_bit_cast(bf16x8, y0);
                rs1[sg2] = __builtin_bit_cast(bf16x8, y1);
                // keep the loads of later steps from being hoisted above (their registers
                // would join the 128 the operands hold)
                if ((sg2 & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
            const uint16_t dd0 = dk[64 * wave + r], dd1 = dk[64 * wave + 32 + r];
            dn0 = __uint_as_float((uint32_t)dd0 << 16);
            dn1 = __uint_as_float((uint32_t)dd1 << 16);
            __syncthreads();  // buckets complete
        }
        // ---- the E tile (rows 32t .. 32t+31, clamped) into LDS, swizzled
        {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int P = tid + kThreads * i;
                const int m = P >> 5, qq = P & 31;
                const int row = min(kTile * t + m, a.n_rows - 1);
                const uint4 v = *reinterpret_cast<const uint4*>(a.row_table + (int64_t)row * a.ld_row + 8 * qq);
                etile[m * 32 + (qq ^ (m & 15))] = v;
            }
        }
        // the first rounds' v pieces of this tile's bucket, loaded now (their latency hides
        // under the MFMAs)
        const int b0 = off[t], b1 = off[t + 1];
        uint4 pv[kPre][2];
        uint32_t pe[kPre];
#pragma unroll
        for (int k = 0; k < kPre; ++k) {
            const int e = b0 + g + 16 * k;
            pe[k] = e < b1 ? srt[e] : 0u;
            const uint16_t* vr = a.col_table + (int64_t)(pe[k] >> 16) * a.ld_col + 16 * q;
            pv[k][0] = e < b1 ? *reinterpret_cast<const uint4*>(vr) : make_uint4(0, 0, 0, 0);
            pv[k][1] = e < b1 ? *reinterpret_cast<const uint4*>(vr + 8) : make_uint4(0, 0, 0, 0);
        }
        __syncthreads();  // the E tile is in LDS
        f32x16 acc0 = {}, acc1 = {};
        // A fragments read two k-steps ahead of their MFMAs (the scheduling barriers keep the
        // compiler from hoisting all sixteen reads: their registers would spill the operands)
        bf16x8 av[3];
        av[0] = __builtin_bit_cast(bf16x8, etile[r * 32 + ((0 + h) ^ (r & 15))]);
        av[1] = __builtin_bit_cast(bf16x8, etile[r * 32 + ((2 + h) ^ (r & 15))]);
#pragma unroll
        for (int sg2 = 0; sg2 < 16; ++sg2) {
            if (sg2 + 2 < 16) {
                const int qq = 2 * (sg2 + 2) + h;
                av[(sg2 + 2) % 3] = __builtin_bit_cast(bf16x8, etile[r * 32 + (qq ^ (r & 15))]);
            }
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[sg2 % 3], rs0[sg2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[sg2 % 3], rs1[sg2], acc1, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        // T'[m][n] = T[m][n] · D_s[n]; register j of lane half h holds row (j&3) + 8(j>>2) + 4h
        {
            const int n0 = 64 * wave + r, n1 = n0 + 32;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int m = (j & 3) + 8 * (j >> 2) + 4 * h;
                tt[m * kTStride + n0] = acc0[j] * dn0;
                tt[m * kTStride + n1] = acc1[j] * dn1;
            }
        }
        __syncthreads();  // T' complete
        const int64_t nb = (int64_t)a.n_slots * B;
#pragma unroll
        for (int k = 0; k < kPre; ++k) {
            const int e = b0 + g + 16 * k;
            if (e >= b1) break;  // (16-lane-group uniform)
            const uint32_t en = pe[k];
            float sc = piece_dot(tt + (int)((en >> 11) & 31) * kTStride, q, pv[k][0], pv[k][1]);
            sc = row_shr_add<8>(sc);
            sc = row_shr_add<4>(sc);
            sc = row_shr_add<2>(sc);
            sc = row_shr_add<1>(sc);
            if (q == 15) {
                const int p = (int)(en & 2047);
                a.out[(p < B ? 0 : nb) + (int64_t)s * B + (p < B ? p : p - B)] = sc;
            }
        }
#pragma unroll 1
        for (int e = b0 + g + 16 * kPre; e < b1; e += 16) {  // rare overflow rounds
            const uint32_t en = srt[e];
            const uint16_t* vr = a.col_table + (int64_t)(en >> 16) * a.ld_col + 16 * q;
            const uint4 v0 = *reinterpret_cast<const uint4*>(vr), v1 = *reinterpret_cast<const uint4*>(vr + 8);
            float sc = piece_dot(tt + (int)((en >> 11) & 31) * kTStride, q, v0, v1);
            sc = row_shr_add<8>(sc);
            sc = row_shr_add<4>(sc);
            sc = row_shr_add<2>(sc);
            sc = row_shr_add<1>(sc);
            if (q == 15) {
                const int p = (int)(en & 2047);
                a.out[(p < B ? 0 : nb) + (int64_t)s * B + (p < B ? p : p - B)] = sc;
            }
        }
        __syncthreads();  // T' and the E tile are free for the next unit
    }
}

}  // namespace

extern "C" int dg_slot_scores_bf16(const uint16_t* row_table, int64_t ld_row, int32_t n_rows,
                                   const uint16_t* col_table, int64_t ld_col, int32_t n_cols,
                                   const uint16_t* Rt, const uint16_t* D, int32_t d,
                                   const int32_t* pos_rows, const int32_t* pos_cols, int32_t n_slots,
                                   int32_t batch, int32_t slot0, const uint32_t* alias_table, int32_t range,
                                   int64_t alias_stride, uint64_t seed, int32_t* neg_rows, float* out,
                                   void* stream) {
    if (!row_table || !col_table || !Rt || !D || !pos_rows || !pos_cols || !alias_table || !neg_rows || !out)
        return DG_EINVAL;
    if (d != kD) return DG_EINVAL;
    if (n_slots < 0 || batch < 1 || 2 * batch > 2048 || slot0 < 0 || alias_stride < 0) return DG_EINVAL;
    if (n_rows < 1 || n_rows > kTile * kMaxTiles || n_cols < 1 || n_cols > 65535) return DG_EINVAL;
    if (range < 1 || range > n_rows) return DG_EINVAL;
    if (ld_row < d || ld_col < d || (ld_row & 7) || (ld_col & 7)) return DG_EALIGN;
    if (!dg::aligned16(row_table) || !dg::aligned16(col_table) || !dg::aligned16(Rt) || !dg::aligned16(D) ||
        !dg::aligned16(alias_table))
        return DG_EALIGN;
    if (n_slots == 0) return DG_OK;
    SlotArgs a{};
    a.row_table = row_table;
    a.col_table = col_table;
    a.Rt = Rt;
    a.D = D;
    a.pos_rows = pos_rows;
    a.pos_cols = pos_cols;
    a.alias = reinterpret_cast<const uint2*>(alias_table);
    a.neg_rows = neg_rows;
    a.out = out;
    a.seed = seed;
    a.alias_stride = alias_stride;
    a.ld_row = ld_row;
    a.ld_col = ld_col;
    a.n_rows = n_rows;
    a.range = range;
    a.batch = batch;
    a.slot0 = slot0;
    a.n_slots = n_slots;
    a.n_tiles = (n_rows + kTile - 1) / kTile;
    a.n_units = (int64_t)n_slots * a.n_tiles;
    int blocks = 512;  // two 58-KB workgroups per CU
    if (a.n_units < blocks) blocks = static_cast<int>(a.n_units);
    hipLaunchKernelGGL(slot_scorer_kernel, dim3(blocks), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       a);
    return dg::launch_status();
}
