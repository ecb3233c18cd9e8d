// bf16 DEDICOM edge scores on gfx950's bf16 MFMA (BASELINE config 5: d = 256 bf16 embeddings
// and parameters, fp32 accumulation, every drug-drug relation slot's positive and negative
// batch in one launch).
//
// Replaces (paths relative to the reference root):
//   DecagonOptimizer.batch_predict for DEDICOM relations     decagon/deep/optimizer.py:63-85
//   (G = R global, L = D_k diagonal: model.py:130-134)
//
// For pair p of relation k = rel[p], u = row_table[row[p]], v = col_table[col[p]]:
//     score[p] = Σ_n ( Σ_i u_i D_k[i] R[i][n] ) D_k[n] v_n         (uᵀ·D_k·R·D_k·v)
//
// Workgroup (1024 threads, 768 at d = 256; one per CU: Rᵀ fills LDS) keeps Rᵀ in LDS — 16-byte slots XOR-
// swizzled by row, so the 32 lanes reading one k-slot of 32 consecutive rows hit 32 distinct
// slots — and its 16 waves loop over tiles of 32 pairs.  A tile is the transposed product
//     Tᵀ[n][p] = Σ_i Rᵀ[n][i] · (u_p ∘ D_k)[i]     on v_mfma_f32_32x32x16_bf16
// (A = Rᵀ from LDS, B = the pairs' scaled rows, built in registers once per tile and reused by
// all d/32 column tiles), so each lane ends owning ONE pair (its column p) and 16 n's of each
// column tile: the D_k·v epilogue reads 8-byte runs of the lane's own v and D_k rows.  The
// lane halves (n mod 8 < 4 or not) meet in one shuffle.  Pairs need not share a relation.
#include "common.h"
#include "decoder_tile.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16v8 __attribute__((ext_vector_type(8)));



__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// LDS-DMA of one dword per lane: lane t's dword at its own global address lands at LDS byte
// lds + 4 t (wave-uniform base).  Inline asm, so the compiler neither tracks nor drains it: the
// kernel retires it with its own s_waitcnt vmcnt.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds4(const void* src, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(lds)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}

constexpr int kCsThreads = 768;    // column-shared paired kernel: threads per workgroup (one per CU)
constexpr int kCs16Threads = 768;
  // config 5's 16x16x32 kernel (704: 208.6 vs 205.6 us)

struct Bf16DecArgs {
    const uint16_t* row_table;
    const uint16_t* col_table;
    const uint16_t* R;      // [d][d] row-major (R[i][n])
    const uint16_t* L;      // [n_rel][d] diagonals, or NULL (identity)
    const int32_t* rows;
    const int32_t* cols;
    const int32_t* rel;     // per pair, or NULL (relation 0)
    float* out;
    int64_t ld_row, ld_col;
    int32_t n_pairs, d;
    // FUSED (config 5's slot form, dg_slot_score_hinge_bf16): pair p < n_pairs is batch entry
    // p % batch of local slot p / batch (relation slot0 + p / batch); its negative row is
    // alias draw slot0·batch + p of that slot's table (written to neg_out), and the hinge terms
    // of every pair pair are summed into loss (per-workgroup partials, ticket, block order)
    const uint2* alias;
    int64_t alias_stride;
    uint64_t seed;
    int32_t* neg_out;
    float* loss;
    float* partial;
    uint32_t* ticket;
    int32_t range, slot0, batch;
    float margin;
};

// threads per workgroup: 16 waves, but 12 at d = 256 (its 16 B-operand fragments need the
// registers of a 3-waves-per-SIMD allocation); one workgroup per CU either way (Rᵀ in LDS)
template <int D>
constexpr int threads_for() { return D == 256 ? 768 : 1024; }

// HAS_L: per-relation diagonals present (DEDICOM) — a template flag, so no load sits behind a
// branch (a runtime `if (L)` split every load into its own basic block, each waited on alone)
// R (D x D bf16, row-major) into LDS, row i's 16-byte slot q at rs[i*SL + (q ^ (i % SL))]: every
// load of the thread's share issued before its first LDS store (a load-store-per-iteration loop
// waits one L2 round trip per slot: 11 in a row at D = 256 and 768 threads, before any work).
template <int D, int THREADS>
__device__ __forceinline__ void stage_r(uint4* rs, const uint16_t* R) {
    constexpr int SL = D / 8, N = D * SL, PER = (N + THREADS - 1) / THREADS, B = 4;
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += B) {  // B slots in flight per thread
        uint4 t[B];
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const int e = (int)threadIdx.x + (k0 + k) * THREADS;
            t[k] = (k0 + k < PER && e < N) ? *reinterpret_cast<const uint4*>(R + (int64_t)e * 8) : uint4{};
        }
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const int e = (int)threadIdx.x + (k0 + k) * THREADS;
            if (k0 + k < PER && e < N) {
                const int i = e / SL, q = e - i * SL;  // row e / SL, slot e % SL
                rs[i * SL + (q ^ (i % SL))] = t[k];
            }
        }
    }
}

template <int D, bool HAS_L>
__global__ __launch_bounds__(threads_for<D>()) void decoder_bf16_kernel(const Bf16DecArgs a) {
    constexpr int kThreads = threads_for<D>();
    constexpr int KS = D / 16;  // k-steps of 16
    constexpr int NT = D / 32;  // column tiles of 32
    constexpr int SL = D / 8;   // 16-byte slots per Rᵀ row
    extern __shared__ uint4 rt[];  // Rᵀ: row n, slot q (k = 8q .. 8q+7) at rt[n*SL + (q ^ (n % SL))]
    const int tid = threadIdx.x;
    // stage Rᵀ: thread handles (n, q) slots; reads R[8q + j][n], j < 8 (column gather, once)
    for (int e = tid; e < D * SL; e += kThreads) {
        const int n = e / SL, q = e - n * SL;
        uint16_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = a.R[(int64_t)(8 * q + j) * D + n];
        uint4 w;
        w.x = v[0] | (uint32_t)v[1] << 16;
        w.y = v[2] | (uint32_t)v[3] << 16;
        w.z = v[4] | (uint32_t)v[5] << 16;
        w.w = v[6] | (uint32_t)v[7] << 16;
        rt[n * SL + (q ^ (n % SL))] = w;
    }
    __syncthreads();

    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 31;
    const int h = lane >> 5;
    const int n_tiles = (a.n_pairs + 31) / 32;
    const int stride = gridDim.x * (kThreads / 64);
#pragma unroll 1
    for (int tile = blockIdx.x * (kThreads / 64) + wave; tile < n_tiles; tile += stride) {
        const int p = tile * 32 + r;
        const bool valid = p < a.n_pairs;
        const int pr = valid ? a.rows[p] : 0;
        const int pc = valid ? a.cols[p] : 0;
        const int pk = (valid && a.rel) ? a.rel[p] : 0;
        const uint16_t* u = a.row_table + (int64_t)pr * a.ld_row;
        const uint16_t* v = a.col_table + (int64_t)pc * a.ld_col;
        const uint16_t* lk = HAS_L ? a.L + (int64_t)pk * D : nullptr;
        // B operand: (u ∘ D_k)[16s + 8h + j] in bf16, s < KS
        bf16x8 bf[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint4 uu = *reinterpret_cast<const uint4*>(u + 16 * s + 8 * h);
            uint4 ll = make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u);  // bf16 1.0
            if (HAS_L) ll = *reinterpret_cast<const uint4*>(lk + 16 * s + 8 * h);
            const uint32_t uw[4] = {uu.x, uu.y, uu.z, uu.w}, lw[4] = {ll.x, ll.y, ll.z, ll.w};
            bf16v8 x;  // round-to-nearest-even by the cast (v_cvt_pk_bf16_f32)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                x[2 * j] = (__bf16)(bf_lo(uw[j]) * bf_lo(lw[j]));
                x[2 * j + 1] = (__bf16)(bf_hi(uw[j]) * bf_hi(lw[j]));
            }
            bf[s] = valid ? __builtin_bit_cast(bf16x8, x) : bf16x8{};
        }
        float part = 0.f;
        // two column tiles at a time: two independent accumulator chains, so each MFMA's
        // operand read and its predecessor's result are not on one serial path.  The tile
        // pair's v runs are loaded before its MFMAs (their latency hides behind them).
        // Row gathers, not MFMAs, bound this kernel: every pair reads its own u and v rows,
        // 32 distinct cache lines per wave load, so loads are kept 16 bytes wide.
#pragma unroll 1
        for (int t = 0; t < NT; t += 2) {
            // Column tiles t, t+1 = n in [32t, 32t + 64).  The A rows are permuted so that lane
            // half h ends owning the 32 CONTIGUOUS n = 32t + 32h + [0, 32): acc0 register j holds
            // n = 32t + 32h + j, acc1 register j holds n + 16 — the epilogue then reads 64-byte
            // runs of v and D_k (4 × 16 B per lane) instead of eight 8-byte pieces each.
            const int nb0 = 32 * t + 32 * h;
            uint4 ev[4], el[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) ev[i] = *reinterpret_cast<const uint4*>(v + nb0 + 8 * i);
            // A row m = r holds C row m = (j&3) + 8(j>>2) + 4h' for register j of lane half h'
            const int na = 32 * t + 32 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3), nb = na + 16;
            f32x16 acc0 = {}, acc1 = {};
            uint4 wa = rt[na * SL + (h ^ (na % SL))];
            uint4 wb = rt[nb * SL + (h ^ (nb % SL))];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                uint4 xa = wa, xb = wb;
                if (s + 1 < KS) {  // the next k-step's Rᵀ fragments, one MFMA pair ahead
                    const int q = 2 * (s + 1) + h;
                    xa = rt[na * SL + (q ^ (na % SL))];
                    xb = rt[nb * SL + (q ^ (nb % SL))];
                }
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wa), bf[s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wb), bf[s], acc1, 0, 0, 0);
                wa = xa;
                wb = xb;
            }
            // D_k's run after the MFMAs: the pairs of a tile mostly share a relation, so these
            // loads hit one line (and registers stay within 3 waves per SIMD)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                el[i] = HAS_L ? *reinterpret_cast<const uint4*>(lk + nb0 + 8 * i)
                              : make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const f32x16& acc = u ? acc1 : acc0;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const uint4 vv = ev[2 * u + i], ll = el[2 * u + i];
                    const uint32_t vw[4] = {vv.x, vv.y, vv.z, vv.w}, lw[4] = {ll.x, ll.y, ll.z, ll.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        part = fmaf(acc[8 * i + 2 * j], bf_lo(lw[j]) * bf_lo(vw[j]), part);
                        part = fmaf(acc[8 * i + 2 * j + 1], bf_hi(lw[j]) * bf_hi(vw[j]), part);
                    }
                }
            }
        }
        part = dg::xor_add<32>(part);
        if (h == 0 && valid) a.out[p] = part;
    }
}


// Paired layout (config 5): a positive (u_p, v) and its negative (u_n, v) share
// v and D_k, so uᵀ·D_k·R·D_k·v = (u ∘ D_k)ᵀ · T with T = R·(D_k ∘ v) computed ONCE for both:
//     T[i][p] = Σ_n R[i][n] · bf16(D_k[n] v_n)      on v_mfma_f32_32x32x16_bf16
// (A = R rows from LDS, B = the pairs' scaled v rows, built once per tile), then
//     pos[p] = Σ_i u_p[i] D_k[i] T[i][p],   neg[p] = Σ_i u_n[i] D_k[i] T[i][p]
// in the epilogue (fp32; a product of two bf16 values is exact in fp32) — half the MFMAs of
// contracting each pair's row side on its own (round 3's first half: one wave scored the
// positive and negative tiles with two MFMA chains, 128 B-operand VGPRs, 2 waves per SIMD:
// 311.7 µs against 221.7 µs for this form), one accumulator chain, and 64 B-operand VGPRs,
// so 3 waves per SIMD hide the row gathers.  The A rows are permuted as above: lane half h
// owns the 16 contiguous i = 32t + 16h + [0, 16) of column tile t (32-byte runs of u_p, u_n
// and D_k).  The bf16 operand rounding sits on D_k∘v instead of u∘D_k: the scores agree with
// the row-side kernels to bf16 operand rounding, not bitwise.
template <int D, bool HAS_L, int THREADS, bool FUSED>
__global__ __launch_bounds__(THREADS) void decoder_bf16_colshared_kernel(const Bf16DecArgs a) {
    constexpr int KS = D / 16;
    constexpr int NT = D / 32;
    constexpr int SL = D / 8;
    extern __shared__ uint4 rs[];  // R: row i, slot q (n = 8q .. 8q+7) at rs[i*SL + (q ^ (i % SL))]
    const int tid = threadIdx.x;
    stage_r<D, THREADS>(rs, a.R);
    __syncthreads();

    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 31;
    const int h = lane >> 5;
    const int nh = a.n_pairs;  // pairs per half
    const int n_tiles = (nh + 31) / 32;
    const int stride = gridDim.x * (THREADS / 64);
    const uint4 ones = make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u);  // bf16 1.0
    float wsum = 0.f;  // FUSED: this wave's hinge terms, its tiles in order
    // a tile's indices (rows, column, relation; FUSED: the negative's alias entry) are loaded one
    // tile ahead, so a tile's row gathers do not wait behind its index loads
    struct Idx {
        int prp, pc, pk, prn, j;
        float u;
        uint2 e;
    };
    auto fetch = [&](int tl, Idx& x) {
        const int p = tl * 32 + r;
        const bool ok = tl < n_tiles && p < nh;
        x.prp = ok ? a.rows[p] : 0;
        x.pc = ok ? a.cols[p] : 0;
        if constexpr (FUSED) {
            x.pk = ok ? a.slot0 + p / a.batch : 0;
            dg::unigram_pick(a.range, a.seed, (uint64_t)a.slot0 * (uint64_t)a.batch + (uint64_t)p, x.j, x.u);
            x.e = ok ? a.alias[x.pk * a.alias_stride + x.j] : make_uint2(0u, 0u);
        } else {
            x.pk = (ok && a.rel) ? a.rel[p] : 0;
            x.prn = ok ? a.rows[nh + p] : 0;
        }
    };
    Idx nxt;
    // tile order: round-major, then wave, then workgroup (tile = k·stride + wave·grid + block),
    // so the last, partial round's tiles land one per workgroup on as many CUs as there are
    // tiles — not all on the first few workgroups, where 12 waves would share each CU's MFMA
    const int first = wave * (int)gridDim.x + (int)blockIdx.x;
    fetch(first, nxt);
#pragma unroll 1
    for (int tile = first; tile < n_tiles; tile += stride) {
        const int p = tile * 32 + r;
        const bool valid = p < nh;
        const Idx cur = nxt;
        fetch(tile + stride, nxt);
        const int prp = cur.prp, pc = cur.pc, pk = cur.pk;
        int prn;
        if constexpr (FUSED) {
            prn = valid ? dg::unigram_take(cur.j, cur.u, cur.e) : 0;
            if (valid && h == 0) a.neg_out[p] = prn;
        } else {
            prn = cur.prn;
        }
        const uint16_t* up = a.row_table + (int64_t)prp * a.ld_row;
        const uint16_t* un = a.row_table + (int64_t)prn * a.ld_row;
        const uint16_t* v = a.col_table + (int64_t)pc * a.ld_col;
        const uint16_t* lk = HAS_L ? a.L + (int64_t)pk * D : nullptr;
        // B operand: bf16(D_k ∘ v)[16s + 8h + j], s < KS
        bf16x8 b[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint4 vv = *reinterpret_cast<const uint4*>(v + 16 * s + 8 * h);
            const uint4 ll = HAS_L ? *reinterpret_cast<const uint4*>(lk + 16 * s + 8 * h) : ones;
            const uint32_t vw[4] = {vv.x, vv.y, vv.z, vv.w}, lw[4] = {ll.x, ll.y, ll.z, ll.w};
            bf16v8 x;  // round-to-nearest-even by the cast (v_cvt_pk_bf16_f32)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                x[2 * j] = (__bf16)(bf_lo(vw[j]) * bf_lo(lw[j]));
                x[2 * j + 1] = (__bf16)(bf_hi(vw[j]) * bf_hi(lw[j]));
            }
            b[s] = valid ? __builtin_bit_cast(bf16x8, x) : bf16x8{};
        }
        float partp = 0.f, partn = 0.f;
#pragma unroll 1
        for (int t = 0; t < NT; ++t) {
            // lane half h owns i = 32t + 16h + [0, 16): register j of the accumulator.  The
            // epilogue's row runs are issued before the MFMAs (their latency hides behind them).
            const int ib0 = 32 * t + 16 * h;
            uint4 ep[2], en[2], el[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                ep[k] = *reinterpret_cast<const uint4*>(up + ib0 + 8 * k);
                en[k] = *reinterpret_cast<const uint4*>(un + ib0 + 8 * k);
            }
            // A row m = r holds C row m = (j&3) + 8(j>>2) + 4h' of register j, lane half h'
            const int ia = 32 * t + 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3);
            f32x16 acc = {};
            uint4 wa = rs[ia * SL + (h ^ (ia % SL))];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                uint4 xa = wa;
                if (s + 1 < KS) xa = rs[ia * SL + ((2 * (s + 1) + h) ^ (ia % SL))];
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wa), b[s], acc, 0, 0, 0);
                wa = xa;
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) el[k] = HAS_L ? *reinterpret_cast<const uint4*>(lk + ib0 + 8 * k) : ones;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t pw[4] = {ep[k].x, ep[k].y, ep[k].z, ep[k].w},
                               nw[4] = {en[k].x, en[k].y, en[k].z, en[k].w},
                               lw[4] = {el[k].x, el[k].y, el[k].z, el[k].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float l0 = bf_lo(lw[j]), l1 = bf_hi(lw[j]);
                    partp = fmaf(acc[8 * k + 2 * j], bf_lo(pw[j]) * l0, partp);
                    partp = fmaf(acc[8 * k + 2 * j + 1], bf_hi(pw[j]) * l1, partp);
                    partn = fmaf(acc[8 * k + 2 * j], bf_lo(nw[j]) * l0, partn);
                    partn = fmaf(acc[8 * k + 2 * j + 1], bf_hi(nw[j]) * l1, partn);
                }
            }
        }
        partp = dg::xor_add<32>(partp);
        partn = dg::xor_add<32>(partn);
        if (h == 0 && valid) {
            a.out[p] = partp;
            a.out[nh + p] = partn;
        }
        if constexpr (FUSED) {  // relu(neg − (pos − margin)), optimizer.py:116-120: a fixed butterfly
            float term = (h == 0 && valid) ? fmaxf(partn - (partp - a.margin), 0.f) : 0.f;
            term = dg::xor_add<1>(dg::xor_add<2>(dg::xor_add<4>(dg::xor_add<8>(dg::xor_add<16>(dg::xor_add<32>(term))))));
            wsum += term;
        }
    }
    if constexpr (FUSED) {
        // the workgroup's partial (its waves in order) is published write-through and drained,
        // then a ticket; the last workgroup adds every partial in block order (sc1 loads, no L2
        // write-back or invalidate — decoder_hinge_kernel's hand-off) and resets the ticket
        __shared__ float red[THREADS / 64];
        __shared__ int last;
        if (lane == 0) red[wave] = wsum;
        __syncthreads();
        if (tid == 0) {
            float s = 0.f;
            for (int w = 0; w < THREADS / 64; ++w) s += red[w];
            __hip_atomic_store(a.partial + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        }
        __syncthreads();
        if (last && tid < 64) {  // wave 0 of the last workgroup
            const float t = dg::block_order_sum(a.partial, (int)gridDim.x, lane);
            if (tid == 0) {
                a.loss[0] = t;
                __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// Config 5's fused step on v_mfma_f32_16x16x32_bf16 (dg_slot_score_hinge_bf16; d = 256, every
// 32-pair tile inside one relation slot).  Same arithmetic as the column-shared kernel above —
// T = R·bf16(D_k∘v) once per (positive, negative) pair, pos / neg = (u∘D_k)ᵀ·T in fp32 — but
// laid out for the load path, which bounds that kernel (PMC on the MI355X: TA busy 74 %, TD
// 82 % of the kernel, MFMA 22 %, waves parked on memory 60 %): there a row load instruction
// spans 32 pairs x 32 B, here 16 pairs x 64 B (the 16x16x32 B operand gives a pair's 4 lane
// groups 8 consecutive k each), and D_k — one relation per tile — is read from LDS (one
// coalesced 512-B load per tile) instead of by 32 of the 80 row loads.
//   wave tile = 32 pairs as two 16-pair halves b (pair 16b + (lane & 15)); lane group g = lane >> 4
//   B[b][s] = bf16(D_k ∘ v)[32s + 8g + j]                         (8 k-steps of 32, 64 VGPRs)
//   M-tile t of T (16 rows): row m holds i(t, m) = 32(t>>1) + 8(m>>2) + 4(t&1) + (m&3), so the
//   accumulator rows of lane group g over tiles 2q, 2q+1 are i = 32q + 8g + [0, 8) — one 16-B
//   load of u_p, u_n and D_k each per two tiles, a pair's 4 lanes reading 64 contiguous bytes
//   A = R rows i(t, m) from LDS (XOR-swizzled 16-B slots), each fragment feeding both halves.
// FUSED = false: the paired scores alone (dg_decoder_score_bf16_paired's form: given negative
// rows, a relation per pair, D_k — or identity — read per lane from global memory); the same
// arithmetic in the same order, so the fused step and its three-launch decomposition agree bit
// for bit.
// FUSED's load path (round 5): the row loads are issued pair-major — lane 4P + c
// reads 16-B chunk c' of pair P's 64-B run, so each quad of lanes reads one row's contiguous
// 64 B — and moved to the MFMA layout (lane 16g + p <- the lane holding pair p's chunk g) by 4
// ds_bpermute per 16 B.  A row load in the MFMA layout, a quad spanning four rows, costs the
// texture path ≈ 60 cycles an instruction against ≈ 17 for a quad reading one run
// (scripts/ta_probe.hip): TA busy 96 M → 35 M per launch.  The chunk order is rotated by 2 in
// pairs 8-15 of a half, so the 32 source lanes of each half-wave's bpermute are distinct mod 32.
// The next tile's indices (rows, columns, alias entries, the draws' j / u, the D_k row) go to
// LDS by LDS-DMA instead of 14 VGPRs, which pays for loading both 64-B halves of the u rows'
// 128-B lines at once (two q per loop iteration).
template <int THREADS, bool FUSED>
__global__ __launch_bounds__(THREADS) void decoder_bf16_cs16_kernel(const Bf16DecArgs a) {
    constexpr int D = 256;
    constexpr int SL = D / 8;                 // 16-byte slots per R row
    constexpr int WAVES = THREADS / 64;
    // FUSED: per wave two index buffers of kIB bytes — rows[32] cols[32] alias.x[32]
    // alias.y[32] j[32] u[32] (i32 / f32), then the tile's D_k row (512 B)
    constexpr int kIB = 1280;
    extern __shared__ uint4 rs[];  // R: row i, slot q at rs[i*SL + (q ^ (i % SL))]; then the index buffers
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    char* ibase = reinterpret_cast<char*>(rs + D * SL) + wave * 2 * kIB;
    const int pl = lane & 15;                   // the lane's pair in each half
    const int g = lane >> 4;                    // its k / row group
    const int ml = FUSED ? lane >> 2 : pl;      // the pair this lane's row loads read
    const int mc = FUSED ? ((lane & 3) + 2 * (lane >> 5)) & 3 : g;  // and their 16-B chunk
    const int xsrc = 4 * (4 * pl + ((g + 2 * (pl >> 3)) & 3));      // FUSED: bpermute source (bytes)
                                                                     // of MFMA lane (g, pl)
    auto xp = [&](const uint4 v) {
        if constexpr (!FUSED) return v;
        return make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.x),
                          (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.y),
                          (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.z),
                          (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.w));
    };
    const int nh = a.n_pairs;
    const int n_tiles = (nh + 31) / 32;
    const int stride = gridDim.x * WAVES;
    // (the host checks that both tables fit 32-bit byte offsets)
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.row_table), 0, 0x7fffffff, 0x00020000);
    const auto crs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.col_table), 0, 0x7fffffff, 0x00020000);
    float wsum = 0.f;
    const uint4 ones = make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u);  // bf16 1.0
    struct Idx {
        int prp[2], pc[2], j[2];  // (non-FUSED: j = the given negative row)
        float u[2];
        uint2 e[2];               // (non-FUSED: e.x = the pair's relation)
    };
    // non-FUSED: tile tl's indices into registers, one tile ahead
    auto fetch = [&](int tl, Idx& x) {
        const bool okt = tl < n_tiles;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int p = tl * 32 + 16 * b + pl;
            const bool ok = okt && p < nh;
            x.prp[b] = ok ? a.rows[p] : 0;
            x.pc[b] = ok ? a.cols[p] : 0;
            x.j[b] = ok ? a.rows[nh + p] : 0;
            x.e[b] = make_uint2((ok && a.rel) ? (uint32_t)a.rel[p] : 0u, 0u);
        }
    };
    // FUSED: tile tl's indices into index buffer buf by LDS-DMA (the draws' j, u by ds_write),
    // one tile ahead; a tile never straddles slots
    auto prefetch = [&](int tl, int buf) {
        const int tc = tl < n_tiles ? tl : 0;  // (past the end: tile 0's addresses, never read)
        const int pk = a.slot0 + (tc * 32) / a.batch;
        char* B = ibase + buf * kIB;
        const int i = lane & 31;
        const int p = tc * 32 + i;
        glds4((lane < 32 ? a.rows : a.cols) + p, lds_addr(B));
        int j;
        float u;
        dg::unigram_pick(a.range, a.seed, (uint64_t)a.slot0 * (uint64_t)a.batch + (uint64_t)p, j, u);
        glds4(reinterpret_cast<const uint32_t*>(a.alias + pk * a.alias_stride + j) + (lane >> 5), lds_addr(B + 256));
        const uint32_t* dsrc = reinterpret_cast<const uint32_t*>(a.L + (int64_t)pk * D) + lane;
        glds4(dsrc, lds_addr(B + 768));
        glds4(dsrc + 64, lds_addr(B + 1024));
        if (lane < 32) {
            reinterpret_cast<int*>(B + 512)[i] = j;
            reinterpret_cast<float*>(B + 640)[i] = u;
        }
    };
    Idx nxt;
    const int first = wave * (int)gridDim.x + (int)blockIdx.x;  // round-major tile order (see above)
    if constexpr (FUSED) prefetch(first, 0);
    stage_r<D, THREADS>(rs, a.R);
    if constexpr (FUSED) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the DMA is not tracked)
    __syncthreads();
    if constexpr (!FUSED) fetch(first, nxt);
    int cur_buf = 0;
#pragma unroll 1
    for (int tile = first; tile < n_tiles; tile += stride) {
        Idx cur;
        const uint4* dkt = nullptr;  // FUSED: this tile's D_k row in LDS
        if constexpr (FUSED) {
            const char* B = ibase + cur_buf * kIB;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int i = 16 * b + ml;
                cur.prp[b] = reinterpret_cast<const int*>(B)[i];
                cur.pc[b] = reinterpret_cast<const int*>(B + 128)[i];
                cur.e[b] = make_uint2(reinterpret_cast<const uint32_t*>(B + 256)[i],
                                      reinterpret_cast<const uint32_t*>(B + 384)[i]);
                cur.j[b] = reinterpret_cast<const int*>(B + 512)[i];
                cur.u[b] = reinterpret_cast<const float*>(B + 640)[i];
            }
            dkt = reinterpret_cast<const uint4*>(B + 768);
            prefetch(tile + stride, cur_buf ^ 1);
        } else {
            cur = nxt;
            fetch(tile + stride, nxt);
        }
        const uint16_t* lk[2];  // non-FUSED: each half's pairs' D_k rows (NULL: identity)
        // rows through buffer loads from the uniform table bases: a 32-bit byte offset per row
        // (1 VGPR) instead of a 64-bit address (2)
        int up[2], un[2];
        bool valid[2];
        bf16x8 bq[2][8];
        uint4 vv[2][8];
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // every v load first (16 in flight), then the B operand
            const int p = tile * 32 + 16 * b + pl;
            valid[b] = p < nh;
            const int pm = tile * 32 + 16 * b + ml;  // the pair this lane's loads read
            const bool vm = pm < nh;
            int prn;
            if constexpr (FUSED) {
                prn = vm ? dg::unigram_take(cur.j[b], cur.u[b], cur.e[b]) : 0;
                if (vm && mc == 0) a.neg_out[pm] = prn;
            } else {
                prn = cur.j[b];
                lk[b] = a.L ? a.L + (int64_t)cur.e[b].x * D + 8 * g : nullptr;
            }
            up[b] = 2 * (cur.prp[b] * (int)a.ld_row + 8 * mc);
            un[b] = 2 * (prn * (int)a.ld_row + 8 * mc);
            const int vo = 2 * (cur.pc[b] * (int)a.ld_col + 8 * mc);
#pragma unroll
            for (int s = 0; s < 8; ++s)
                vv[b][s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(crs, vo + 64 * s, 0, 0));
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            uint4 llf = ones;
            if constexpr (FUSED) llf = dkt[4 * s + g];  // D_k[32s + 8g .. +8], shared by both halves
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                uint4 ll = llf;
                if constexpr (!FUSED) ll = lk[b] ? *reinterpret_cast<const uint4*>(lk[b] + 32 * s) : ones;
                const uint32_t lw[4] = {ll.x, ll.y, ll.z, ll.w};
                const uint4 vt = xp(vv[b][s]);
                const uint32_t vw[4] = {vt.x, vt.y, vt.z, vt.w};
                bf16v8 x;  // round-to-nearest-even by the cast (v_cvt_pk_bf16_f32)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    x[2 * j] = (__bf16)(bf_lo(vw[j]) * bf_lo(lw[j]));
                    x[2 * j + 1] = (__bf16)(bf_hi(vw[j]) * bf_hi(lw[j]));
                }
                bq[b][s] = valid[b] ? __builtin_bit_cast(bf16x8, x) : bf16x8{};
            }
        }
        float pp[2] = {0.f, 0.f}, pn[2] = {0.f, 0.f};
        // M-tiles 2q, 2q+1: rows i = 32q + 8g + [0, 8) of this lane group; ep / en: the lane's
        // 16 B of u_p / u_n at those rows
        auto qbody = [&](const int q, const uint4 (&ep)[2], const uint4 (&en)[2]) {
            f32x4 acc[2][2] = {};

            // the row's swizzle key, opaque per iteration: its 16 slot offsets are q-invariant,
            // and hoisted out of the loop they hold 16 VGPRs (spilled at 3 waves per SIMD)
            int key = 8 * (pl >> 2) + (pl & 3);
            asm volatile("" : "+v"(key));
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // M-tile t = 2q + h: A row m = pl -> i(t, m)
                const int ia = 32 * q + 4 * h + key;  // i % SL = 4h + key
                const int kx = 4 * h + key;
                uint4 wa = rs[ia * SL + (g ^ kx)];
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    uint4 xa = wa;
                    if (s + 1 < 8) xa = rs[ia * SL + ((4 * (s + 1) + g) ^ kx)];
                    acc[0][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa), bq[0][s],
                                                                        acc[0][h], 0, 0, 0);
                    acc[1][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa), bq[1][s],
                                                                        acc[1][h], 0, 0, 0);
                    wa = xa;
                    __builtin_amdgcn_sched_barrier(0);  // one A fragment ahead, no deeper
                }
                // (keeps the second tile's A reads from being hoisted above the first tile's
                // MFMAs: 64 more live VGPRs, spilled at 3 waves per SIMD)
                __builtin_amdgcn_sched_barrier(0);
            }
            uint4 elf = ones;
            if constexpr (FUSED) elf = dkt[4 * q + g];  // D_k[32q + 8g .. +8]
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                uint4 el = elf;
                if constexpr (!FUSED) el = lk[b] ? *reinterpret_cast<const uint4*>(lk[b] + 32 * q) : ones;
                const uint32_t lw[4] = {el.x, el.y, el.z, el.w};
                const uint4 ept = xp(ep[b]), ent = xp(en[b]);
                const uint32_t pw[4] = {ept.x, ept.y, ept.z, ept.w};
                const uint32_t nw[4] = {ent.x, ent.y, ent.z, ent.w};
#pragma unroll
                for (int h = 0; h < 2; ++h) {  // accumulator register r of tile 2q + h is row 32q + 8g + 4h + r
#pragma unroll
                    for (int r2 = 0; r2 < 2; ++r2) {  // elements 4h + 2r2, 4h + 2r2 + 1: word 2h + r2
                        const float l0 = bf_lo(lw[2 * h + r2]), l1 = bf_hi(lw[2 * h + r2]);
                        // (D_k∘T)[i] once for both rows: 2 products instead of 4
                        const float t0 = acc[b][h][2 * r2] * l0, t1 = acc[b][h][2 * r2 + 1] * l1;
                        pp[b] = fmaf(t0, bf_lo(pw[2 * h + r2]), pp[b]);
                        pp[b] = fmaf(t1, bf_hi(pw[2 * h + r2]), pp[b]);
                        pn[b] = fmaf(t0, bf_lo(nw[2 * h + r2]), pn[b]);
                        pn[b] = fmaf(t1, bf_hi(nw[2 * h + r2]), pn[b]);
                    }
                }
                // Each half's sums pass through an opaque copy, so the compiler cannot pair
                // the two halves' chains into packed fp32 ops (as it does in the FUSED form
                // without this).  The paired form multiplies u_p[i]·D_k[i] of both halves by
                // `v_pk_mul_f32 D, A, B op_sel:[0,1]` (low result from src1's high dword), and
                // on the MI355X that instruction intermittently returned 0 for lanes 48-63 in
                // this kernel: every wrong score (~2 % of half tiles per launch) is the right
                // one minus exactly one such product of lane group 3 (DESIGN.md §5,
                // scripts/hazard_match.py).  tests/test_cpu_isa.py keeps the form out of the
                // library.
                asm volatile("" : "+v"(pp[b]), "+v"(pn[b]));
            }
        };
        auto uload = [&](int off) {
            return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rrs, off, 0, 0));
        };
        if constexpr (FUSED) {
#pragma unroll 1
            for (int q = 0; q < 8; q += 2) {  // both 64-B halves of the pairs' 128-B lines at once
                uint4 ep0[2], en0[2], ep1[2], en1[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    ep0[b] = uload(up[b] + 64 * q);
                    ep1[b] = uload(up[b] + 64 * q + 64);
                    en0[b] = uload(un[b] + 64 * q);
                    en1[b] = uload(un[b] + 64 * q + 64);
                }
                qbody(q, ep0, en0);
                qbody(q + 1, ep1, en1);
            }
        } else {
#pragma unroll 1
            for (int q = 0; q < 8; ++q) {
                uint4 ep[2], en[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    ep[b] = uload(up[b] + 64 * q);
                    en[b] = uload(un[b] + 64 * q);
                }
                qbody(q, ep, en);
            }
        }
        if constexpr (FUSED) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's index DMA landed
            cur_buf ^= 1;
        }
        float term = 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // the pair's 4 lane groups, in a fixed butterfly
            pp[b] = dg::xor_add<32>(dg::xor_add<16>(pp[b]));
            pn[b] = dg::xor_add<32>(dg::xor_add<16>(pn[b]));
            const int p = tile * 32 + 16 * b + pl;
            if (g == 0 && valid[b]) {
                a.out[p] = pp[b];
                a.out[nh + p] = pn[b];
            }
            if (FUSED && g == 0 && valid[b]) term += fmaxf(pn[b] - (pp[b] - a.margin), 0.f);  // optimizer.py:116-120
        }
        if constexpr (FUSED) {
            term = dg::xor_add<1>(dg::xor_add<2>(dg::xor_add<4>(dg::xor_add<8>(dg::xor_add<16>(dg::xor_add<32>(term))))));
            wsum += term;
        }
    }
    if constexpr (!FUSED) return;
    // the workgroup's partial (its waves in order), write-through + drained, then a ticket; the
    // last workgroup adds every partial in block order (decoder_bf16_colshared_kernel's hand-off)
    __shared__ float red[WAVES];
    __shared__ int last;
    if (lane == 0) red[wave] = wsum;
    __syncthreads();
    if (tid == 0) {
        float t = 0.f;
        for (int w = 0; w < WAVES; ++w) t += red[w];
        __hip_atomic_store(a.partial + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && tid < 64) {  // wave 0 of the last workgroup
        const float t = dg::block_order_sum(a.partial, (int)gridDim.x, lane);
        if (tid == 0) {
            a.loss[0] = t;
            __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
}  // namespace

extern "C" int dg_decoder_score_bf16(const uint16_t* row_table, int64_t ld_row, const uint16_t* col_table,
                                     int64_t ld_col, const int32_t* row_idx, const int32_t* col_idx,
                                     const int32_t* rel_idx, int32_t n_pairs, const uint16_t* G,
                                     const uint16_t* l_table, int32_t d, float* out, void* stream) {
    if (n_pairs < 0 || !row_table || !col_table || !row_idx || !col_idx || !G || !out) return DG_EINVAL;
    if (d != 64 && d != 128 && d != 256) return DG_EINVAL;
    if (ld_row < d || ld_col < d || (ld_row & 7) || (ld_col & 7)) return DG_EALIGN;
    if (!dg::aligned16(row_table) || !dg::aligned16(col_table) || (l_table && !dg::aligned16(l_table)))
        return DG_EALIGN;
    if (n_pairs == 0) return DG_OK;
    Bf16DecArgs a{row_table, col_table, G, l_table, row_idx, col_idx, rel_idx, out, ld_row, ld_col, n_pairs, d};
    const int n_tiles = (n_pairs + 31) / 32;
    const int waves = (d == 256 ? 768 : 1024) / 64;
    int blocks = (n_tiles + waves - 1) / waves;
    if (blocks > 256) blocks = 256;  // persistent: one Rᵀ-holding workgroup per CU
    const int lds = d * d * 2;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    static std::atomic<uint64_t> configured_l{0}, configured_nl{0};
    dg::lds_optin(reinterpret_cast<const void*>(&decoder_bf16_kernel<256, true>), 160 * 1024, configured_l);
    dg::lds_optin(reinterpret_cast<const void*>(&decoder_bf16_kernel<256, false>), 160 * 1024, configured_nl);
#define DG_DEC_LAUNCH(DD, HL) \
    hipLaunchKernelGGL((decoder_bf16_kernel<DD, HL>), dim3(blocks), dim3(threads_for<DD>()), lds, st, a)
    const bool hl = l_table != nullptr;
    if (d == 256) {
        if (hl) DG_DEC_LAUNCH(256, true); else DG_DEC_LAUNCH(256, false);
    } else if (d == 128) {
        if (hl) DG_DEC_LAUNCH(128, true); else DG_DEC_LAUNCH(128, false);
    } else {
        if (hl) DG_DEC_LAUNCH(64, true); else DG_DEC_LAUNCH(64, false);
    }
#undef DG_DEC_LAUNCH
    return dg::launch_status();
}

// The 16x16x32 kernel's row loads are buffer loads with 32-bit byte offsets.
static bool fits_32bit_offsets(int64_t n_rows, int64_t ld) { return n_rows * ld * 2 < 0x7fffffffLL; }

extern "C" int dg_decoder_score_bf16_paired(const uint16_t* row_table, int64_t ld_row, int64_t n_row_table,
                                            const uint16_t* col_table, int64_t ld_col, int64_t n_col_table,
                                            const int32_t* row_idx, const int32_t* col_idx,
                                            const int32_t* rel_idx, int32_t n_half, const uint16_t* G,
                                            const uint16_t* l_table, int32_t d, float* out, void* stream) {
    if (n_half < 0 || !row_table || !col_table || !row_idx || !col_idx || !G || !out) return DG_EINVAL;
    if (n_row_table < 1 || n_col_table < 1) return DG_EINVAL;
    if (d != 64 && d != 128 && d != 256) return DG_EINVAL;
    if (ld_row < d || ld_col < d || (ld_row & 7) || (ld_col & 7)) return DG_EALIGN;
    if (!dg::aligned16(row_table) || !dg::aligned16(col_table) || (l_table && !dg::aligned16(l_table)))
        return DG_EALIGN;
    if (n_half == 0) return DG_OK;
    Bf16DecArgs a{row_table, col_table, G, l_table, row_idx, col_idx, rel_idx, out, ld_row, ld_col, n_half, d};
    const int n_tiles = (n_half + 31) / 32;
    const int lds = d * d * 2;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (!dg::aligned16(G)) return DG_EALIGN;  // R rows are staged into LDS in 16-byte pieces
    if (d == 256 && fits_32bit_offsets(n_row_table, ld_row) && fits_32bit_offsets(n_col_table, ld_col)) {
        // the 16x16x32 form (decoder_bf16_cs16_kernel, FUSED = false): bit-identical scores to
        // dg_slot_score_hinge_bf16's; 32-bit byte offsets into the tables are required
        constexpr int kT16 = kCs16Threads;
        const int lds16 = d * d * 2;  // R
        int blocks16 = (n_tiles + kT16 / 64 - 1) / (kT16 / 64);
        if (blocks16 > 256) blocks16 = 256;
        static std::atomic<uint64_t> configured16p{0};
        dg::lds_optin(reinterpret_cast<const void*>(&decoder_bf16_cs16_kernel<kT16, false>), lds16, configured16p);
        hipLaunchKernelGGL((decoder_bf16_cs16_kernel<kT16, false>), dim3(blocks16), dim3(kT16), lds16, st, a);
        return dg::launch_status();
    }
    constexpr int kThreads = kCsThreads;
    static std::atomic<uint64_t> configured_l{0}, configured_nl{0};
    dg::lds_optin(reinterpret_cast<const void*>(&decoder_bf16_colshared_kernel<256, true, kThreads, false>),
                  160 * 1024, configured_l);
    dg::lds_optin(reinterpret_cast<const void*>(&decoder_bf16_colshared_kernel<256, false, kThreads, false>),
                  160 * 1024, configured_nl);
#define DG_DEC_LAUNCH(DD, HL) \
    hipLaunchKernelGGL((decoder_bf16_colshared_kernel<DD, HL, kThreads, false>), dim3(blocks), dim3(kThreads), lds, \
                       st, a)
    int blocks = (n_tiles + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 256) blocks = 256;  // persistent: one R-holding workgroup per CU
    const bool hl = l_table != nullptr;
    if (d == 256) {
        if (hl) DG_DEC_LAUNCH(256, true); else DG_DEC_LAUNCH(256, false);
    } else if (d == 128) {
        if (hl) DG_DEC_LAUNCH(128, true); else DG_DEC_LAUNCH(128, false);
    } else {
        if (hl) DG_DEC_LAUNCH(64, true); else DG_DEC_LAUNCH(64, false);
    }
#undef DG_DEC_LAUNCH
    return dg::launch_status();
}

extern "C" int dg_slot_score_hinge_bf16(const uint16_t* row_table, int64_t ld_row, int64_t n_row_table,
                                        const uint16_t* col_table, int64_t ld_col, int64_t n_col_table,
                                        const int32_t* pos_rows, const int32_t* pos_cols,
                                        const uint32_t* alias_table, int32_t range, int64_t alias_stride,
                                        int32_t slot0, int32_t n_slots, int32_t batch, uint64_t seed,
                                        const uint16_t* G, const uint16_t* l_table, int32_t d, float margin,
                                        float* out, int32_t* neg_rows, float* loss, void* workspace,
                                        void* stream) {
    if (n_slots < 0 || batch < 1 || slot0 < 0 || range < 1 || alias_stride < 0) return DG_EINVAL;
    if (n_row_table < range || n_col_table < 1) return DG_EINVAL;
    if (!row_table || !col_table || !pos_rows || !pos_cols || !alias_table || !G || !l_table || !out ||
        !neg_rows || !loss || !workspace)
        return DG_EINVAL;
    if (d != 256) return DG_EINVAL;
    if (ld_row < d || ld_col < d || (ld_row & 7) || (ld_col & 7)) return DG_EALIGN;
    if (!dg::aligned16(row_table) || !dg::aligned16(col_table) || !dg::aligned16(l_table) || !dg::aligned16(G) ||
        !dg::aligned16(workspace))
        return DG_EALIGN;
    if ((int64_t)n_slots * batch > 0x7fffffffLL) return DG_EINVAL;
    const int32_t nh = n_slots * batch;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (nh == 0) return hipMemsetAsync(loss, 0, sizeof(float), st) == hipSuccess ? DG_OK : DG_EINVAL;
    Bf16DecArgs a{row_table, col_table, G, l_table, pos_rows, pos_cols, nullptr, out, ld_row, ld_col, nh, d};
    a.alias = reinterpret_cast<const uint2*>(alias_table);
    a.alias_stride = alias_stride;
    a.seed = seed;
    a.neg_out = neg_rows;
    a.loss = loss;
    a.ticket = reinterpret_cast<uint32_t*>(workspace);
    a.partial = reinterpret_cast<float*>(workspace) + 4;
    a.range = range;
    a.slot0 = slot0;
    a.batch = batch;
    a.margin = margin;
    constexpr int kThreads = kCsThreads;
    const int n_tiles = (nh + 31) / 32;
    int blocks = (n_tiles + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > DG_HINGE_WS_BLOCKS) blocks = DG_HINGE_WS_BLOCKS;  // persistent; the workspace's partials
    // the 16x16x32 form: every 32-pair tile inside one slot (one D_k), tables within 32-bit
    // byte offsets (its row loads are buffer loads)
    if (batch % 32 == 0 && fits_32bit_offsets(n_row_table, ld_row) && fits_32bit_offsets(n_col_table, ld_col)) {
        constexpr int kT16 = kCs16Threads;
        const int lds16 = d * d * 2 + (kT16 / 64) * 2 * 1280;  // R + per wave two index buffers
        int blocks16 = (n_tiles + kT16 / 64 - 1) / (kT16 / 64);
        if (blocks16 > DG_HINGE_WS_BLOCKS) blocks16 = DG_HINGE_WS_BLOCKS;
        static std::atomic<uint64_t> configured16{0};
        dg::lds_optin(reinterpret_cast<const void*>(&decoder_bf16_cs16_kernel<kT16, true>), lds16, configured16);
        hipLaunchKernelGGL((decoder_bf16_cs16_kernel<kT16, true>), dim3(blocks16), dim3(kT16), lds16, st, a);
        return dg::launch_status();
    }
    // the opt-in is the dynamic R buffer exactly: the kernel's static LDS (the hinge partials)
    // comes on top of it, and static + dynamic must stay within the CU's 160 KB
    static std::atomic<uint64_t> configured{0};
    dg::lds_optin(reinterpret_cast<const void*>(&decoder_bf16_colshared_kernel<256, true, kThreads, true>),
                  d * d * 2, configured);
    hipLaunchKernelGGL((decoder_bf16_colshared_kernel<256, true, kThreads, true>), dim3(blocks), dim3(kThreads),
                       d * d * 2, st, a);
    return dg::launch_status();
}
