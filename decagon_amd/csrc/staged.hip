// LDS-staged relation SpMM for gfx950 (MI355X): groups with many relations over a narrow
// column space (polypharmacy drug×drug: 1,928 relations of 645×645).
//
// Reference ops replaced: tf.sparse_tensor_dense_matmul(adj_mats[edge_type][k], x) and
// tf.add_n (decagon/deep/layers.py:90-92, :114-116) for such groups.
//
// Why: gathering 16-byte pieces of random 256-byte X rows through L1/L2/Infinity Cache
// saturates at ~11 TB/s of gathered bytes on MI355X whatever the L2 hit rate,
// and every nonzero gathers a full row.  Here a workgroup copies each relation's dense
// operand slice into LDS once and every nonzero gathers from LDS (ds_read_b128).
//
// Layout (decagon_amd/sparse.py: staged_layout): per relation, a long row becomes a group of
// ≤ 8 equal-length segments ("virtual rows", zero-padded), groups sorted by length and kept
// inside one 64-lane wave, and each wave's nonzeros a dense diagonal-major block [rlw][64]
// (rlw a multiple of 4; holes are zero pairs on one of sixteen zero columns, one per bank
// class, so a hole never collides with a nonzero's bank slot).  Thread i owns virtual row i, so at diagonal m the
// 64 threads of a wave read 64 consecutive (col, value) pairs — one coalesced 512-byte load
// straight from global memory at woff + 64m + lane, no table and no test, prefetched four
// diagonals ahead in registers (the next relation's first four before the barrier).  The
// relation tables (woff, rlw, vinfo) come from global memory a relation ahead.  Each lane's
// nonzeros are placed on diagonals by the host (layout.cpp: a bipartite edge colouring per
// ds_read_b128 lane group) so the group's 16 lanes gather from distinct bank slots wherever
// the relation allows.
//
// Workgroup = 1024 threads, one per (output chunk c, 16-float column slice s), ONE barrier per
// relation: the slab slice X_slab(k)[:, 16s .. +16) and k's tables live in one of two LDS
// buffers (columns 80 B apart: the bank slot of float4 j of column v is (5v+j) mod 16, plus
// an all-zero column n_cols for padding pairs):
//   for relation k of the chunk:
//     [barrier: relation k-1's gathers are done, relation k's slab buffer is complete]
//     relation k+1's slab slice (prefetched into registers during k-1) → the other buffer;
//     prefetch relation k+2's; load relation k+1's tables
//     thread i: part = Σ_{m < len[i]} val · xs[col]   (4 × ds_read_b128 + 16 fmaf per nonzero)
//     a group's segments are folded by a DPP shift tree; its first lane does
//     acc[row] += part (one writer per row per relation)
//   out[c][r][16s .. +16) = acc[r]
// Fixed summation order, no atomics: bitwise reproducible.
#include "common.h"

namespace {

constexpr int kMaxThreads = 1024;
constexpr int kLdsBytes = 160 * 1024;
constexpr int kMetaInts = 256;  // a chunk's tables: jm offsets (nk + 1) and slabs (nk), nk <= 64
constexpr int kDummyRow = 1023;
constexpr int kMaxVarChunks = DG_STAGED_MAX_CHUNKS;  // variable output chunks a group (kernarg table)
#ifdef DG_STAGED_PROF
constexpr int kProfSlots = 6;  // per wave: barrier, put+prefetch, tables, gather, accumulate, relations
#endif

struct StagedGroupK {
    const int2* pairs;
    const int32_t* jm;
    const int32_t* jmoff;
    const int32_t* slab;
    const float* x;
    float* out;
    int32_t x_ld;
    int32_t n_rows;
    int32_t n_cols;
    int32_t n_rels;
    int32_t out_chunk;
    int32_t n_out_chunks;
    int32_t n_slices;
    int32_t block_begin;
    int32_t n_blocks;
    int32_t var;       // 1: chunk c is relations [cstart[c], cstart[c + 1]) (variable sizes)
    // PROJ form: the slab of relation k is H · W[slab(k)] (H [n_cols][64], W [K][64][d]),
    // computed in the workgroup on the fp32 MFMA instead of read from x
    const float* h;
    const float* w;
    int32_t h_ld;
    int32_t pad2;
    // var form: the output chunks' first relations (kernarg: a block-uniform scalar read, no
    // dependent global load before the chunk's tables)
    uint16_t cstart[kMaxVarChunks + 1];
};

struct StagedArgs {
    StagedGroupK g[DG_MAX_GROUPS];
    int32_t n_groups;
    int32_t d;
    int32_t xs_f4;     // float4 slots of one slab buffer (+ the zero column)
    int32_t acc_f4;    // float4 slots of the accumulator
    int32_t acc_st;    // float4 slots per accumulator row: 5 (80 B, bank slot (5·row + j) mod 16,
                       // a bijection of row & 15) when LDS allows, else 4
    int32_t pad;
#ifdef DG_STAGED_PROF
    unsigned long long* prof;  // per block, per wave: kProfSlots counters (see DG_TICK below)
#endif
};

// Async global->LDS copy of 16 bytes per lane (global_load_lds_dwordx4): lane t's float4 at
// base + voff lands at LDS byte lds + 16 t.  Inline asm, so the compiler neither tracks it
// nor drains it with vmcnt(0) at the next global-load use or barrier (cdna_hip_programming.md
// "Pipelining across barriers"): the kernel retires it with a counted s_waitcnt itself.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const float* base, uint32_t voff, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :: "v"(voff), "s"(base), "s"(lds) : "memory", "m0");
}
#pragma clang diagnostic pop

// Relation barrier: this wave's slab copies are retired (every VMEM op but the last four —
// the next relation's first pair loads, always issued last — is complete) and its LDS ops
// are done; then s_barrier.
__device__ __forceinline__ void relation_barrier() {
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// lane l += lane l + S of its 16-lane row (DPP row_shl:S), where S < the lane's group size
template <int S>
__device__ __forceinline__ void fold_step(float4 (&part)[4], int gsz) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float* v = reinterpret_cast<float*>(&part[q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float o = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(v[e]), 0x100 + S, 0xF, 0xF, true));
            if (S < gsz) v[e] += o;
        }
    }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool PROJ>
__global__ __launch_bounds__(kMaxThreads) void spmm_staged_kernel(const StagedArgs a) {
    extern __shared__ float4 lds[];
    const int tid = threadIdx.x;
    const int T = blockDim.x;
    const int b = blockIdx.x;
    int gi = 0;
#pragma unroll 1
    while (gi + 1 < a.n_groups && b >= a.g[gi + 1].block_begin) ++gi;
    const StagedGroupK& g = a.g[gi];
    // XCD-contiguous item map (see spmm.hip): the slices of one chunk run on one XCD, so the
    // chunk's pairs come from HBM once and are re-read from that XCD's L2.
    const int lb = b - g.block_begin;
    const int per = g.n_blocks >> 3;
    const int item = (lb & 7) * per + (lb >> 3);
    if (item >= g.n_out_chunks * g.n_slices) return;  // block-uniform, before any barrier
    const int c = item / g.n_slices;
    const int s = item - c * g.n_slices;
    const int d = a.d;
    const int col0 = s * 16;
    const int n_rows = g.n_rows;
    const int n_cols = g.n_cols;
    const int k0 = g.var ? static_cast<int>(g.cstart[c]) : c * g.out_chunk;
    const int nk = g.var ? static_cast<int>(g.cstart[c + 1]) - k0
                         : min(g.out_chunk, g.n_rels - k0);  // relations of this chunk
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // LDS: xs[2] (columns 0..n_cols-1, then the zero column) | meta | acc
    float4* xs0 = lds;  // buffer 0 at offset 0
    int* jof = reinterpret_cast<int*>(xs0 + 2 * a.xs_f4);
    int* slb = jof + (nk + 1);
    float4* acc = reinterpret_cast<float4*>(jof + kMetaInts);

    for (int i = tid; i <= nk; i += T) jof[i] = g.jmoff[k0 + i];
    for (int i = tid; i < nk; i += T) slb[i] = g.slab ? g.slab[k0 + i] : k0 + i;
    const int ast = a.acc_st;
    for (int i = tid; i < n_rows * ast; i += T) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    // the sixteen zero columns n_cols .. n_cols + 15 (one per bank class) that holes read
    if (tid < 128) xs0[(tid >> 6) * a.xs_f4 + (n_cols + ((tid >> 2) & 15)) * 5 + (tid & 3)] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();

    // relation i's slab slice -> buffer i & 1 by glds: slot q of the buffer (column v = q / 5,
    // float4 j = q mod 5, j = 4 the pad slot: any valid source) — columns 80 B apart, so the
    // 16-byte bank slot of float4 j of column v is (5v + j) mod 16, a bijection of v & 15 for
    // every j.  Wave w copies slots 64(w + 16r) .. +63; the zero column is never written.
    const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(xs0));
    auto slab_copy = [&](int i) {
        const float* xk = g.x + (int64_t)__builtin_amdgcn_readfirstlane(slb[i]) * n_cols * g.x_ld + col0;
        const uint32_t dst = lds0 + (i & 1) * a.xs_f4 * 16;
        const int n5 = n_cols * 5;
        // unrolled (n_cols <= 1024: at most five rounds): the copies issue back to back
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            const int q0 = 64 * wave + 1024 * r;
            const int q = q0 + lane;
            const int v = (q * 52429) >> 18;  // q / 5 (q < 5120)
            const int j = min(q - 5 * v, 3);
            const int off = __umul24(v, g.x_ld) + min(col0 + 4 * j, d - 4) - col0;
            if (q < n5) glds16(xk, off * 4, dst + q0 * 16);
        }
    };
    // PROJ: relation i's slab slice computed on the fp32 MFMA — slabᵀ[n][v] = Σ_k W[k][col0 + n]
    // H[v][k] on v_mfma_f32_16x16x4_f32 (A = W slice: lane l holds W[16q + m][col0 + (l & 15)],
    // q = l >> 4, for MFMA m; B = Hᵀ: H[v][16q + m] for its tile's row v = 16t + (l & 15); the
    // contraction order k = 16q + m is free), so lane l ends with slab[v][col0 + 4q .. +3] —
    // one ds_write_b128 into the buffer's row v.  Wave w makes 16-row tiles w, w + 16, ...; the
    // W slice (16 floats per lane) is loaded a relation ahead, H rows come from L2.
    const int pq = lane >> 4, pn = lane & 15;
    auto load_w = [&](int i, float (&wa)[16]) {
        const int sl = __builtin_amdgcn_readfirstlane(slb[i]);
        const float* w = g.w + ((int64_t)sl * 64 + 16 * pq) * d + min(col0 + pn, d - 1);
#pragma unroll
        for (int m = 0; m < 16; ++m) wa[m] = w[m * d];
    };
    // one 16-row tile at a time (measured: two tiles with interleaved accumulators made the
    // layer-2 launch 10 us slower — their MFMAs then crowd the gathers of the SIMD's other waves)
    auto slab_make = [&](int i, const float (&wa)[16]) {
        float4* buf = xs0 + (i & 1) * a.xs_f4;
        const int n_tiles = (n_cols + 15) >> 4;
#pragma unroll 1
        for (int t = wave; t < n_tiles; t += kMaxThreads / 64) {
            const int v = 16 * t + pn;
            const float4* hp = reinterpret_cast<const float4*>(g.h + (int64_t)min(v, n_cols - 1) * g.h_ld + 16 * pq);
            float4 hv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) hv[j] = hp[j];
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[4 * j], hv[j].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[4 * j + 1], hv[j].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[4 * j + 2], hv[j].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[4 * j + 3], hv[j].w, acc, 0, 0, 0);
            }
            if (v < n_cols) buf[v * 5 + pq] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
    };
    // relation i's tables, straight from global memory (L2-resident, read a relation ahead):
    // this wave's pair block (woff, rlw diagonals), its largest group, this lane's vinfo
    // (read unconditionally — jm ends with 1024 spare ints; used only by waves with rlw > 0)
    auto tables = [&](int i, int& woff, int& rlw, int& big, int& vi) {
        const int32_t* t = g.jm + __builtin_amdgcn_readfirstlane(jof[i]);
        woff = t[4 + wave];
        const int rw = t[20 + wave];
        rlw = rw & 0xFFFF;  // this wave's diagonals
        big = rw >> 16;     // its largest group (1: no split row, no segment combine)
        vi = t[36 + tid];
    };
    // the pairs of diagonals m .. m+3 of this lane: one coalesced 512-byte load per diagonal
    // (waves without pairs read block 0: a group has >= 256 pairs)
    auto pairs4 = [&](int base, int2 (&u)[4]) {
        const int2* p = g.pairs + base + lane;
#pragma unroll
        for (int q = 0; q < 4; ++q) u[q] = p[64 * q];
    };
    // a finished relation's sums into the accumulators: a group's segments (consecutive lanes
    // of this wave) folded by a DPP shift tree, then its first lane adds the row
    auto accumulate = [&](float4 (&part)[4], int vi, int big) {
        const int seg = (vi >> 10) & 7, gsz = ((vi >> 13) & 7) + 1;
        // a group's gsz (1, 2, 4 or 8) segments sit on lanes from a multiple of gsz, inside one
        // 16-lane DPP row (staged_layout): a shift-left tree (lane l += lane l + s, s < gsz)
        // folds them into the first lane — VALU only, no LDS permute
        if (big > 1) fold_step<1>(part, gsz);
        if (big > 2) fold_step<2>(part, gsz);
        if (big > 4) fold_step<4>(part, gsz);
        const int row = vi & 1023;
        if (seg == 0 && row != kDummyRow) {
            float4* ar = acc + row * ast;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float4 o = ar[j];
                dg::add4(o, part[j]);
                ar[j] = o;
            }
        }
    };

    float wa[16];  // PROJ: the W slice of the next slab to make
    if constexpr (PROJ) {
        load_w(0, wa);
        slab_make(0, wa);
        if (nk > 1) load_w(1, wa);
    } else {
        slab_copy(0);
    }
    int woff, rlw, big, vi;
    tables(0, woff, rlw, big, vi);
    woff = __builtin_amdgcn_readfirstlane(woff);
    rlw = __builtin_amdgcn_readfirstlane(rlw);
    int2 un[4];
    pairs4(woff, un);
    if constexpr (PROJ)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // slab 0 written
    else
        relation_barrier();  // slab 0 complete

    float4 part[4];
    int pvi = 0, pbig = 1, prlw = 0;  // the previous relation's lane info (none yet)
#ifdef DG_STAGED_PROF
    unsigned long long c_bar = 0, c_put = 0, c_start = 0, c_gather = 0, c_acc = 0,
                       c0 = __builtin_readcyclecounter(), c1;
#define DG_TICK(acc_) (c1 = __builtin_readcyclecounter(), acc_ += c1 - c0, c0 = c1)
#else
#define DG_TICK(acc_) ((void)0)
#endif
#pragma unroll 1
    for (int i = 0; i < nk; ++i) {
        // relation i-1's sums (deferred past the barrier: they cover un's latency)
        if (prlw > 0) accumulate(part, pvi, __builtin_amdgcn_readfirstlane(pbig));
        DG_TICK(c_acc);
        if constexpr (PROJ) {
            if (i + 1 < nk) {  // the other buffer: last read by relation i-1
                slab_make(i + 1, wa);
                if (i + 2 < nk) load_w(i + 2, wa);
            }
        } else {
            // un (relation i's first diagonals) must arrive before the slab copy is queued
            // behind it: vmcnt retires in order
            asm volatile("" :: "v"(un[0].x), "v"(un[0].y), "v"(un[1].x), "v"(un[1].y), "v"(un[2].x),
                         "v"(un[2].y), "v"(un[3].x), "v"(un[3].y));
            if (i + 1 < nk) slab_copy(i + 1);  // the other buffer: last read by relation i-1
        }
        DG_TICK(c_put);
        int nwoff, nrlw, nbig, nvi;
        tables(min(i + 1, nk - 1), nwoff, nrlw, nbig, nvi);
        const float4* xs = xs0 + (i & 1) * a.xs_f4;
        DG_TICK(c_start);
#pragma unroll
        for (int j = 0; j < 4; ++j) part[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
        for (int m = 0; m < rlw; m += 4) {
            int2 u[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) u[q] = un[q];
            if (m + 4 < rlw) pairs4(woff + 64 * (m + 4), un);
            float4 gx[4][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4* xq = xs + __umul24(u[q].x, 5);
#pragma unroll
                for (int j = 0; j < 4; ++j) gx[q][j] = xq[j];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float v = __int_as_float(u[q].y);
#pragma unroll
                for (int j = 0; j < 4; ++j) dg::fma4(part[j], v, gx[q][j]);
            }
        }
        DG_TICK(c_gather);
        pvi = vi;
        pbig = big;
        prlw = rlw;
        woff = __builtin_amdgcn_readfirstlane(nwoff);
        rlw = __builtin_amdgcn_readfirstlane(nrlw);
        big = nbig;
        vi = nvi;
        // the next relation's first diagonals: the last VMEM ops before the barrier
        pairs4(woff, un);
        if constexpr (PROJ)
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // gathers done; slab i+1 written
        else
            relation_barrier();  // relation i's gathers done; slab i+1 complete
        DG_TICK(c_bar);
    }
    if (prlw > 0) accumulate(part, pvi, __builtin_amdgcn_readfirstlane(pbig));
#ifdef DG_STAGED_PROF
    if (lane == 0) {
        unsigned long long* pw = a.prof + ((int64_t)b * (kMaxThreads / 64) + (tid >> 6)) * kProfSlots;
        pw[0] = c_bar;
        pw[1] = c_put;
        pw[2] = c_start;
        pw[3] = c_gather;
        pw[4] = c_acc;
        pw[5] = nk;
    }
#endif
#undef DG_TICK
    __syncthreads();
    for (int q = tid; q < n_rows * 4; q += T) {
        const int r = q >> 2, j = q & 3;
        if (col0 + 4 * j < d)
            *reinterpret_cast<float4*>(g.out + ((int64_t)c * n_rows + r) * d + col0 + 4 * j) = acc[r * ast + j];
    }
}

}  // namespace

#ifdef DG_STAGED_PROF
static unsigned long long* dg_staged_prof_last = nullptr;
static int64_t dg_staged_prof_blocks = 0;
extern "C" int64_t dg_staged_prof_copy(unsigned long long* host, int64_t max_blocks) {
    const int64_t n = dg_staged_prof_blocks < max_blocks ? dg_staged_prof_blocks : max_blocks;
    if (!dg_staged_prof_last || n <= 0) return 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(host, dg_staged_prof_last, n * 16 * kProfSlots * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    return n;
}
#endif

namespace {
int staged_launch(const dg_staged_group* groups, const dg_staged_proj* projs, int32_t n_groups, int32_t d,
                  void* stream) {
    if (n_groups < 1 || !groups) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
    if (d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    StagedArgs a{};
    a.d = d;
    int64_t blocks = 0;
    int max_cols = 0, max_rows = 0;
    for (int i = 0; i < n_groups; ++i) {
        const dg_staged_group& s = groups[i];
        if (s.jm_len < 36 + kMaxThreads) return DG_EINVAL;  // one table + the spare ints
        if (s.n_rows < 0 || s.n_cols < 0 || s.n_rels < 0 || s.out_chunk < 1 || s.out_chunk > 64) return DG_EINVAL;
        if (s.n_rows >= kDummyRow || s.n_cols > kMaxThreads) return DG_EINVAL;  // rows fit 10 bits
        if (s.n_rows == 0 || s.n_rels == 0) continue;
        if (!s.pairs || !s.jm || !s.jmoff || !s.out) return DG_EINVAL;
        if (!dg::aligned16(s.out) || !dg::aligned16(s.pairs)) return DG_EALIGN;
        if (projs) {  // slabs from H · W: 64-wide H rows, 16-byte aligned
            const dg_staged_proj& pj = projs[i];
            if (!pj.h || !pj.w || pj.din != 64 || pj.h_ld < 64) return DG_EINVAL;
            if (!dg::aligned16(pj.h) || (pj.h_ld & 3)) return DG_EALIGN;
            if ((int64_t)s.n_cols * pj.h_ld > 0x7fffffffLL) return DG_EINVAL;
        } else {
            if (!s.x) return DG_EINVAL;
            if (!dg::aligned16(s.x) || (s.x_ld & 3) || s.x_ld < d) return DG_EALIGN;
            if ((int64_t)s.x_rows * s.x_ld > 0x7fffffffLL) return DG_EINVAL;
        }
        StagedGroupK& k = a.g[a.n_groups++];
        if (projs) {
            k.h = projs[i].h;
            k.w = projs[i].w;
            k.h_ld = static_cast<int32_t>(projs[i].h_ld);
        }
        k.pairs = reinterpret_cast<const int2*>(s.pairs);
        k.jm = s.jm;
        k.jmoff = s.jmoff;
        k.slab = s.slab;
        k.x = s.x;
        k.out = s.out;
        k.x_ld = static_cast<int32_t>(s.x_ld);
        k.n_rows = s.n_rows;
        k.n_cols = s.n_cols;
        k.n_rels = s.n_rels;
        k.out_chunk = s.out_chunk < s.n_rels ? s.out_chunk : s.n_rels;
        k.n_out_chunks = dg::ceil_div(s.n_rels, k.out_chunk);
        if (s.chunk_start) {  // variable chunks: 0 = c_0 < c_1 < ... < c_n = n_rels, each <= 64
            const int32_t nc = s.n_chunks;
            if (nc < 1 || nc > kMaxVarChunks || s.n_rels > 65535 || s.chunk_start[0] != 0 || s.chunk_start[nc] != s.n_rels)
                return DG_EINVAL;
            for (int32_t c = 0; c < nc; ++c) {
                const int32_t len = s.chunk_start[c + 1] - s.chunk_start[c];
                if (len < 1 || len > 64) return DG_EINVAL;
                k.cstart[c] = static_cast<uint16_t>(s.chunk_start[c]);
            }
            k.cstart[nc] = static_cast<uint16_t>(s.n_rels);
            k.var = 1;
            k.n_out_chunks = nc;
        }
        k.n_slices = dg::ceil_div(d, 16);
        // XCD-aligned at chunk granularity: XCD x takes chunks [x·cpx, (x+1)·cpx) with all their
        // slices, so a chunk's pairs are read into one L2 (the kernel's item map is
        // (lb & 7)·per + (lb >> 3), per = n_blocks / 8 = cpx·n_slices)
        const int64_t cpx = (k.n_out_chunks + 7) / 8;
        k.n_blocks = static_cast<int32_t>(8 * cpx * k.n_slices);
        k.block_begin = static_cast<int32_t>(blocks);
        blocks += k.n_blocks;
        max_cols = s.n_cols > max_cols ? s.n_cols : max_cols;
        max_rows = s.n_rows > max_rows ? s.n_rows : max_rows;
    }
    if (blocks == 0) return DG_OK;
    if (blocks > 0x7fffffff) return DG_EINVAL;
    const int threads = kMaxThreads;  // one thread per virtual row (staged_layout: at most 1024)
    a.xs_f4 = (max_cols + 16) * 5;    // + the sixteen zero columns
    a.acc_st = 4;
    a.acc_f4 = max_rows * 4;
    int64_t lds = 2 * (int64_t)a.xs_f4 * 16 + kMetaInts * 4 + (int64_t)a.acc_f4 * 16;
    if (lds > kLdsBytes) return DG_EINVAL;
    // 80-byte accumulator rows when they fit: a wave's row updates (rows of consecutive virtual
    // rows) then spread over the 16 bank slots instead of 4 (64-byte rows: slot (4·row + j) mod 16)
    if (lds + (int64_t)max_rows * 16 <= kLdsBytes) {
        a.acc_st = 5;
        a.acc_f4 = max_rows * 5;
        lds += (int64_t)max_rows * 16;
    }
#ifdef DG_STAGED_PROF
    {
        static unsigned long long* buf = nullptr;
        static int64_t have_blocks = 0;
        if (have_blocks < blocks) {
            if (buf) (void)hipFree(buf);
            (void)hipMalloc(&buf, blocks * 16 * kProfSlots * sizeof(unsigned long long));
            have_blocks = blocks;
        }
        (void)hipMemset(buf, 0, blocks * 16 * kProfSlots * sizeof(unsigned long long));
        a.prof = buf;
        dg_staged_prof_last = buf;
        dg_staged_prof_blocks = blocks;
    }
#endif
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (projs) {
        static std::atomic<uint64_t> configured{0};
        dg::lds_optin(reinterpret_cast<const void*>(&spmm_staged_kernel<true>), kLdsBytes, configured);
        hipLaunchKernelGGL(spmm_staged_kernel<true>, dim3(static_cast<unsigned>(blocks)), dim3(threads),
                           static_cast<int>(lds), st, a);
    } else {
        static std::atomic<uint64_t> configured{0};
        dg::lds_optin(reinterpret_cast<const void*>(&spmm_staged_kernel<false>), kLdsBytes, configured);
        hipLaunchKernelGGL(spmm_staged_kernel<false>, dim3(static_cast<unsigned>(blocks)), dim3(threads),
                           static_cast<int>(lds), st, a);
    }
    return dg::launch_status();
}
}  // namespace

extern "C" int dg_spmm_staged_f32(const dg_staged_group* groups, int32_t n_groups, int32_t d,
                                  void* stream) {
    return staged_launch(groups, nullptr, n_groups, d, stream);
}

extern "C" int dg_spmm_staged_proj_f32(const dg_staged_group* groups, const dg_staged_proj* projs,
                                       int32_t n_groups, int32_t d, void* stream) {
    if (!projs) return DG_EINVAL;
    return staged_launch(groups, projs, n_groups, d, stream);
}
