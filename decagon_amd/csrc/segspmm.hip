// Relation-segment SpMM for gfx950 (MI355X): one wave per (row, relation) — the sharded
// config-S form (one relation set per GPU, every node type row-split).
//
// Reference ops replaced (paths relative to the reference root):
//   tf.sparse_tensor_dense_matmul(adj_mats[edge_type][k], x)  decagon/deep/layers.py:90, :114
//   tf.matmul(x, weights_k)                                    decagon/deep/layers.py:113
//   tf.add_n(outputs) over a chunk of relations               decagon/deep/layers.py:92, :116
//
// Why: at N GPUs a rank owns n/N rows of every node type, each carrying N relation sets.  One
// workgroup per row (dg_gcn_fused_f32) leaves most CUs idle at 113 rows per rank, and the layer-2
// operands H1_j·W2_k of every relation would have to be projected on every rank (all of H1 is
// gathered; the projection of a source row is needed by every rank whose rows it touches).
// Here the item is (chunk, row) with one wave per relation of the chunk, and layer 2 is
// reassociated,
//     Σ_k Â_k[r]·(H1·W2_k) = Σ_k (Â_k[r]·H1)·W2_k,
// so a rank gathers the shared 64-wide H1 rows and projects only the aggregates of its own rows.
//
// Per wave (row r, relation t of chunk c):
//   [W: issue the 8 float4 loads of this lane's W2 slice, before the pairs]
//   pairs of the segment (one coalesced load of ≤ 64, the next 64 prefetched), the batch's 64
//   gathers in flight at once (LP lanes per gathered row), a shuffle butterfly → y = Â_k[r]·X
//   [W: y through the wave's LDS slot to the matvec layout (lane: output float4 l&7, input
//    slice 8(l>>3) .. +8), 32 fmaf, a butterfly over the 8 slices → z = y·W_k]
// then the chunk's waves add their rows in relation order (LDS, one barrier) and the first
// wave of the row writes out[c][r].  Fixed order, no atomics: bitwise reproducible.
#include <vector>

#include "common.h"
#include "peer.h"

// gathers in flight per lane (U: plain sums, UP: the reassociated form), per kernel —
// measured at config S (rows 4-81 nonzeros per relation), the occupancy they leave matters
// more than the round trips they save:
//   spmm_seg (N = 8 rank share, ≈ 650 workgroups): U 8 / UP 4 → 27.1 µs a step (U 4 / UP 2 27.3,
//   UP 8 28.4, U 16 32.7);  fused seg (N = 1, 900 workgroups): U 4 → 20.4 µs (8: 21.4)
constexpr int kSegU = 8;     // spmm_seg, plain sums
constexpr int kSegUP = 4;    // spmm_seg, reassociated (W slice read after the gathers)
constexpr int kFsegU = 4;    // fused seg, plain sums
constexpr int kFsegUP = 4;   // fused seg, reassociated (W slabs read after the gathers: layer 2 at
                             // config S 6.87 us, against 7.35 with the slice held in 32 VGPRs through
                             // the gathers and 9.45 staged in LDS per workgroup; step 19.36 / 19.66 /
                             // 21.88 us at 200 steps)
constexpr int kSegMinNW = 1; // waves per workgroup, at least (else: the launch's largest chunk)
// the wave-table forms' gathers in flight per lane (config S step at 200 steps, round 5: 4 / 4
// 15.56-15.63 us; 8 / 8 15.88-15.93; 16 / 16 18.30-18.32; the W slice issued before the gathers
// instead of after them 15.92-15.97, with 8 / 8 16.75-16.81)
constexpr int kTabU = 4;
constexpr int kTabUP = 4;

namespace {

struct SegGroupK {
    const int32_t* rowptr;
    const int32_t* seg;
    const int32_t* vcol;
    const float* val;
    const int32_t* slab;
    const float* x;
    const float* w;
    float* out;
    int32_t x_ld;
    int32_t n_rows;
    int32_t n_cols;
    int32_t n_chunks;
    int32_t chunk;
    int32_t n_rels;
    int32_t rpb;         // rows per workgroup: NW / chunk
    int32_t row_blocks;
    int32_t block_begin;
    int32_t n_blocks;
};

struct SegArgs {
    SegGroupK g[DG_MAX_GROUPS];
    int32_t n_groups;
    int32_t nw;  // waves per workgroup
};

// Broadcast lane m of each 16-lane row to the row (DPP row_newbcast:m — VALU, no LDS).  m
// must fold to a constant (every caller's loops are unrolled).
template <int M>
__device__ __forceinline__ int row_bcast(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + M, 0xF, 0xF, false);
}

__device__ __forceinline__ int row_bcast_rt(int v, int m) {
    switch (m) {
#define DG_RB(M) \
    case M: return row_bcast<M>(v);
        DG_RB(0) DG_RB(1) DG_RB(2) DG_RB(3) DG_RB(4) DG_RB(5) DG_RB(6) DG_RB(7)
        DG_RB(8) DG_RB(9) DG_RB(10) DG_RB(11) DG_RB(12) DG_RB(13) DG_RB(14) DG_RB(15)
#undef DG_RB
        default: return 0;
    }
}

// y = Σ_{p in [beg, end)} val[p] · X[vcol[p]] (X row v at xb + v·x_ld), folded: every lane
// holds float4 (lane % LP) of the row (LP ∈ {8, 16}).  A batch of 64 pairs is one coalesced
// load — permuted so that the pair a lane group needs at step m sits in its own 16-lane row,
// lane m (LP 16) or lane 8·h + m (LP 8, the row's two groups h) — and handed to the groups by
// DPP row broadcasts; UU gathers per lane in flight; the next batch's pairs are loaded before
// this batch's gathers.
template <int LP, int UU>
__device__ __forceinline__ float4 seg_gather(const int32_t* __restrict__ vcol, const float* __restrict__ val,
                                             const float* xb, int x_ld, int beg, int end) {
    static_assert(LP == 16 || LP == 8, "seg_gather: 64- or 32-float rows");
    constexpr int G = dg::kWave / LP;  // nonzeros side by side
    constexpr int S = dg::kWave / G;   // steps per batch of 64
    constexpr int U = UU ? UU : S;
    static_assert(U >= 1 && U <= S && S % U == 0, "seg_gather: the unroll must divide the steps of a batch");
    const int lane = threadIdx.x & 63;
    const int sub = lane / LP;
    const float* xq = xb + (lane % LP) * 4;
    // lane l holds pair perm(l) of the batch (pair m·G + sub: lane 16·sub + m, or 16·(sub/2) + 8·(sub%2) + m)
    const int perm = LP == 16 ? 4 * (lane & 15) + (lane >> 4)
                              : 8 * (lane & 7) + 2 * (lane >> 4) + ((lane >> 3) & 1);
    const bool odd = LP == 8 && ((lane >> 3) & 1);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int vc = 0;
    float vv = 0.f;
    if (beg + perm < end) {
        vc = vcol[beg + perm];
        vv = val[beg + perm];
    }
#pragma unroll 1
    for (int base = beg; base < end; base += 64) {
        const int n = min(64, end - base);
        const int eoff = vc * x_ld;
        const int vbits = __float_as_int(vv);
        vc = 0;
        vv = 0.f;
        if (base + 64 + perm < end) {
            vc = vcol[base + 64 + perm];
            vv = val[base + 64 + perm];
        }
#pragma unroll
        for (int it = 0; it < S / U; ++it) {
            if (it * U * G >= n) break;  // wave-uniform
            int o[U];
            float w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int m = it * U + u;
                int oe, we;
                if constexpr (LP == 16) {
                    oe = row_bcast_rt(eoff, m);
                    we = row_bcast_rt(vbits, m);
                } else {
                    const int o0 = row_bcast_rt(eoff, m), o1 = row_bcast_rt(eoff, 8 + m);
                    const int w0 = row_bcast_rt(vbits, m), w1 = row_bcast_rt(vbits, 8 + m);
                    oe = odd ? o1 : o0;
                    we = odd ? w1 : w0;
                }
                o[u] = oe;
                w[u] = __int_as_float(we);
            }
            float4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool ok = (it * U + u) * G + sub < n;
                xv[u] = ok ? *reinterpret_cast<const float4*>(xq + o[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
                if (!ok) w[u] = 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) dg::fma4(acc, w[u], xv[u]);
        }
    }
    acc = dg::xor_sum4_from<LP>(acc);
    return acc;
}

// The same sum with the pairs handed out by ds_bpermute (__shfl) in a rolled loop: measured
// faster than the DPP form in the reassociated kernels (layer 2 at S: 6.9 vs 8.0 µs), whose
// W slice leaves fewer registers for the unrolled broadcasts.
template <int LP, int UU>
__device__ __forceinline__ float4 seg_gather_shfl(const int32_t* __restrict__ vcol, const float* __restrict__ val,
                                             const float* xb, int x_ld, int beg, int end) {
    constexpr int G = dg::kWave / LP;
    constexpr int U = UU ? UU : LP;  // (U·G = 64: one batch per round trip)
    static_assert(U >= 1 && U <= LP && LP % U == 0, "seg_gather_shfl: the unroll must divide the steps of a batch");
    const int lane = threadIdx.x & 63;
    const int sub = lane / LP;
    const float* xq = xb + (lane % LP) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int vc = 0;
    float vv = 0.f;
    if (beg + lane < end) {
        vc = vcol[beg + lane];
        vv = val[beg + lane];
    }
#pragma unroll 1
    for (int base = beg; base < end; base += 64) {
        const int n = min(64, end - base);
        const int eoff = vc * x_ld;
        const float v = vv;
        vc = 0;
        vv = 0.f;
        if (base + 64 + lane < end) {
            vc = vcol[base + 64 + lane];
            vv = val[base + 64 + lane];
        }
#pragma unroll 1
        for (int s0 = 0; s0 < n; s0 += U * G) {
            int o[U];
            float w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int src = (s0 + u * G + sub) & 63;
                o[u] = __shfl(eoff, src);
                w[u] = __shfl(v, src);
            }
            float4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool ok = s0 + u * G + sub < n;
                xv[u] = ok ? *reinterpret_cast<const float4*>(xq + o[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
                if (!ok) w[u] = 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) dg::fma4(acc, w[u], xv[u]);
        }
    }
    acc = dg::xor_sum4_from<LP>(acc);
    return acc;
}

// One wave's share: relation t of chunk c in row r — its segment's sum y = Σ val·X[vcol]
// (lanes hold float4 lane % LP of the row).
template <int LP, int U>
__device__ __forceinline__ float4 seg_wave(const SegGroupK& g, int c, int r, int t) {
    const int64_t si = ((int64_t)c * g.n_rows + r) * g.chunk + t;
    const int beg = g.seg[si];
    const int end = t + 1 < g.chunk ? g.seg[si + 1] : g.rowptr[(int64_t)c * g.n_rows + r + 1];
    return seg_gather<LP, U>(g.vcol, g.val, g.x, g.x_ld, beg, end);
}

// The reassociated wave (layer 2, d_in 64 -> d_out 32): y = Â_k[r]·H, then z = y·W_k with
// this lane's W_k slice (rows 8(l>>3) .. +8, output float4 l & 7) read from global memory after
// the gathers — one more L2 round trip at the end instead of 32 VGPRs held through them, which
// buys gathers in flight (config S layer 2: 6.87 us, against 7.35 with the slice held and 9.45
// with the workgroup's slabs staged in LDS).  beg / end: the segment.
template <int UP>
__device__ __forceinline__ float4 seg_wave_proj(const SegGroupK& g, int k, int beg, int end, float4* ybuf) {
    const int lane = threadIdx.x & 63;
    const int s = g.slab ? g.slab[k] : k;
    const int ms = lane >> 3;
    const float4* w = reinterpret_cast<const float4*>(g.w + (int64_t)s * (64 * 32)) + (8 * ms) * 8 + (lane & 7);
    float4 wv[8];
    const float* xb = g.x - (int64_t)s * g.n_cols * g.x_ld;  // vcol = s·n_cols + col addresses row col
    const float4 y = seg_gather_shfl<16, UP>(g.vcol, g.val, xb, g.x_ld, beg, end);
#pragma unroll
    for (int i = 0; i < 8; ++i) wv[i] = w[8 * i];
    if (lane < 16) ybuf[lane] = y;
    __builtin_amdgcn_wave_barrier();
    const float4 ya = ybuf[2 * ms];
    const float4 yb = ybuf[2 * ms + 1];
    float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    dg::fma4(z, ya.x, wv[0]);
    dg::fma4(z, ya.y, wv[1]);
    dg::fma4(z, ya.z, wv[2]);
    dg::fma4(z, ya.w, wv[3]);
    dg::fma4(z, yb.x, wv[4]);
    dg::fma4(z, yb.y, wv[5]);
    dg::fma4(z, yb.z, wv[6]);
    dg::fma4(z, yb.w, wv[7]);
    z = dg::xor_sum4_from<8>(z);
    return z;
}

// PROJ: d_in = 64 (LP = 16), d_out = 32; otherwise d_out = d_in = 4·LP.  a.nw waves per
// workgroup (the launch's largest chunk, so a chunk-6 group wastes no wave slot; rows per
// workgroup nw / chunk), at most NW.  (A form whose last-arriving workgroup also finished
// each row — write-through partials, an arrival counter per row, no epilogue launch — measured
// slower at every N: 29.1 against 25.4 µs a rank share at N = 8, 42.8 against 30.5 with the peer
// exchange, 25.7 / 33.3 with two relation sets per chunk; removed in round 5)
template <int LP, bool PROJ, int NW>
__global__ __launch_bounds__(64 * NW) void spmm_seg_kernel(const SegArgs a) {
    constexpr int DOUT4 = PROJ ? 8 : LP;  // float4s of an output row
    __shared__ float4 ybuf[NW][16];
    __shared__ float4 zbuf[NW][DOUT4];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (segment bounds: scalar loads)
    int gi = 0;
#pragma unroll 1
    while (gi + 1 < a.n_groups && (int)blockIdx.x >= a.g[gi + 1].block_begin) ++gi;
    const SegGroupK& g = a.g[gi];
    // XCD-contiguous item map (block lb runs on XCD lb % 8): one chunk's rows stay on few XCDs
    const int lb = blockIdx.x - g.block_begin;
    const int per = g.n_blocks >> 3;
    const int item = (lb & 7) * per + (lb >> 3);
    const bool wg_live = item < g.n_chunks * g.row_blocks;
    if (!wg_live) return;  // workgroup-uniform, before any barrier
    const int c = item / g.row_blocks;
    const int r0 = (item - c * g.row_blocks) * g.rpb;
    const int slot = wave / g.chunk;
    const int t = wave - slot * g.chunk;
    const int r = r0 + slot;
    const bool row_ok = slot < g.rpb && r < g.n_rows;
    const int k = c * g.chunk + t;
    float4 res = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (PROJ) {
        const bool live = row_ok && k < g.n_rels;
        int beg = 0, end = 0;
        if (live) {
            const int64_t si = ((int64_t)c * g.n_rows + r) * g.chunk + t;
            beg = g.seg[si];
            end = t + 1 < g.chunk ? g.seg[si + 1] : g.rowptr[(int64_t)c * g.n_rows + r + 1];
        }
        if (live) res = seg_wave_proj<kSegUP>(g, k, beg, end, ybuf[wave]);
    } else if (row_ok && k < g.n_rels) {
        res = seg_wave<LP, kSegU>(g, c, r, t);  // wave-uniform
    }
    if (lane < DOUT4) zbuf[wave][lane] = res;  // relations past the group's end add zeros
    __syncthreads();
    if (row_ok && t == 0 && lane < DOUT4) {
        float4 s = zbuf[wave][lane];
        for (int u = 1; u < g.chunk; ++u) dg::add4(s, zbuf[wave + u][lane]);
        *reinterpret_cast<float4*>(g.out + ((int64_t)c * g.n_rows + r) * (4 * DOUT4) + 4 * lane) = s;
    }
}

// The fused form (dg_gcn_fused_seg_f32): one workgroup per output row of a target node type
// i, one wave per (group, relation) — every group one chunk — then, in LDS, each group's
// relations summed in order and L2-normalised (layers.py:93 / :117) by one wave, the groups
// summed in order and relu'd (model.py:75) by wave 0, which writes the row.  With PROJ this is
// layer 2 reassociated, so layer 1 needs no projection epilogue and no GEMM runs.
struct FsTargetK {
    float* out;
    int32_t n_rows;
    int32_t g_begin;
    int32_t g_count;
    int32_t relu;
    int32_t block_begin;
    int32_t waves;  // waves per row: one per relation of the target's groups (<= 16)
    int32_t rpb;    // rows per workgroup: nw / waves (at most kFsMaxRpb)
    int32_t pad;
};

struct FsArgs {
    SegGroupK g[DG_MAX_GROUPS];
    FsTargetK t[DG_MAX_GROUPS];
    int32_t n_targets;
    int32_t nw;
    dg::PeerK P;  // PEER: every finished row also goes to every peer's copy (peer.h)
};

constexpr int kFsMaxRpb = 4;  // rows per workgroup, at most (1: no change at config S)

#ifdef DG_FSEG_PROF
// Profiling build only (scripts/fseg_prof.py): per (launch form, workgroup, wave) the
// s_memrealtime (100 MHz) stamps of the phases below, and the XCC id.
constexpr int kFsProfSlots = 8;
constexpr int kFsProfMaxBlocks = 4096;
__device__ unsigned long long g_fs_prof[2][kFsProfMaxBlocks][16][kFsProfSlots];
#define DG_FS_STAMP(i) \
    do { if (lane == 0 && blockIdx.x < kFsProfMaxBlocks) g_fs_prof[PROJ][blockIdx.x][wave][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define DG_FS_STAMP(i) ((void)0)
#endif

template <int LP, bool PROJ, int NW, bool PEER>
__global__ __launch_bounds__(64 * NW) void gcn_fused_seg_kernel(const FsArgs a) {
    constexpr int DOUT4 = PROJ ? 8 : LP;
    __shared__ float4 ybuf[NW][16];
    __shared__ float4 zbuf[NW][DOUT4];
    __shared__ float4 nbuf[kFsMaxRpb][DG_MAX_GROUPS][DOUT4];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    DG_FS_STAMP(0);  // (profiling build: wave start)
    int ti = 0;
#pragma unroll 1
    while (ti + 1 < a.n_targets && (int)blockIdx.x >= a.t[ti + 1].block_begin) ++ti;
    const FsTargetK& T = a.t[ti];
    // (rows in dispatch order: XCD-contiguous row blocks measured slower at config S, 18.60 vs
    // 18.16 µs a step — a random graph's rows gather from every XCD's share of the operand)
    const int r0 = (blockIdx.x - T.block_begin) * T.rpb;
    // wave -> (row slot, group gl, relation k of the group): each slot's groups' relations back
    // to back; k = c·chunk + t (chunk c, relation t: a rank's row block of several relation
    // sets keeps one chunk per set)
    const int slot = wave / T.waves;
    const int wi = wave - slot * T.waves;
    const int r = r0 + slot;
    int gl = 0, base = 0;
#pragma unroll 1
    while (gl < T.g_count && wi >= base + a.g[T.g_begin + gl].n_rels) base += a.g[T.g_begin + gl++].n_rels;
    float4 res = make_float4(0.f, 0.f, 0.f, 0.f);
    DG_FS_STAMP(1);  // target / group found
    if constexpr (PROJ) {
        const bool live = slot < T.rpb && r < T.n_rows && gl < T.g_count;
        const int gi = T.g_begin + (gl < T.g_count ? gl : 0);
        const int k = wi - base;
        int beg = 0, end = 0;
        if (live) {
            const SegGroupK& g = a.g[gi];
            const int c = k / g.chunk, t = k - c * g.chunk;
            const int64_t si = ((int64_t)c * g.n_rows + r) * g.chunk + t;
            beg = g.seg[si];
            end = t + 1 < g.chunk ? g.seg[si + 1] : g.rowptr[(int64_t)c * g.n_rows + r + 1];
        }
#ifdef DG_FSEG_PROF
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
        DG_FS_STAMP(2);  // segment bounds loaded
        if (live) res = seg_wave_proj<kFsegUP>(a.g[gi], k, beg, end, ybuf[wave]);
    } else if (slot < T.rpb && r < T.n_rows && gl < T.g_count) {
        const SegGroupK& g = a.g[T.g_begin + gl];
        const int k = wi - base;
        const int c = k / g.chunk;
        res = seg_wave<LP, kFsegU>(g, c, r, k - c * g.chunk);
    }
#ifdef DG_FSEG_PROF
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
    DG_FS_STAMP(3);  // the wave's relation sum done
    if (lane < DOUT4) zbuf[wave][lane] = res;
    __syncthreads();
    DG_FS_STAMP(4);  // every wave of the workgroup done
    // one wave per (row slot, group): its relations summed in order, L2-normalised
    if (wave < T.rpb * T.g_count) {
        const int s2 = wave / T.g_count, gg = wave - s2 * T.g_count;
        int gb = s2 * T.waves;
#pragma unroll 1
        for (int u = 0; u < gg; ++u) gb += a.g[T.g_begin + u].n_rels;
        const int K = a.g[T.g_begin + gg].n_rels;
        const int q = lane % DOUT4;
        float4 sum = zbuf[gb][q];
#pragma unroll 1
        for (int u = 1; u < K; ++u) dg::add4(sum, zbuf[gb + u][q]);
        // tf.nn.l2_normalize: x * rsqrt(max(sum(x^2), 1e-12))
        float ss = sum.x * sum.x + sum.y * sum.y + sum.z * sum.z + sum.w * sum.w;
        ss = dg::xor_sum_below<DOUT4>(ss);
        const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
        if (lane < DOUT4) nbuf[s2][gg][lane] = make_float4(sum.x * inv, sum.y * inv, sum.z * inv, sum.w * inv);
    }
    __syncthreads();
    DG_FS_STAMP(5);  // groups normalised
    if (wave < T.rpb && r0 + wave < T.n_rows && lane < DOUT4) {
        float4 tot = nbuf[wave][0][lane];
        for (int u = 1; u < T.g_count; ++u) dg::add4(tot, nbuf[wave][u][lane]);
        if (T.relu) {
            tot.x = fmaxf(tot.x, 0.f);
            tot.y = fmaxf(tot.y, 0.f);
            tot.z = fmaxf(tot.z, 0.f);
            tot.w = fmaxf(tot.w, 0.f);
        }
        const int64_t o = (int64_t)(r0 + wave) * (4 * DOUT4) + 4 * lane;
        *reinterpret_cast<float4*>(T.out + o) = tot;
        if constexpr (PEER) dg::peer_store4(a.P, T.out, (uint32_t)T.n_rows * (16 * DOUT4), (uint32_t)o * 4, tot);
    }
#ifdef DG_FSEG_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DG_FS_STAMP(6);  // row stored
    if (lane == 0 && blockIdx.x < kFsProfMaxBlocks) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_fs_prof[PROJ][blockIdx.x][wave][7] = xcc;
    }
#endif
    if constexpr (PEER) dg::peer_arrive(a.P);  // the last workgroup raises the flags and waits
}

// The wave-table form of the fused launch (dg_gcn_fused_tab_f32, round 5): the same rows, waves
// and arithmetic as gcn_fused_seg_kernel, but every value a wave needs before its gathers —
// its relation segment's bounds, gather base, W slab, and its roles in the two finishing
// phases — is precomputed on the host into a 64-byte descriptor per (workgroup, wave), and the
// segment's first 64 (vcol, value) pairs are stored at a fixed slot per wave.  So a wave's
// first memory round trip loads its descriptor (one s_load_dwordx16) and its first pairs (one
// dwordx2 per lane) together, instead of the target / group search over the launch arguments,
// the segment bounds and then the pairs — three to five dependent round trips (config S,
// scripts/fseg_prof.py: search 0.64 µs, bounds 0.60 µs median per wave before this).  Pairs
// past the first 64 follow in batches of 64 from `ovf`.  Batches of 64 as in the seg form, so
// the results are bitwise the seg form's.
static_assert(sizeof(dg_tab_desc) == 64, "dg_tab_desc: one s_load_dwordx16");
// pairs: [blocks * NW * 64] first batch of each wave (hand-out order); desc: [blocks * NW];
// ovf: later batches, 64 entries each.  (Separate pointer arguments: loaded together.)
// A wave's relation sum from its wave-table slot (the first pairs already in `first`): batches
// of 64 pairs, the first from the slot, the rest from ovf, each prefetched before the batch
// before it is gathered; U gathers in flight per lane, the pairs handed out by DPP row
// broadcasts (seg_gather's: pair m·G + sub of a batch in lane 16·sub + m).  PROJ: then the
// 64-wide aggregate times the relation's W slab (seg_wave_proj's arithmetic).
template <bool PROJ, int U>
__device__ __forceinline__ float4 tab_wave(const dg_tab_desc& D, const uint2 first, const uint2* __restrict__ ovf,
                                           float4* ybuf, const int S) {
    constexpr int LP = 16;
    constexpr int G = dg::kWave / LP;
    const int lane = threadIdx.x & 63;
    float4 res = make_float4(0.f, 0.f, 0.f, 0.f);
    if (D.cnt > 0) {  // wave-uniform
        // batches of 64 pairs: the first from the slot, the rest from ovf, each prefetched
        // before the batch before it is gathered
        const float* xq = D.x + (lane % LP) * 4;
        const int sub = lane / LP;
        int vc = (int)first.x;
        int vb = (int)first.y;
        const uint2* nx = ovf + D.ovf;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        // the first batch is the slot's S pairs (round 6: slot_pairs), the rest batches of 64;
        // a lane group takes pairs sub, sub + 4, ... in order across the batches whatever S (a
        // multiple of 4), so the sums are bitwise those of 64-pair first batches
        int bsz = S;
#pragma unroll 1
        for (int base = 0; base < D.cnt; base += bsz, bsz = 64) {
            const int n = min(bsz, D.cnt - base);
            const int eoff = vc * D.x_ld;
            const int vbits = vb;
            vc = 0;
            vb = 0;
            if (base + bsz < D.cnt) {
                const uint2 q = nx[lane];
                vc = (int)q.x;
                vb = (int)q.y;
                nx += 64;
            }
            // DPP row broadcasts (the seg form's seg_gather): pair m·G + sub of the batch sits in
            // lane 16·sub + m.  Round 6: layer 2 (PROJ) too — since its W slice is read after the
            // gathers the unrolled broadcasts' registers fit (46 → 46 VGPRs), and its launch
            // measured 5.64–5.72 → 5.33–5.48 µs against the ds_bpermute hand-out (same pair order
            // per lane group: the same bits).
            constexpr int S = dg::kWave / G;
#pragma unroll
            for (int it = 0; it < S / U; ++it) {
                if (it * U * G >= n) break;  // wave-uniform
                int o[U];
                float w[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    o[u] = row_bcast_rt(eoff, it * U + u);
                    w[u] = __int_as_float(row_bcast_rt(vbits, it * U + u));
                }
                float4 xv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool ok = (it * U + u) * G + sub < n;
                    xv[u] = ok ? *reinterpret_cast<const float4*>(xq + o[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
                    if (!ok) w[u] = 0.f;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) dg::fma4(acc, w[u], xv[u]);
            }
        }
        acc = dg::xor_sum4_from<LP>(acc);
#ifdef DG_FSEG_PROF
        if constexpr (PROJ) {  // (profiling build: stamp 2 = the gathers done, before the projection)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            DG_FS_STAMP(2);
        }
#endif
        if constexpr (PROJ) {
            // z = y·W_k: this lane's W slice (rows 8(l>>3) .. +8, output float4 l & 7) read
            // after the gathers, as in seg_wave_proj
            const int ms = lane >> 3;
            const float4* w = reinterpret_cast<const float4*>(D.w) + (8 * ms) * 8 + (lane & 7);
            float4 wv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) wv[i] = w[8 * i];
            if (lane < 16) ybuf[lane] = acc;
            __builtin_amdgcn_wave_barrier();
            const float4 ya = ybuf[2 * ms];
            const float4 yb = ybuf[2 * ms + 1];
            float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            dg::fma4(z, ya.x, wv[0]);
            dg::fma4(z, ya.y, wv[1]);
            dg::fma4(z, ya.z, wv[2]);
            dg::fma4(z, ya.w, wv[3]);
            dg::fma4(z, yb.x, wv[4]);
            dg::fma4(z, yb.y, wv[5]);
            dg::fma4(z, yb.z, wv[6]);
            dg::fma4(z, yb.w, wv[7]);
            z = dg::xor_sum4_from<8>(z);
            res = z;
        } else {
            res = acc;
        }
    }
    return res;
}

// v of lane ^ M for any M < 64: the power-of-two partners of M's bits composed (lane ^ a ^ b
// = lane ^ (a | b) for disjoint bits), each an exact value move (common.h's xor_get)
template <int M>
__device__ __forceinline__ float xor_get_any(float x) {
    if constexpr (M == 0) {
        return x;
    } else {
        constexpr int LOW = M & -M;
        return xor_get_any<M - LOW>(dg::xor_get<LOW>(x));
    }
}
template <int M>
__device__ __forceinline__ float4 xor_get4_any(const float4& v) {
    return make_float4(xor_get_any<M>(v.x), xor_get_any<M>(v.y), xor_get_any<M>(v.z), xor_get_any<M>(v.w));
}
// tot += the value of lane set V, V + 1, ... (< n, wave-uniform), in that order; lane set v is
// lanes [W·v, W·(v+1)), read from lane ^ W·v
template <int W, int V, int SETS>
__device__ __forceinline__ void add_lane_sets(float4& tot, const float4& v, int n) {
    if constexpr (V < SETS) {
        if (V < n) dg::add4(tot, xor_get4_any<W * V>(v));
        add_lane_sets<W, V + 1, SETS>(tot, v, n);
    }
}

// rows[0][q] + rows[1][q] + ... + rows[K-1][q], added in that order (((r0 + r1) + r2) + ...).
// (Measured, round 6: the LDS reads of each run of 8 rows issued before the first add — predicated
// reads and selects — made config S's layer 1 0.2 µs slower than this loop: 4.47-4.56 against
// 4.29-4.34 µs; scripts/variants/serial_lds_sum.py kept the A/B.)
template <int W>
__device__ __forceinline__ float4 lds_ordered_sum(const float4 (*rows)[W], int K, int q) {
    float4 s = rows[0][q];
#pragma unroll 1
    for (int u = 1; u < K; ++u) dg::add4(s, rows[u][q]);
    return s;
}

// Byte offset of this lane's first-batch pair in a slot of S pairs: lane 16·sub + m' holds pair
// 4m' + sub, stored at slot entry sub·S/4 + m'; lanes with m' >= S/4 (no such pair in the slot)
// read their row's last entry — the same cache lines, never used.
__device__ __forceinline__ uint32_t slot_lane_offset(int lane, int S) {
    const int q = S >> 2, m = lane & 15;
    return 8u * (uint32_t)((lane >> 4) * q + (m < q ? m : q - 1));
}

// PEER (dg_gcn_fused_tab_peer_f32): each finished row also goes to every peer's copy of its
// target (desc.pad[0] = the row's byte offset in the target, pad[1] = the target's bytes), and
// the launch ends with the exchange (peer.h).
template <bool PROJ, int NW, bool PEER>
__global__ __launch_bounds__(64 * NW) void gcn_tab_kernel(const uint2* __restrict__ pairs,
                                                          const dg_tab_desc* __restrict__ desc,
                                                          const uint2* __restrict__ ovf, const int S,
                                                          const dg::PeerK P) {
    constexpr int DOUT4 = PROJ ? 8 : 16;
    __shared__ float4 ybuf[NW][16];
    __shared__ float4 zbuf[NW][DOUT4];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wi = (int64_t)blockIdx.x * NW + wave;
    DG_FS_STAMP(0);  // (profiling build: wave start)
    // The descriptor's scalar loads are issued first (the asm below clobbers memory, so they
    // cannot sink past it), then the first pairs, and one asm block both issues the pairs load
    // and waits for it: `first` exists for the compiler only once it has landed, so no copy or
    // use of it can be scheduled between issue and wait.  Both loads are in flight
    // together: the wave's first round trip fetches both.
    const dg_tab_desc D = desc[wi];  // (uniform: scalar loads)
    uint2 first;
    asm volatile("global_load_dwordx2 %0, %1, %2\n\ts_waitcnt vmcnt(0)"
                 : "=&v"(first) : "v"(slot_lane_offset(lane, S)), "s"(pairs + wi * S) : "memory");
    // every descriptor field and the ovf base in SGPRs here, so no scalar load is sunk below
    // the branch into a round trip of its own
    asm volatile("" ::"s"(D.x), "s"(D.w), "s"(D.orow), "s"(D.cnt), "s"(D.x_ld), "s"(D.ovf), "s"(D.role), "s"(D.wr),
                 "s"(ovf));
#ifdef DG_FSEG_PROF
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
    DG_FS_STAMP(1);  // descriptor and first pairs in registers
    if constexpr (!PROJ) DG_FS_STAMP(2);  // (layer 2: stamp 2 marks its gathers done, in tab_wave)
    const float4 res = tab_wave<PROJ, PROJ ? kTabUP : kTabU>(D, first, ovf, ybuf[wave], S);
#ifdef DG_FSEG_PROF
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
    DG_FS_STAMP(3);  // the wave's relation sum done
    if (lane < DOUT4) zbuf[wave][lane] = res;
    __syncthreads();
    DG_FS_STAMP(4);  // every wave of the workgroup done
    // Round 6: the row's finishing wave (D.orow) does the rest alone, without a second barrier:
    // lane set u (lanes [DOUT4·u, DOUT4·(u+1))) sums group u's waves in order and L2-normalises
    // the sum, then the groups are added in order across the lane sets (lane set 0 reads set v
    // from lane ^ DOUT4·v), relu'd and stored.  The same adds, butterflies and order as the
    // per-group normalising waves of round 5 plus the nbuf hand-off: the same bits.
    // desc.pad[2]: K − 1 of group u in bits 4u .. 4u+3; desc.pad[3]: the row slot's first wave.
    if (D.orow != nullptr) {
        constexpr int SETS = 64 / DOUT4;
        const int gc = D.wr & 0xff;
        const uint32_t kc = (uint32_t)D.pad[2];
        const int u = lane / DOUT4, q = lane % DOUT4;
        int gb = D.pad[3];
#pragma unroll
        for (int v = 0; v + 1 < SETS; ++v)
            if (v < u && v < gc) gb += (int)((kc >> (4 * v)) & 15u) + 1;
        const bool mine = u < gc;
        const int K = mine ? (int)((kc >> (4 * u)) & 15u) + 1 : 1;
        const float4 sum = lds_ordered_sum<DOUT4>(&zbuf[mine ? gb : 0], K, q);
        // tf.nn.l2_normalize: x * rsqrt(max(sum(x^2), 1e-12))
        float ss = sum.x * sum.x + sum.y * sum.y + sum.z * sum.z + sum.w * sum.w;
        ss = dg::xor_sum_below<DOUT4>(ss);
        const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
        const float4 nv = make_float4(sum.x * inv, sum.y * inv, sum.z * inv, sum.w * inv);
        float4 tot = nv;
        add_lane_sets<DOUT4, 1, SETS>(tot, nv, gc);  // ((n0 + n1) + n2) + ...
        DG_FS_STAMP(5);  // groups normalised and summed
        if (lane < DOUT4) {
            if ((D.wr >> 8) & 1) {
                tot.x = fmaxf(tot.x, 0.f);
                tot.y = fmaxf(tot.y, 0.f);
                tot.z = fmaxf(tot.z, 0.f);
                tot.w = fmaxf(tot.w, 0.f);
            }
            reinterpret_cast<float4*>(D.orow)[lane] = tot;
            if constexpr (PEER)
                dg::peer_store4(P, reinterpret_cast<const float*>(reinterpret_cast<const char*>(D.orow) - D.pad[0]),
                                (uint32_t)D.pad[1], (uint32_t)D.pad[0] + 16u * lane, tot);
        }
    }
#ifdef DG_FSEG_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DG_FS_STAMP(6);  // row stored
    if (lane == 0 && blockIdx.x < kFsProfMaxBlocks) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_fs_prof[PROJ][blockIdx.x][wave][7] = xcc;
    }
#endif
    if constexpr (PEER) dg::peer_arrive(P);  // the last workgroup raises the flags and waits
}

// The wave-table form of spmm_seg_kernel (dg_spmm_seg_tab_f32, round 5): the same workgroups
// (XCD-contiguous item map included), waves, batches and sums — bitwise its chunk partials —
// with each wave's segment, gather base, W slab and (for the first wave of a row's chunk) the
// partial row it writes and the waves it sums precomputed on the host: desc.orow != NULL marks
// that wave, desc.role bits 8-15 the chunk's waves.
template <bool PROJ, int NW>
__global__ __launch_bounds__(64 * NW) void seg_tab_kernel(const uint2* __restrict__ pairs,
                                                          const dg_tab_desc* __restrict__ desc,
                                                          const uint2* __restrict__ ovf, const int S) {
    constexpr int DOUT4 = PROJ ? 8 : 16;
    __shared__ float4 ybuf[NW][16];
    __shared__ float4 zbuf[NW][DOUT4];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wi = (int64_t)blockIdx.x * NW + wave;
    const dg_tab_desc D = desc[wi];  // (as gcn_tab_kernel: descriptor first, pairs load + wait in one asm)
    uint2 first;
    asm volatile("global_load_dwordx2 %0, %1, %2\n\ts_waitcnt vmcnt(0)"
                 : "=&v"(first) : "v"(slot_lane_offset(lane, S)), "s"(pairs + wi * S) : "memory");
    asm volatile("" ::"s"(D.x), "s"(D.w), "s"(D.orow), "s"(D.cnt), "s"(D.x_ld), "s"(D.ovf), "s"(D.role), "s"(ovf));
    const float4 res = tab_wave<PROJ, PROJ ? kSegUP : kSegU>(D, first, ovf, ybuf[wave], S);
    if (lane < DOUT4) zbuf[wave][lane] = res;  // relations past the group's end add zeros
    __syncthreads();
    if (D.orow != nullptr && lane < DOUT4) {
        const int K = (D.role >> 8) & 0xff;
        reinterpret_cast<float4*>(D.orow)[lane] = lds_ordered_sum<DOUT4>(&zbuf[wave], K, lane);
    }
}

}  // namespace

namespace {
// Validate one dg_seg_group and copy it into the kernel form (skip: nothing to compute).
int convert_seg(const dg_seg_group& s, bool proj, int d_in, SegGroupK& k, bool& skip) {
    if (s.n_rows < 0 || s.n_chunks < 1 || s.chunk < 1 || s.chunk > 16 || s.n_rels < 0 || s.n_cols < 0 ||
        s.x_rows < 0)
        return DG_EINVAL;
    if ((int64_t)s.n_chunks * s.chunk < s.n_rels || (int64_t)(s.n_chunks - 1) * s.chunk >= s.n_rels)
        return DG_EINVAL;  // every chunk holds at least one relation
    if ((s.w != nullptr) != proj) return DG_EINVAL;  // a weight stack exactly when d_in != d_out
    skip = s.n_rows == 0 || s.n_rels == 0;
    if (skip) return DG_OK;
    if (!s.rowptr || !s.seg || !s.x) return DG_EINVAL;
    if (!dg::aligned16(s.x) || (s.x_ld & 3)) return DG_EALIGN;
    if (proj && !dg::aligned16(s.w)) return DG_EALIGN;
    if (s.x_ld < d_in) return DG_EINVAL;
    if ((int64_t)s.x_rows * s.x_ld > 0x7fffffffLL) return DG_EINVAL;  // 32-bit gather offsets
    k = SegGroupK{};
    k.rowptr = s.rowptr;
    k.seg = s.seg;
    k.vcol = s.vcol;
    k.val = s.val;
    k.slab = s.slab;
    k.x = s.x;
    k.w = s.w;
    k.out = s.out;
    k.x_ld = static_cast<int32_t>(s.x_ld);
    k.n_rows = s.n_rows;
    k.n_cols = s.n_cols;
    k.n_chunks = s.n_chunks;
    k.chunk = s.chunk;
    k.n_rels = s.n_rels;
    return DG_OK;
}

int seg_shape(int32_t d_in, int32_t d_out, bool& proj) {
    proj = d_in == 64 && d_out == 32;
    return proj || (d_in == d_out && (d_in == 32 || d_in == 64)) ? DG_OK : DG_EINVAL;
}
}  // namespace

namespace {
// The launch dispatch of both kernels: runtime switches onto the instantiated template forms.
template <int NW>
void launch_seg(bool proj, int d_in, dim3 grid, dim3 block, hipStream_t st, const SegArgs& a) {
    if (proj)
        hipLaunchKernelGGL((spmm_seg_kernel<16, true, NW>), grid, block, 0, st, a);
    else if (d_in == 64)
        hipLaunchKernelGGL((spmm_seg_kernel<16, false, NW>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((spmm_seg_kernel<8, false, NW>), grid, block, 0, st, a);
}

template <int NW, bool PEER>
void launch_fs(bool proj, int d_in, dim3 grid, dim3 block, hipStream_t st, const FsArgs& a) {
    if (proj)
        hipLaunchKernelGGL((gcn_fused_seg_kernel<16, true, NW, PEER>), grid, block, 0, st, a);
    else if (d_in == 64)
        hipLaunchKernelGGL((gcn_fused_seg_kernel<16, false, NW, PEER>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((gcn_fused_seg_kernel<8, false, NW, PEER>), grid, block, 0, st, a);
}

int seg_launch(const dg_seg_group* groups, int32_t n_groups, int32_t d_in, int32_t d_out, void* stream) {
    if (n_groups < 0 || (n_groups > 0 && groups == nullptr)) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
    bool proj = false;
    if (seg_shape(d_in, d_out, proj) != DG_OK) return DG_EINVAL;
    SegArgs args{};
    int64_t blocks = 0;
    int ng = 0;
    int nw = kSegMinNW;
    for (int i = 0; i < n_groups; ++i)
        if (groups[i].chunk > nw && groups[i].n_rows > 0 && groups[i].n_rels > 0) nw = groups[i].chunk;
    if (nw > 16) return DG_EINVAL;
    args.nw = nw;
    for (int i = 0; i < n_groups; ++i) {
        const dg_seg_group& s = groups[i];
        bool skip = false;
        const int rc = convert_seg(s, proj, d_in, args.g[ng], skip);
        if (rc != DG_OK) return rc;
        if (skip) continue;
        SegGroupK& k = args.g[ng++];
        if (!s.out) return DG_EINVAL;
        if (!dg::aligned16(s.out)) return DG_EALIGN;
        k.rpb = nw / s.chunk;
        k.row_blocks = dg::ceil_div(s.n_rows, k.rpb);
        const int64_t items = (int64_t)s.n_chunks * k.row_blocks;
        k.n_blocks = static_cast<int32_t>(8 * ((items + 7) / 8));
        k.block_begin = static_cast<int32_t>(blocks);
        blocks += k.n_blocks;
        if (blocks > 0x7fffffff) return DG_EINVAL;
    }
    args.n_groups = ng;
    if (blocks == 0) return DG_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(blocks)), block(64 * nw);  // (launch bounds: 8 or 16 waves)
    if (nw <= 8)
        launch_seg<8>(proj, d_in, grid, block, st, args);
    else
        launch_seg<16>(proj, d_in, grid, block, st, args);
    return dg::launch_status();
}

int fused_seg_launch(const dg_seg_group* groups, int32_t n_groups, const dg_fused_target* targets, int32_t n_targets,
                     int32_t d_in, int32_t d_out, const dg_peer_xchg* xchg, void* stream) {
    if (n_groups < 1 || !groups || n_targets < 1 || !targets) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS || n_targets > DG_MAX_GROUPS) return DG_ETOOMANY;
    bool proj = false;
    if (seg_shape(d_in, d_out, proj) != DG_OK) return DG_EINVAL;
    FsArgs a{};
    for (int i = 0; i < n_groups; ++i) {
        bool skip = false;
        const int rc = convert_seg(groups[i], proj, d_in, a.g[i], skip);
        if (rc != DG_OK) return rc;
        if (groups[i].n_rels < 1 || groups[i].n_rows < 1) return DG_EINVAL;  // (convert_seg checked the chunks)
    }
    int64_t blocks = 0;
    int nw = 1;
    for (int t = 0; t < n_targets; ++t) {
        const dg_fused_target& s = targets[t];
        if (!s.out || !dg::aligned16(s.out) || s.n_rows < 0 || s.g_count < 1 || s.g_begin < 0 ||
            s.g_begin + s.g_count > n_groups || (s.flags & ~DG_EPI_RELU))
            return DG_EINVAL;
        int items = 0;
        for (int g = s.g_begin; g < s.g_begin + s.g_count; ++g) {
            if (groups[g].n_rows != s.n_rows) return DG_EINVAL;
            items += groups[g].n_rels;
        }
        if (items > 16) return DG_EINVAL;  // one wave per relation of the row
        const int waves = items;
        nw = waves > nw ? waves : nw;
        FsTargetK& k = a.t[t];
        k.out = s.out;
        k.n_rows = s.n_rows;
        k.g_begin = s.g_begin;
        k.g_count = s.g_count;
        k.relu = (s.flags & DG_EPI_RELU) ? 1 : 0;
        k.waves = waves;
    }
    // rows per workgroup: a target with fewer relations per row than the widest one fills the
    // workgroup's waves with more rows
    for (int t = 0; t < n_targets; ++t) {
        FsTargetK& k = a.t[t];
        k.rpb = nw / k.waves < kFsMaxRpb ? nw / k.waves : kFsMaxRpb;
        k.block_begin = static_cast<int32_t>(blocks);
        blocks += dg::ceil_div(k.n_rows, k.rpb);
    }
    if (blocks > 0x7fffffff) return DG_EINVAL;
    a.n_targets = n_targets;
    a.nw = nw;
    if (xchg) {
        const int rc = dg::peer_convert(xchg, a.P);
        if (rc != DG_OK) return rc;
        for (int t = 0; t < n_targets; ++t)  // 32-bit buffer offsets into each peer's copy
            if ((int64_t)targets[t].n_rows * d_out * 4 > 0x7fffffffLL) return DG_EINVAL;
        if (blocks == 0) blocks = 1;  // no rows here: one workgroup still takes part in the exchange
    }
    if (blocks == 0) return DG_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(blocks)), block(64 * nw);
    if (xchg) {
        if (nw <= 8)
            launch_fs<8, true>(proj, d_in, grid, block, st, a);
        else
            launch_fs<16, true>(proj, d_in, grid, block, st, a);
    } else if (nw <= 8) {
        launch_fs<8, false>(proj, d_in, grid, block, st, a);
    } else {
        launch_fs<16, false>(proj, d_in, grid, block, st, a);
    }
    return dg::launch_status();
}
}  // namespace

#ifdef DG_FSEG_PROF
// Profiling build only: copy the last fused-seg launch's stamps of form proj (0 / 1).
extern "C" int64_t dg_fseg_prof_copy(int proj, unsigned long long* host, int64_t max_blocks) {
    const int64_t n = max_blocks < kFsProfMaxBlocks ? max_blocks : kFsProfMaxBlocks;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fs_prof), n * 16 * kFsProfSlots * 8, (size_t)(proj ? 1 : 0) *
                            kFsProfMaxBlocks * 16 * kFsProfSlots * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return n;
}
extern "C" int dg_fseg_prof_clear() {
    static unsigned long long zero[2 * kFsProfMaxBlocks * 16 * kFsProfSlots] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fs_prof), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int dg_spmm_seg_f32(const dg_seg_group* groups, int32_t n_groups, int32_t d_in, int32_t d_out,
                               void* stream) {
    return seg_launch(groups, n_groups, d_in, d_out, stream);
}

extern "C" int dg_gcn_fused_seg_f32(const dg_seg_group* groups, int32_t n_groups, const dg_fused_target* targets,
                                    int32_t n_targets, int32_t d_in, int32_t d_out, void* stream) {
    return fused_seg_launch(groups, n_groups, targets, n_targets, d_in, d_out, nullptr, stream);
}

namespace {
int fused_tab_launch(const dg_wave_table* t, int32_t d_in, int32_t d_out, const dg_peer_xchg* xchg, void* stream) {
    if (!t) return DG_EINVAL;
    bool proj = false;
    if (seg_shape(d_in, d_out, proj) != DG_OK || (!proj && d_in != 64)) return DG_EINVAL;
    if (t->n_blocks < 0 || t->nw < 1 || t->nw > 16 || t->nw_stride != (t->nw <= 8 ? 8 : 16)) return DG_EINVAL;
    if (t->n_blocks == 0) return xchg ? DG_EINVAL : DG_OK;  // (an exchange needs a workgroup a rank)
    if (!t->pairs || !t->desc || !dg::aligned16(t->pairs) || (reinterpret_cast<uintptr_t>(t->desc) & 63))
        return DG_EALIGN;
    const int S = t->slot_pairs ? t->slot_pairs : 64;
    if (S != 16 && S != 32 && S != 48 && S != 64) return DG_EINVAL;
    if ((int64_t)t->n_blocks * t->nw_stride * S > 0x7fffffffLL) return DG_EINVAL;
    dg::PeerK P{};
    if (xchg) {
        const int rc = dg::peer_convert(xchg, P);
        if (rc != DG_OK) return rc;
    }
    const uint2* pr = reinterpret_cast<const uint2*>(t->pairs);
    const uint2* ov = reinterpret_cast<const uint2*>(t->ovf);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(t->n_blocks)), block(64 * t->nw);
#define DG_TAB_LAUNCH(PR, NWV, PE) \
    hipLaunchKernelGGL((gcn_tab_kernel<PR, NWV, PE>), grid, block, 0, st, pr, t->desc, ov, S, P)
    if (xchg) {
        if (t->nw_stride == 8) {
            if (proj) DG_TAB_LAUNCH(true, 8, true); else DG_TAB_LAUNCH(false, 8, true);
        } else {
            if (proj) DG_TAB_LAUNCH(true, 16, true); else DG_TAB_LAUNCH(false, 16, true);
        }
    } else {
        if (t->nw_stride == 8) {
            if (proj) DG_TAB_LAUNCH(true, 8, false); else DG_TAB_LAUNCH(false, 8, false);
        } else {
            if (proj) DG_TAB_LAUNCH(true, 16, false); else DG_TAB_LAUNCH(false, 16, false);
        }
    }
#undef DG_TAB_LAUNCH
    return dg::launch_status();
}
}  // namespace

extern "C" int dg_gcn_fused_tab_f32(const dg_wave_table* t, int32_t d_in, int32_t d_out, void* stream) {
    return fused_tab_launch(t, d_in, d_out, nullptr, stream);
}

extern "C" int dg_gcn_fused_tab_peer_f32(const dg_wave_table* t, int32_t d_in, int32_t d_out,
                                         const dg_peer_xchg* xchg, void* stream) {
    if (!xchg) return DG_EINVAL;
    return fused_tab_launch(t, d_in, d_out, xchg, stream);
}

extern "C" int dg_spmm_seg_tab_f32(const dg_wave_table* t, int32_t d_in, int32_t d_out, void* stream) {
    if (!t) return DG_EINVAL;
    bool proj = false;
    if (seg_shape(d_in, d_out, proj) != DG_OK || (!proj && d_in != 64)) return DG_EINVAL;
    if (t->n_blocks < 0 || t->nw < 1 || t->nw > 16 || t->nw_stride != (t->nw <= 8 ? 8 : 16)) return DG_EINVAL;
    if (t->n_blocks == 0) return DG_OK;
    if (!t->pairs || !t->desc || !dg::aligned16(t->pairs) || (reinterpret_cast<uintptr_t>(t->desc) & 63))
        return DG_EALIGN;
    const int S = t->slot_pairs ? t->slot_pairs : 64;
    if (S != 16 && S != 32 && S != 48 && S != 64) return DG_EINVAL;
    if ((int64_t)t->n_blocks * t->nw_stride * S > 0x7fffffffLL) return DG_EINVAL;
    const uint2* pr = reinterpret_cast<const uint2*>(t->pairs);
    const uint2* ov = reinterpret_cast<const uint2*>(t->ovf);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(t->n_blocks)), block(64 * t->nw);
    if (t->nw_stride == 8) {
        if (proj)
            hipLaunchKernelGGL((seg_tab_kernel<true, 8>), grid, block, 0, st, pr, t->desc, ov, S);
        else
            hipLaunchKernelGGL((seg_tab_kernel<false, 8>), grid, block, 0, st, pr, t->desc, ov, S);
    } else {
        if (proj)
            hipLaunchKernelGGL((seg_tab_kernel<true, 16>), grid, block, 0, st, pr, t->desc, ov, S);
        else
            hipLaunchKernelGGL((seg_tab_kernel<false, 16>), grid, block, 0, st, pr, t->desc, ov, S);
    }
    return dg::launch_status();
}

extern "C" int dg_gcn_fused_seg_peer_f32(const dg_seg_group* groups, int32_t n_groups,
                                         const dg_fused_target* targets, int32_t n_targets, int32_t d_in,
                                         int32_t d_out, const dg_peer_xchg* xchg, void* stream) {
    if (!xchg) return DG_EINVAL;
    return fused_seg_launch(groups, n_groups, targets, n_targets, d_in, d_out, xchg, stream);
}
