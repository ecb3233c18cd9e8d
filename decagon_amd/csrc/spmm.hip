// Relation-group CSR SpMM and the fused GCN layer for gfx950 (MI355X).
//
// Reference ops replaced (paths relative to the reference root):
//   tf.sparse_tensor_dense_matmul(adj_mats[edge_type][k], x)  decagon/deep/layers.py:90, :114
//   tf.sparse_tensor_dense_matmul(x_sparse_feat, weights_k)   decagon/deep/layers.py:89
//   tf.add_n(outputs) / tf.nn.l2_normalize(outputs, dim=1)     decagon/deep/layers.py:92-93, :116-117
//   tf.nn.relu(tf.add_n(hid1)) / tf.add_n(embeds)              decagon/deep/model.py:75, :88
//
// Data layout: a group's relations are stored as a chunk-merged CSR.
// For chunk c (a run of consecutive relations) and row r, the nonzeros of every relation of
// the chunk in row r are contiguous, [rowptr[c*n_rows + r], rowptr[c*n_rows + r + 1]), and
// each carries a virtual column v = k*n_cols + col: the row of the relation-stacked dense
// operand X = [X_0; X_1; ...] it multiplies.  Σ_{k in chunk} Â_k[r]·X_k is then one sparse
// dot product over one contiguous range — built once at upload, so no kernel ever looks up
// per-relation row pointers.
//
// Work decomposition: a wave owns one (chunk, row) range.  A dense row of width d is held by
// LP = d/4 lanes (one float4 each), so a wave consumes G = 64/LP nonzeros per step (d=64:
// 16 lanes x 4; d=32: 8 x 8).  64 (vcol, val) pairs come in with one coalesced load (the next
// 64 are prefetched while the current ones are consumed), are handed to the lane groups with
// ds_bpermute, and up to kUnroll 16-byte gathers per lane are kept in flight.  The G partial sums
// are folded with a shuffle butterfly: fixed order, no atomics.
// Partial mode writes out[c][r][:]; fused mode (one chunk per group) finishes the layer in
// the same workgroup: L2 norm per group, Σ over the node type's groups, relu, and optionally
// the next layer's projection of the finished row.
#include "common.h"
#include "dropout.h"
#include "peer.h"

#ifndef DG_PROJ_UNROLL
#define DG_PROJ_UNROLL 16  // W loads per batch of the projection chain (measured: 8 → 16 −0.4 µs at S)
#endif

#define DG_LP_SWITCH(LPV, CALL)                     \
    switch (LPV) {                                  \
        case 1: CALL(1); break;                     \
        case 2: CALL(2); break;                     \
        case 4: CALL(4); break;                     \
        case 8: CALL(8); break;                     \
        case 16: CALL(16); break;                   \
        case 32: CALL(32); break;                   \
        case 64: CALL(64); break;                   \
        default: return DG_EINVAL;                  \
    }

namespace {

struct SpmmGroupK {
    const int32_t* rowptr;
    const int32_t* vcol;
    const float* val;
    const float* x;
    float* out;
    int32_t x_ld;  // elements; the host guarantees x_rows * x_ld < 2^31
    int32_t n_rows;
    int32_t n_chunks;
    int32_t row_blocks;
    int32_t block_begin;
    int32_t n_blocks;
    int64_t chunk_x;  // shared pattern: elements between the chunks' X slabs (0: merged CSR)
    // DG_GROUP_DROPOUT (shared pattern only): per-chunk masks on the pattern's values
    const uint64_t* drop_state;  // NULL: no dropout
    const int32_t* drop_index;
    uint32_t drop_tag;
    float drop_keep;
    int32_t drop_stride;
    float beta;  // dg_spmm_csr_f32: out = acc + beta·out (0: out is written without being read)
};

// The dropout scale of nonzero p in chunk c (DG_GROUP_DROPOUT, dropout.h's stream).
__device__ __forceinline__ float drop_mul(const SpmmGroupK& g, uint32_t key, uint32_t base, int p) {
    const uint32_t e = g.drop_index ? (uint32_t)g.drop_index[p] : (uint32_t)p;
    return dg::keep_scale(key, base + e, g.drop_keep);
}

struct SpmmArgs {
    SpmmGroupK g[DG_MAX_GROUPS];
    int32_t n_groups;
    int32_t d;
};

#ifndef DG_ROWS_PER_WAVE
#define DG_ROWS_PER_WAVE 2
#endif
// partial mode: 4 waves x kRowsPerWave consecutive (chunk, row) items; a wave issues every row's
// pointers and first (vcol, val) batch before it gathers the first row, so the later rows' two
// dependent loads hide under the earlier rows' gathers
constexpr int kRowsPerWave = DG_ROWS_PER_WAVE;
constexpr int kRowsPerBlock = 4 * kRowsPerWave;
#ifndef DG_KUNROLL
#define DG_KUNROLL 8
#endif
#ifndef DG_GROUP_KUNROLL
#define DG_GROUP_KUNROLL 4
#endif
#ifndef DG_GROUP_U4_BLOCKS
#define DG_GROUP_U4_BLOCKS 2048
#endif
// Partial-mode launches of at least this many workgroups (8 waves a SIMD) keep kGroupUnroll
// gathers in flight instead of kUnroll: they are occupancy-bound and the shorter unroll holds
// fewer VGPRs (config P forward 432-435 → 421-424 µs, training 1.70 → 1.68 ms; 2 no better,
// 16 worse); smaller launches keep kUnroll (config S training: 4 costs 3-4 µs a step).  Same
// bits either way.
constexpr int kUnroll = DG_KUNROLL;  // gathers in flight per lane
constexpr int kGroupUnroll = DG_GROUP_KUNROLL;

// The first batch of 64 (vcol, val) pairs of a range (batch wpart): lane l holds pair l.
__device__ __forceinline__ void range_head(const SpmmGroupK& g, int beg, int end, int wpart, uint32_t dkey,
                                           uint32_t dbase, int& vc, float& vv) {
    const int lane = threadIdx.x & 63;
    const int base = beg + wpart * 64;
    vc = 0;
    vv = 0.f;
    if (base + lane < end) {
        vc = g.vcol[base + lane];
        vv = g.val[base + lane];
        if (g.drop_state) vv *= drop_mul(g, dkey, dbase, base + lane);
    }
}

// acc = Σ_{p in [beg, end)} val[p] * X[vcol[p]][:], over every wcount-th batch of 64
// starting at batch wpart, whose first batch (vc, vv) range_head loaded.  Returns the folded
// row in every lane (lane l holds columns 4(l%LP) .. 4(l%LP)+3).
// U nonzeros per lane group of batch entries [s0, s0 + U*G) (entries past n contribute 0):
// every lane's gathers are issued before the first fma.
template <int LP, int U>
__device__ __forceinline__ void gather_step(float4& acc, const float* __restrict__ xq, bool qact, int eoff, float v,
                                            int s0, int n, int sub) {
    constexpr int G = dg::kWave / LP;
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
        const bool ok = qact && (s0 + u * G + sub) < n;
        xv[u] = ok ? *reinterpret_cast<const float4*>(xq + o[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
        if (!ok) w[u] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) dg::fma4(acc, w[u], xv[u]);
}

// U gathers in flight per lane.  Each lane's fma order is the nonzero order for every U (the
// entries past n add 0), so every U gives the same bits.
template <int LP, int U = kUnroll>
__device__ __forceinline__ float4 range_body(const SpmmGroupK& g, const float* xb, int beg, int end, int d,
                                             int wpart, int wcount, uint32_t dkey, uint32_t dbase, int vc,
                                             float vv) {
    constexpr int G = dg::kWave / LP;
    const int lane = threadIdx.x & 63;
    const int sub = lane / LP;
    const int q = lane % LP;
    const bool qact = q * 4 < d;
    const float* __restrict__ xq = xb + q * 4;
    const int32_t* __restrict__ vcolp = g.vcol;
    const float* __restrict__ valp = g.val;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int stride = wcount * 64;
    int base = beg + wpart * 64;
#pragma unroll 1
    for (; base < end; base += stride) {
        const int n = min(64, end - base);
        const int eoff = vc * g.x_ld;
        const float v = vv;
        const int nb = base + stride;  // prefetch the next batch of this wave
        vc = 0;
        vv = 0.f;
        if (nb + lane < end) {
            vc = vcolp[nb + lane];
            vv = valp[nb + lane];
            if (g.drop_state) vv *= drop_mul(g, dkey, dbase, nb + lane);
        }
#pragma unroll 1
        for (int s0 = 0; s0 < n; s0 += U * G) gather_step<LP, U>(acc, xq, qact, eoff, v, s0, n, sub);
    }
    acc = dg::xor_sum4_from<LP>(acc);
    return acc;
}

template <int LP>
__device__ __forceinline__ float4 range_sum(const SpmmGroupK& g, const float* xb, int beg, int end, int d,
                                            int wpart = 0, int wcount = 1, uint32_t dkey = 0,
                                            uint32_t dbase = 0) {
    int vc;
    float vv;
    range_head(g, beg, end, wpart, dkey, dbase, vc, vv);
    return range_body<LP>(g, xb, beg, end, d, wpart, wcount, dkey, dbase, vc, vv);
}

// Partial mode: one wave per (chunk, row); writes out[c][r][:].
template <int LP, int U>
__global__ __launch_bounds__(256) void spmm_groups_kernel(const SpmmArgs args) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    int gi = 0;
#pragma unroll 1
    while (gi + 1 < args.n_groups && b >= args.g[gi + 1].block_begin) ++gi;
    const SpmmGroupK& g = args.g[gi];
    // XCD-contiguous item map: local block lb runs on XCD label lb % 8, and each XCD takes a
    // contiguous, chunk-major run of items, so one chunk's dense rows stay in one L2.
    const int lb = b - g.block_begin;
    const int per = g.n_blocks >> 3;
    const int item = (lb & 7) * per + (lb >> 3);
    if (item >= g.n_chunks * g.row_blocks) return;
    const int c = item / g.row_blocks;
    const int r0 = (item - c * g.row_blocks) * kRowsPerBlock + wave * kRowsPerWave;
    if (r0 >= g.n_rows) return;  // wave-uniform; no barriers in this kernel
    const int d = args.d;
    const int64_t slot0 = (int64_t)c * g.n_rows + r0;
    // shared pattern: every chunk reads rowptr[r] over its own X slab
    const int64_t ps0 = g.chunk_x ? r0 : slot0;
    const uint32_t dkey = g.drop_state ? dg::drop_key(g.drop_state, g.drop_tag) : 0u;
    const uint32_t dbase = (uint32_t)c * (uint32_t)g.drop_stride;
    const int nr = min(kRowsPerWave, g.n_rows - r0);  // this wave's rows (the last wave may hold fewer)
    int rp[kRowsPerWave + 1];
#pragma unroll
    for (int j = 0; j <= kRowsPerWave; ++j) rp[j] = g.rowptr[ps0 + min(j, nr)];
    int vc[kRowsPerWave];
    float vv[kRowsPerWave];
#pragma unroll
    for (int j = 0; j < kRowsPerWave; ++j) range_head(g, rp[j], rp[j + 1], 0, dkey, dbase, vc[j], vv[j]);
#pragma unroll
    for (int j = 0; j < kRowsPerWave; ++j) {
        if (j >= nr) break;
        const float4 acc = range_body<LP, U>(g, g.x + c * g.chunk_x, rp[j], rp[j + 1], d, 0, 1, dkey, dbase, vc[j],
                                          vv[j]);
        if (lane < LP && lane * 4 < d) {
            float4* o = reinterpret_cast<float4*>(g.out + (slot0 + j) * d + lane * 4);
            float4 y = acc;
            if (g.beta != 0.f) {  // kernel-argument uniform: tf.sparse_tensor_dense_matmul + beta·Y
                const float4 old = *o;
                y = make_float4(fmaf(g.beta, old.x, acc.x), fmaf(g.beta, old.y, acc.y), fmaf(g.beta, old.z, acc.z),
                                fmaf(g.beta, old.w, acc.w));
            }
            *o = y;
        }
    }
}

// Fused mode (every group of a node type in one chunk): one workgroup per RPB consecutive
// output rows of node type i; W waves per (row, group (i, j)) share the row's nonzeros.  The
// waves of a group meet in LDS, the group's first wave L2-normalises the group sum
// (layers.py:93), then the row's first wave adds the groups in order and applies relu
// (model.py:75) or not (model.py:88).
// Optional projection epilogue (layer 1 only): for every layer-2 group whose source node
// type is i, P_k[r][:] = out[r][:] · W2_k — the next layer's H_j·W_k (layers.py:113) for
// these rows, a k-ordered fmaf chain exactly like the MFMA path — so layer 2 needs no GEMM.
// A thread owns one (relation, column) of W2 and runs the chains of all RPB rows, so each W2
// column is read once per RPB rows (the projection reads W2 from L2 and is bound by those
// bytes: one row per workgroup read ≈40 KB of W2 per 256 B of output).
#ifndef DG_FUSED_RPB
#define DG_FUSED_RPB 1  // rows per workgroup, at most (measured at S: 4 rows 10.5 us, 2 rows 9.4, 1 row 9.0-9.2)
#endif
constexpr int kFusedRpb = DG_FUSED_RPB;

struct FusedTargetK {
    float* out;
    int32_t n_rows;
    int32_t g_begin;
    int32_t g_count;
    int32_t relu;
    int32_t block_begin;
    int32_t pad;
};

struct ProjK {
    const float* w;
    const int32_t* rel_map;
    float* out;
    int32_t n_rels;
    int32_t target;
    int32_t d_out;
    int32_t pad;
};

struct FusedArgs {
    SpmmGroupK g[DG_MAX_GROUPS];
    FusedTargetK t[DG_MAX_GROUPS];
    ProjK p[DG_MAX_GROUPS];
    int32_t n_groups;
    int32_t n_targets;
    int32_t n_projs;
    int32_t d;
    int32_t wpg;  // waves per group
    int32_t rpb;  // rows per workgroup (blockDim = 64 · rpb · max groups · wpg)
};

// The fused layer for workgroup b.
template <int LP>
__device__ __forceinline__ void fused_body(const FusedArgs& a, const int b) {
    __shared__ float4 pbuf[16][LP];
    __shared__ float4 ybuf[kFusedRpb][DG_MAX_GROUPS][LP];
    __shared__ float hrow[kFusedRpb][4 * LP];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int ti = 0;
#pragma unroll 1
    while (ti + 1 < a.n_targets && b >= a.t[ti + 1].block_begin) ++ti;
    const FusedTargetK& t = a.t[ti];
    const int d = a.d;
    const int W = a.wpg;
    const int RPB = a.rpb;
    const int wpr = (int)(blockDim.x >> 6) / RPB;  // waves per row slot
    const int slot = wave / wpr;
    const int wr = wave - slot * wpr;
    const int r0 = (b - t.block_begin) * RPB;
    const int r = r0 + slot;
    const bool live = r < t.n_rows;  // wave-uniform; every wave still meets every barrier
    const int gl = wr / W;
    const int part = wr - gl * W;
    const int q = lane % LP;
    if (live && gl < t.g_count) {
        const SpmmGroupK& g = a.g[t.g_begin + gl];
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!g.rowptr) {  // DG_GROUP_DENSE_ROWS: the sum is x[r], or Σ of its n_chunks slots in slot order
            if (part == 0 && q * 4 < d) {
                const float* xr = g.x + (int64_t)r * g.x_ld + q * 4;
#pragma unroll 1
                for (int c = 0; c < g.n_chunks; ++c) dg::add4(s, *reinterpret_cast<const float4*>(xr + c * g.chunk_x));
            }
        } else {
            s = range_sum<LP>(g, g.x, g.rowptr[r], g.rowptr[r + 1], d, part, W);
        }
        if (lane < LP) pbuf[wave][lane] = s;
    }
    __syncthreads();
    if (live && gl < t.g_count && part == 0) {
        float4 s = pbuf[wave][q];
        for (int w = 1; w < W; ++w) dg::add4(s, pbuf[wave + w][q]);
        // tf.nn.l2_normalize: x * rsqrt(max(sum(x^2), 1e-12)); columns >= d hold zeros
        float ss = s.x * s.x + s.y * s.y + s.z * s.z + s.w * s.w;
        ss = dg::xor_sum_below<LP>(ss);
        const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
        if (lane < LP) ybuf[slot][gl][lane] = make_float4(s.x * inv, s.y * inv, s.z * inv, s.w * inv);
    }
    __syncthreads();
    if (live && wr == 0 && lane < LP) {
        float4 tot = ybuf[slot][0][lane];
        for (int g = 1; g < t.g_count; ++g) dg::add4(tot, ybuf[slot][g][lane]);
        if (t.relu) {
            tot.x = fmaxf(tot.x, 0.f);
            tot.y = fmaxf(tot.y, 0.f);
            tot.z = fmaxf(tot.z, 0.f);
            tot.w = fmaxf(tot.w, 0.f);
        }
        if (lane * 4 < d) *reinterpret_cast<float4*>(t.out + (int64_t)r * d + lane * 4) = tot;
        reinterpret_cast<float4*>(hrow[slot])[lane] = tot;
    }
    if (a.n_projs == 0) return;  // launch-uniform
    __syncthreads();
    // every projection output (entry, relation, column) of this target in one index space, so
    // the block's threads run a single load/fmaf chain each instead of one chain per entry
    int total = 0;
#pragma unroll 1
    for (int pi = 0; pi < a.n_projs; ++pi)
        if (a.p[pi].target == ti) total += a.p[pi].n_rels * a.p[pi].d_out;
    const int nr = min(RPB, t.n_rows - r0);  // live rows of this workgroup
#pragma unroll 1
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
        int pi = 0, rem = idx;
#pragma unroll 1
        for (;; ++pi) {
            if (a.p[pi].target != ti) continue;
            const int n = a.p[pi].n_rels * a.p[pi].d_out;
            if (rem < n) break;
            rem -= n;
        }
        const ProjK& pj = a.p[pi];
        const int dout = pj.d_out;
        const int kk = rem / dout;
        const int c = rem - kk * dout;
        const int rel = pj.rel_map ? pj.rel_map[kk] : kk;
        const float* __restrict__ wcol = pj.w + (int64_t)rel * d * dout + c;
        float acc[kFusedRpb];
#pragma unroll
        for (int s2 = 0; s2 < kFusedRpb; ++s2) acc[s2] = 0.f;
#pragma unroll DG_PROJ_UNROLL
        for (int k = 0; k < d; ++k) {
            const float w = wcol[(int64_t)k * dout];
#pragma unroll
            for (int s2 = 0; s2 < kFusedRpb; ++s2) acc[s2] = fmaf(hrow[s2][k], w, acc[s2]);
        }
        float* po = pj.out + ((int64_t)rel * t.n_rows + r0) * dout + c;
#pragma unroll
        for (int s2 = 0; s2 < kFusedRpb; ++s2) {
            if (s2 >= nr) continue;
            po[(int64_t)s2 * dout] = acc[s2];
        }
    }
}

template <int LP>
__global__ __launch_bounds__(1024) void gcn_fused_kernel(const FusedArgs a) {
    fused_body<LP>(a, blockIdx.x);
}

struct EpiGroupK {
    const float* partial;
    float* sum;  // the group's pre-normalisation sum, or nullptr
    int32_t n_chunks;
    int32_t push;  // PEER launches: the sum also goes to every peer's copy (the peer all-reduce's slot)
};

struct EpiTargetK {
    float* out;
    int32_t n_rows;
    int32_t g_begin;      // its groups: g[g_begin .. g_begin + g_count)
    int32_t g_count;
    int32_t block_begin;  // its first workgroup
    int32_t push;         // PEER launches: its rows also go to every peer's copy (DG_EPI_PUSH)
    int32_t pad;
};

struct EpiArgs {
    EpiGroupK g[DG_MAX_GROUPS];
    EpiTargetK t[DG_EPI_MAX_TARGETS];
    int32_t n_targets;
    int32_t d;
    int32_t flags;
    int32_t pad;
    dg::PeerK P;  // PEER launches: the finished rows also go to every peer's copy (peer.h)
};

constexpr int kEpiBatch = 8;  // partial loads in flight a lane (epilogue_row)

// One wave per output row: LP lanes cover the row's d floats (a float4 each) and the
// wave's CG = 64/LP lane groups split the chunks (group cg sums chunks cg, cg+CG, ... with
// kEpiBatch loads in flight), combined by an xor butterfly — every lane ends with the same bits, so the
// result is deterministic; then the L2 norm over the row's LP lanes.
template <int LP, bool PEER>
__device__ __forceinline__ void epilogue_row(const EpiArgs& a, const EpiTargetK& t, int r, int cg, int q) {
    constexpr int CG = dg::kWave / LP;
    const int d = a.d;
    const bool qok = q * 4 < d;
    const int64_t plane = (int64_t)t.n_rows * d;
    const int64_t off = (int64_t)r * d + q * 4;
    const bool crelu = a.flags & DG_EPI_CHUNK_RELU;
    auto relu4 = [](float4 v) {
        return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
    };

    float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
    for (int gi = t.g_begin; gi < t.g_begin + t.g_count; ++gi) {
        const float* __restrict__ p = a.g[gi].partial + off;
        const int nc = a.g[gi].n_chunks;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        if (qok) {
            // eight loads in flight a lane, the last batch predicated: a staged group's 64-128
            // output chunks (16 a lane group) in two round trips instead of four
#pragma unroll 1
            for (int c = cg; c < nc; c += kEpiBatch * CG) {
                float4 v[kEpiBatch];
#pragma unroll
                for (int u = 0; u < kEpiBatch; ++u)
                    v[u] = c + u * CG < nc ? *reinterpret_cast<const float4*>(p + (c + u * CG) * plane)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int u = 0; u < kEpiBatch; ++u)
                    if (c + u * CG < nc) dg::add4(s, crelu ? relu4(v[u]) : v[u]);
            }
        }
        s = dg::xor_sum4_from<LP>(s);
        if (a.g[gi].sum && qok && cg == 0) {
            *reinterpret_cast<float4*>(a.g[gi].sum + off) = s;
            if constexpr (PEER)
                if (a.g[gi].push) dg::peer_store4(a.P, a.g[gi].sum, (uint32_t)(plane * 4), (uint32_t)(off * 4), s);
        }
        if (a.flags & DG_EPI_L2NORM) {
            // tf.nn.l2_normalize: x * rsqrt(max(sum(x^2), 1e-12)); all-zero rows stay zero.
            float ss = s.x * s.x + s.y * s.y + s.z * s.z + s.w * s.w;
            ss = dg::xor_sum_below<LP>(ss);
            const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
            s.x *= inv;
            s.y *= inv;
            s.z *= inv;
            s.w *= inv;
        }
        dg::opaque4(s);
        dg::add4(tot, s);
    }
    if (a.flags & DG_EPI_RELU) tot = relu4(tot);
    if (qok && cg == 0) {
        *reinterpret_cast<float4*>(t.out + off) = tot;
        if constexpr (PEER)
            if (t.push) dg::peer_store4(a.P, t.out, (uint32_t)(plane * 4), (uint32_t)(off * 4), tot);
    }
}

// PEER: the rows are also stored into every peer's copy of the row-split output and the launch
// ends with the peer-store exchange (peer.h: the last workgroup raises the flags and waits), so
// every wave reaches the closing barrier.
// The row-table form of the epilogue (dg_gcn_epilogue_tab_f32, round 5): one wave per row as
// above, the same sums in the same order (bitwise its rows), but each row's target, partial
// bases and chunk counts come from a host-built 64-byte descriptor, and every group's partial
// loads (up to two a lane a group: n_chunks <= 2·CG) are issued together — one round trip
// instead of the target search, then a kernel-argument and a partial round trip per group.
static_assert(sizeof(dg_epi_row_desc) == 64, "dg_epi_row_desc: one s_load_dwordx16");
template <int LP, bool PEER>
__global__ __launch_bounds__(256) void epilogue_tab_kernel(const dg_epi_row_desc* __restrict__ rows, int n_rows,
                                                           int flags, const dg::PeerK P) {
    constexpr int CG = dg::kWave / LP;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int cg = lane / LP;
    const int q = lane % LP;
    const int r = (int)blockIdx.x * 4 + wave;
    if (r < n_rows) {  // wave-uniform
        const dg_epi_row_desc D = rows[r];
        const int ng = D.info & 7;
        const bool crelu = flags & DG_EPI_CHUNK_RELU;
        auto relu4 = [](float4 v) {
            return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
        };
        float4 v[4][2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int nc = (D.n_chunks >> (8 * g)) & 0xff;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = cg + j * CG;
                v[g][j] = (g < ng && c < nc) ? *reinterpret_cast<const float4*>(D.part[g] + (int64_t)c * D.plane + q * 4)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (g >= ng) break;  // wave-uniform
            const int nc = (D.n_chunks >> (8 * g)) & 0xff;
            float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                if (cg + j * CG < nc) dg::add4(sm, crelu ? relu4(v[g][j]) : v[g][j]);
            // more chunks than two a lane group: four loads in flight, in order
            int c = cg + 2 * CG;
#pragma unroll 1
            for (; c + 3 * CG < nc; c += 4 * CG) {
                float4 w[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    w[u] = *reinterpret_cast<const float4*>(D.part[g] + (int64_t)(c + u * CG) * D.plane + q * 4);
#pragma unroll
                for (int u = 0; u < 4; ++u) dg::add4(sm, crelu ? relu4(w[u]) : w[u]);
            }
#pragma unroll 1
            for (; c < nc; c += CG) {
                const float4 w = *reinterpret_cast<const float4*>(D.part[g] + (int64_t)c * D.plane + q * 4);
                dg::add4(sm, crelu ? relu4(w) : w);
            }
            sm = dg::xor_sum4_from<LP>(sm);
            if (flags & DG_EPI_L2NORM) {
                float ss = sm.x * sm.x + sm.y * sm.y + sm.z * sm.z + sm.w * sm.w;
                ss = dg::xor_sum_below<LP>(ss);
                const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
                sm.x *= inv;
                sm.y *= inv;
                sm.z *= inv;
                sm.w *= inv;
            }
            dg::opaque4(sm);
            dg::add4(tot, sm);
        }
        if (flags & DG_EPI_RELU) tot = relu4(tot);
        if (cg == 0) {
            *reinterpret_cast<float4*>(D.out + D.off + q * 4) = tot;
            if constexpr (PEER)
                if ((D.info >> 8) & 1) dg::peer_store4(P, D.out, (uint32_t)D.bytes, (uint32_t)((D.off + q * 4) * 4), tot);
        }
    }
    if constexpr (PEER) dg::peer_arrive(P);
}

template <int LP, bool PEER>
__global__ __launch_bounds__(256) void epilogue_kernel(const EpiArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cg = lane / LP;
    const int q = lane % LP;
    int ti = 0;  // node type of this workgroup (several finish in one launch)
#pragma unroll 1
    while (ti + 1 < a.n_targets && (int)blockIdx.x >= a.t[ti + 1].block_begin) ++ti;
    const EpiTargetK& t = a.t[ti];
    const int r = ((int)blockIdx.x - t.block_begin) * 4 + wave;
    if (r < t.n_rows) epilogue_row<LP, PEER>(a, t, r, cg, q);  // wave-uniform
    if constexpr (PEER) dg::peer_arrive(a.P);
}

// Partial mode over a SMALL shared operand (every nonzero of the launch gathers from one
// dense X of at most kLdsRowsMax rows — the backward's Âᵀ·dS, whose operand dS_ij is the
// same for all K relations of the group): a workgroup copies a 32-float column slice of X
// into LDS once (rows 144 B apart: the 16-byte bank slot of float4 j of row v is
// (9v + j) mod 16, a bijection of v mod 16), then its 16 waves walk up to 16 x 128 (chunk, row)
// items, 16 rows at a time per wave: 4 lanes per row, two float4 column pieces each.  A row's
// (vcol, val) pairs come in 4 at a time with one coalesced load per lane group (the next 4
// prefetched), are handed out by shuffles (two per nonzero and 16 rows), and each gathers two
// ds_read_b128 per lane.
// No per-relation barrier, no operand re-read from L2.
constexpr int kLdsSlice = 32;                 // floats per column slice
constexpr int kLdsRowF4 = 9;                  // float4 slots per staged row (8 + 1 pad)
constexpr int kLdsRowsMax = 160 * 1024 / (16 * kLdsRowF4);
constexpr int kLdsItemsMax = 128;            // (chunk, row) items per wave (at most)

struct LdsGroupK {
    const int32_t* rowptr;
    const int32_t* vcol;
    const float* val;
    const float* x;
    float* out;
    int32_t x_ld;
    int32_t x_rows;
    int32_t n_items;      // n_chunks * n_rows
    int32_t item_blocks;  // ceil(n_items / (16 * per_wave))
    int32_t block_begin;
    int32_t per_wave;     // items per wave: a multiple of 16, <= kLdsItemsMax
    int32_t persist;      // workgroups per column slice; workgroup p takes item blocks p, p + persist, ...
};

struct LdsArgs {
    LdsGroupK g[DG_MAX_GROUPS];
    int32_t n_groups;
    int32_t d;
    int32_t n_slices;
    int32_t pad;
};

__global__ __launch_bounds__(1024) void spmm_lds_kernel(const LdsArgs a) {
    extern __shared__ float4 xs[];
    const int b = blockIdx.x;
    int gi = 0;
#pragma unroll 1
    while (gi + 1 < a.n_groups && b >= a.g[gi + 1].block_begin) ++gi;
    const LdsGroupK& g = a.g[gi];
    const int lb = b - g.block_begin;
    const int s = lb / g.persist;                 // column slice
    const int p0 = lb - s * g.persist;            // first item block
    const int d = a.d;
    const int c0 = s * kLdsSlice;
    const int cw = min(kLdsSlice, d - c0);        // columns of this slice (multiple of 4)
    // the slice staged with 8 loads in flight per thread (a load-store-per-iteration loop waits
    // one L2 round trip per float4: ≈ 150 in a row for 19,085 rows)
    const int total = g.x_rows * 8;
#pragma unroll 1
    for (int q0 = threadIdx.x; q0 < total; q0 += 8 * (int)blockDim.x) {
        float4 t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int q = q0 + k * (int)blockDim.x;
            const int v = q >> 3, j = q & 7;
            t[k] = (q < total && 4 * j < cw) ? *reinterpret_cast<const float4*>(g.x + (int64_t)v * g.x_ld + c0 + 4 * j)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int q = q0 + k * (int)blockDim.x;
            if (q < total) xs[(q >> 3) * kLdsRowF4 + (q & 7)] = t[k];
        }
    }
    __syncthreads();  // the only barrier
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int rg = lane >> 2;                     // row of the wave's 16
    const int q = lane & 3;                       // float4 pieces q and q + 4 of the slice
    const bool qok0 = 4 * q < cw, qok1 = 4 * (q + 4) < cw;
    // the slice is staged once per workgroup; the workgroup then walks its item blocks
#pragma unroll 1
    for (int ib = p0; ib < g.item_blocks; ib += g.persist) {
        // this wave's per_wave (<= 128) consecutive items: their row pointers in three registers
        // (one coalesced load), so a row's range never waits on memory
        const int pw = g.per_wave;
        const int wbase = (ib * 16 + wave) * pw;
        const int item_end = min(g.n_items, wbase + pw);
        if (wbase >= item_end) continue;
        const int rp0 = g.rowptr[min(wbase + lane, g.n_items)];
        const int rp1 = g.rowptr[min(wbase + 64 + lane, g.n_items)];
        const int rp2 = g.rowptr[min(wbase + 128, g.n_items)];  // (read only when pw == 128)
        auto rp = [&](int idx) {  // row pointer wbase + idx, idx in [0, 128]
            const int v0 = __shfl(rp0, idx & 63), v1 = __shfl(rp1, idx & 63);
            return idx < 64 ? v0 : (idx < 128 ? v1 : rp2);
        };
        int nb = rp(rg), ne = rp(rg + 1);
        int npc = nb + q < ne ? g.vcol[nb + q] : 0;
        float npv = nb + q < ne ? g.val[nb + q] : 0.f;
#pragma unroll 1
        for (int t = 0; wbase + 16 * t < item_end; ++t) {
            const int item = wbase + 16 * t + rg;
            const int beg = nb, end = ne;
            int vc = npc;
            float vv = npv;
            if (16 * t + 16 < pw) {  // the next 16 rows' ranges and first pairs
                nb = rp(16 * t + 16 + rg);
                ne = rp(16 * t + 17 + rg);
                npc = nb + q < ne ? g.vcol[nb + q] : 0;
                npv = nb + q < ne ? g.val[nb + q] : 0.f;
            }
            float4 acc0 = make_float4(0.f, 0.f, 0.f, 0.f), acc1 = acc0;
#pragma unroll 1
            for (int cb = beg; __any(cb < end); cb += 4) {
                const int cv = vc;
                const float w = vv;
                const int p = cb + 4 + q;  // the next 4 pairs of this row
                vc = p < end ? g.vcol[p] : 0;
                vv = p < end ? g.val[p] : 0.f;
                // pair u of the row's four goes to the row's 4 lanes by a DPP quad broadcast
                // (quad_perm [u,u,u,u]: a VALU move, no LDS instruction beside the gathers)
                const int xv4[4] = {__builtin_amdgcn_mov_dpp(cv, 0x00, 0xF, 0xF, false),
                                    __builtin_amdgcn_mov_dpp(cv, 0x55, 0xF, 0xF, false),
                                    __builtin_amdgcn_mov_dpp(cv, 0xAA, 0xF, 0xF, false),
                                    __builtin_amdgcn_mov_dpp(cv, 0xFF, 0xF, 0xF, false)};
                const int wi = __float_as_int(w);
                const int wv4[4] = {__builtin_amdgcn_mov_dpp(wi, 0x00, 0xF, 0xF, false),
                                    __builtin_amdgcn_mov_dpp(wi, 0x55, 0xF, 0xF, false),
                                    __builtin_amdgcn_mov_dpp(wi, 0xAA, 0xF, 0xF, false),
                                    __builtin_amdgcn_mov_dpp(wi, 0xFF, 0xF, 0xF, false)};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float wv = __int_as_float(wv4[u]);  // 0 past the row's end
                    const float4* xr = xs + xv4[u] * kLdsRowF4;
                    dg::fma4(acc0, wv, xr[q]);
                    dg::fma4(acc1, wv, xr[q + 4]);
                }
            }
            float* o = g.out + (int64_t)item * d + c0;
            if (item < item_end && qok0) *reinterpret_cast<float4*>(o + 4 * q) = acc0;
            if (item < item_end && qok1) *reinterpret_cast<float4*>(o + 4 * (q + 4)) = acc1;
        }
    }
}

}  // namespace

extern "C" int32_t dg_abi_version(void) { return 38; }


namespace {

// Validate one descriptor and copy it into the kernel form.  Returns DG_OK or an error.
int convert_group(const dg_rel_group& s, int d, bool need_out, SpmmGroupK& k, bool allow_shared = false,
                  bool allow_dense = false) {
    if (s.n_rows < 0 || s.n_chunks < 1 || s.x_rows < 0) return DG_EINVAL;
    if (s.flags & ~(DG_GROUP_SHARED_PATTERN | DG_GROUP_DROPOUT | DG_GROUP_DENSE_ROWS)) return DG_EINVAL;
    if (s.flags & DG_GROUP_DENSE_ROWS) {  // row r of the sum is x[r]: no adjacency
        if (!allow_dense || s.flags != DG_GROUP_DENSE_ROWS || s.n_chunks < 1 || s.n_chunks > DG_PEER_MAX ||
            s.x_rows < s.n_rows || !s.x)
            return DG_EINVAL;
        if (!dg::aligned16(s.x) || (s.x_ld & 3)) return DG_EALIGN;
        if (s.x_ld < d || (int64_t)s.x_rows * s.x_ld > 0x7fffffffLL) return DG_EINVAL;
        k = SpmmGroupK{};
        k.x = s.x;
        k.x_ld = static_cast<int32_t>(s.x_ld);
        k.n_rows = s.n_rows;
        k.n_chunks = s.n_chunks;                  // slots, summed in slot order
        k.chunk_x = (int64_t)s.x_rows * s.x_ld;  // slot c at x + c·x_rows·x_ld
        k.drop_keep = 1.f;
        return DG_OK;  // k.rowptr == nullptr marks the dense form in the kernel
    }
    if ((s.flags & DG_GROUP_SHARED_PATTERN) && !allow_shared) return DG_EINVAL;
    if (s.flags & DG_GROUP_DROPOUT) {  // per-chunk masks of a shared pattern only
        if (!(s.flags & DG_GROUP_SHARED_PATTERN) || !s.drop_state || s.drop_stride < 0) return DG_EINVAL;
        if (!(s.drop_keep > 0.f && s.drop_keep <= 1.f)) return DG_EINVAL;
        if ((int64_t)s.n_chunks * s.drop_stride > 0xffffffffLL) return DG_EINVAL;  // 32-bit mask counter
    }
    // vcol/val may be NULL for a group without nonzeros (rowptr all zero: never read)
    if (!s.rowptr || !s.x || (need_out && !s.out)) return DG_EINVAL;
    if (!dg::aligned16(s.x) || (need_out && !dg::aligned16(s.out)) || (s.x_ld & 3)) return DG_EALIGN;
    if (s.x_ld < d) return DG_EINVAL;
    if ((int64_t)s.x_rows * s.x_ld > 0x7fffffffLL) return DG_EINVAL;  // 32-bit gather offsets
    k.rowptr = s.rowptr;
    k.vcol = s.vcol;
    k.val = s.val;
    k.x = s.x;
    k.out = s.out;
    k.x_ld = static_cast<int32_t>(s.x_ld);
    k.n_rows = s.n_rows;
    k.n_chunks = s.n_chunks;
    k.row_blocks = dg::ceil_div(s.n_rows, kRowsPerBlock);
    k.chunk_x = (s.flags & DG_GROUP_SHARED_PATTERN) ? (int64_t)s.x_rows * s.x_ld : 0;
    const bool drop = (s.flags & DG_GROUP_DROPOUT) != 0;
    k.drop_state = drop ? s.drop_state : nullptr;
    k.drop_index = drop ? s.drop_index : nullptr;
    k.drop_tag = s.drop_tag;
    k.drop_keep = drop ? s.drop_keep : 1.f;
    k.drop_stride = drop ? s.drop_stride : 0;
    return DG_OK;
}

}  // namespace

extern "C" int dg_spmm_groups_f32(const dg_rel_group* groups, int32_t n_groups, int32_t d,
                                  void* stream) {
    if (n_groups < 0 || (n_groups > 0 && groups == nullptr)) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
    if (d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    SpmmArgs args{};
    args.d = d;
    int64_t blocks = 0;
    int ng = 0;
    for (int i = 0; i < n_groups; ++i) {
        const dg_rel_group& s = groups[i];
        if (s.n_rows == 0) continue;
        SpmmGroupK& k = args.g[ng];
        const int rc = convert_group(s, d, true, k, true);
        if (rc != DG_OK) return rc;
        ++ng;
        const int64_t items = (int64_t)k.n_chunks * k.row_blocks;
        k.n_blocks = static_cast<int32_t>(8 * ((items + 7) / 8));
        k.block_begin = static_cast<int32_t>(blocks);
        blocks += k.n_blocks;
        if (blocks > 0x7fffffff) return DG_EINVAL;
    }
    args.n_groups = ng;
    if (blocks == 0) return DG_OK;
    const int lp = dg::lanes_per_row(d);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(blocks)), block(256);
#define DG_LAUNCH_SPMM(L)                                                                  \
    if (blocks >= DG_GROUP_U4_BLOCKS)                                                     \
        hipLaunchKernelGGL((spmm_groups_kernel<L, kGroupUnroll>), grid, block, 0, st, args); \
    else                                                                                  \
        hipLaunchKernelGGL((spmm_groups_kernel<L, kUnroll>), grid, block, 0, st, args)
    DG_LP_SWITCH(lp, DG_LAUNCH_SPMM)
#undef DG_LAUNCH_SPMM
    return dg::launch_status();
}

namespace {
// The fused launch's arguments, grid and workgroup size (dg_gcn_fused_f32's checks).
int prep_fused(const dg_rel_group* groups, int32_t n_groups, const dg_fused_target* targets, int32_t n_targets,
               const dg_proj* projs, int32_t n_projs, int32_t waves_per_group, int32_t d, FusedArgs& a,
               int64_t& blocks, int& threads) {
    if (n_groups < 1 || !groups || n_targets < 1 || !targets) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS || n_targets > DG_MAX_GROUPS || n_projs > DG_MAX_GROUPS)
        return DG_ETOOMANY;
    if (n_projs < 0 || (n_projs > 0 && !projs)) return DG_EINVAL;
    if (d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    if (waves_per_group < 1) return DG_EINVAL;
    a.d = d;
    a.n_groups = n_groups;
    a.n_targets = n_targets;
    a.n_projs = n_projs;
    a.wpg = waves_per_group;
    for (int i = 0; i < n_groups; ++i) {
        // fused mode: the whole group is one chunk (dense rows: n_chunks slots)
        if (groups[i].n_chunks != 1 && !(groups[i].flags & DG_GROUP_DENSE_ROWS)) return DG_EINVAL;
        const int rc = convert_group(groups[i], d, false, a.g[i], false, true);
        if (rc != DG_OK) return rc;
    }
    blocks = 0;
    int max_groups = 1;
    for (int t = 0; t < n_targets; ++t) {
        const dg_fused_target& s = targets[t];
        if (!s.out || !dg::aligned16(s.out) || s.n_rows < 0 || s.g_count < 1 || s.g_begin < 0 ||
            s.g_begin + s.g_count > n_groups || (s.flags & ~DG_EPI_RELU))
            return DG_EINVAL;
        for (int g = s.g_begin; g < s.g_begin + s.g_count; ++g)
            if (a.g[g].n_rows != s.n_rows) return DG_EINVAL;
        FusedTargetK& k = a.t[t];
        k.out = s.out;
        k.n_rows = s.n_rows;
        k.g_begin = s.g_begin;
        k.g_count = s.g_count;
        k.relu = (s.flags & DG_EPI_RELU) ? 1 : 0;
        max_groups = s.g_count > max_groups ? s.g_count : max_groups;
    }
    if (max_groups * waves_per_group > 16) return DG_EINVAL;  // 1024 threads per workgroup
    // rows per workgroup: as many row slots as fit 1024 threads (at most kFusedRpb)
    int rpb = 16 / (max_groups * waves_per_group);
    rpb = rpb < 1 ? 1 : (rpb > kFusedRpb ? kFusedRpb : rpb);
    a.rpb = rpb;
    for (int t = 0; t < n_targets; ++t) {
        a.t[t].block_begin = static_cast<int32_t>(blocks);
        blocks += dg::ceil_div(targets[t].n_rows, rpb);
    }
    for (int i = 0; i < n_projs; ++i) {
        const dg_proj& s = projs[i];
        if (!s.w || !s.out || s.n_rels < 0 || s.d_out < 1 || s.target < 0 || s.target >= n_targets)
            return DG_EINVAL;
        a.p[i] = ProjK{s.w, s.rel_map, s.out, s.n_rels, s.target, s.d_out, 0};
    }
    if (blocks > 0x7fffffff) return DG_EINVAL;
    threads = 64 * rpb * max_groups * waves_per_group;
    return DG_OK;
}
}  // namespace

extern "C" int dg_gcn_fused_f32(const dg_rel_group* groups, int32_t n_groups,
                                const dg_fused_target* targets, int32_t n_targets,
                                const dg_proj* projs, int32_t n_projs, int32_t waves_per_group,
                                int32_t d, void* stream) {
    FusedArgs a{};
    int64_t blocks = 0;
    int threads = 0;
    const int rc = prep_fused(groups, n_groups, targets, n_targets, projs, n_projs, waves_per_group, d, a, blocks,
                              threads);
    if (rc != DG_OK) return rc;
    if (blocks == 0) return DG_OK;
    const int lp = dg::lanes_per_row(d);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(blocks)), block(threads);
#define DG_LAUNCH_FUSED(L) hipLaunchKernelGGL(gcn_fused_kernel<L>, grid, block, 0, st, a)
    DG_LP_SWITCH(lp, DG_LAUNCH_FUSED)
#undef DG_LAUNCH_FUSED
    return dg::launch_status();
}

extern "C" int dg_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                               int32_t n_rows, int32_t n_cols, const float* x, int64_t ldx,
                               float* y, int64_t ldy, int32_t d, float beta, void* stream) {
    if (ldy != d || !(beta == beta) || beta == INFINITY || beta == -INFINITY) return DG_EINVAL;
    if (n_rows < 0 || n_cols < 0 || d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    if (n_rows == 0) return DG_OK;
    dg_rel_group s{};
    s.rowptr = rowptr;
    s.vcol = col;
    s.val = val;
    s.x = x;
    s.out = y;
    s.x_ld = ldx;
    s.n_rows = n_rows;
    s.n_chunks = 1;
    s.x_rows = n_cols;
    SpmmArgs args{};
    args.d = d;
    SpmmGroupK& k = args.g[0];
    const int rc = convert_group(s, d, true, k);
    if (rc != DG_OK) return rc;
    k.beta = beta;
    k.n_blocks = static_cast<int32_t>(8 * ((k.row_blocks + 7) / 8));
    k.block_begin = 0;
    args.n_groups = 1;
    const int lp = dg::lanes_per_row(d);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(k.n_blocks)), block(256);
#define DG_LAUNCH_CSR(L) hipLaunchKernelGGL((spmm_groups_kernel<L, kUnroll>), grid, block, 0, st, args)
    DG_LP_SWITCH(lp, DG_LAUNCH_CSR)
#undef DG_LAUNCH_CSR
    return dg::launch_status();
}

extern "C" int dg_rownorm_l2_f32(const float* x, float* y, int32_t n_rows, int32_t d, int32_t flags, void* stream) {
    if (flags & ~DG_EPI_RELU) return DG_EINVAL;
    if (n_rows < 0 || d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    if (n_rows == 0) return DG_OK;
    if (!x || !y) return DG_EINVAL;
    const dg_epi_group g{x, nullptr, 1, 0};
    return dg_gcn_epilogue_f32(&g, 1, y, n_rows, d, DG_EPI_L2NORM | flags, stream);
}

namespace {
int epilogue_launch(const dg_epi_target* targets, int32_t n_targets, int32_t d, int32_t flags,
                    const dg_peer_xchg* xchg, void* stream) {
    if (n_targets < 1 || targets == nullptr) return DG_EINVAL;
    if (n_targets > DG_EPI_MAX_TARGETS) return DG_ETOOMANY;
    if (d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    if (flags & ~(DG_EPI_L2NORM | DG_EPI_RELU | DG_EPI_CHUNK_RELU)) return DG_EINVAL;
    EpiArgs a{};
    int ng = 0;
    int64_t blocks = 0;
    for (int ti = 0; ti < n_targets; ++ti) {
        const dg_epi_target& T = targets[ti];
        if (T.n_groups < 1 || !T.groups || T.n_rows < 0) return DG_EINVAL;
        if (ng + T.n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
        if (T.n_rows == 0) continue;
        if (!T.out || !dg::aligned16(T.out)) return T.out ? DG_EALIGN : DG_EINVAL;
        EpiTargetK& k = a.t[a.n_targets++];
        k.out = T.out;
        k.n_rows = T.n_rows;
        k.g_begin = ng;
        k.g_count = T.n_groups;
        k.block_begin = static_cast<int32_t>(blocks);
        if (T.target_flags & ~DG_EPI_PUSH) return DG_EINVAL;
        k.push = (xchg && (T.target_flags & DG_EPI_PUSH)) ? 1 : 0;
        for (int i = 0; i < T.n_groups; ++i) {
            if (!T.groups[i].partial || T.groups[i].n_chunks < 1) return DG_EINVAL;
            if (!dg::aligned16(T.groups[i].partial) || !dg::aligned16(T.groups[i].sum_out)) return DG_EALIGN;
            a.g[ng].partial = T.groups[i].partial;
            a.g[ng].sum = T.groups[i].sum_out;
            a.g[ng].n_chunks = T.groups[i].n_chunks;
            if (T.groups[i].group_flags & ~DG_EPI_PUSH) return DG_EINVAL;
            if ((T.groups[i].group_flags & DG_EPI_PUSH) && !T.groups[i].sum_out) return DG_EINVAL;
            a.g[ng].push = (xchg && (T.groups[i].group_flags & DG_EPI_PUSH)) ? 1 : 0;
            ++ng;
        }
        blocks += dg::ceil_div(T.n_rows, 4);  // one wave per row
    }
    if (blocks == 0) {
        if (!xchg) return DG_OK;
        blocks = 1;  // no rows here: one workgroup still takes part in the exchange
    }
    if (blocks > 0x7fffffff) return DG_EINVAL;
    a.d = d;
    a.flags = flags;
    const int lp = dg::lanes_per_row(d);
    dim3 grid(static_cast<unsigned>(blocks)), block(256);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (xchg) {
        const int rc = dg::peer_convert(xchg, a.P);
        if (rc != DG_OK) return rc;
        for (int ti = 0; ti < a.n_targets; ++ti)  // 32-bit buffer offsets into each peer's copy
            if ((int64_t)a.t[ti].n_rows * d * 4 > 0x7fffffffLL) return DG_EINVAL;
#define DG_LAUNCH_EPI(L) hipLaunchKernelGGL((epilogue_kernel<L, true>), grid, block, 0, st, a)
        DG_LP_SWITCH(lp, DG_LAUNCH_EPI)
#undef DG_LAUNCH_EPI
    } else {
#define DG_LAUNCH_EPI(L) hipLaunchKernelGGL((epilogue_kernel<L, false>), grid, block, 0, st, a)
        DG_LP_SWITCH(lp, DG_LAUNCH_EPI)
#undef DG_LAUNCH_EPI
    }
    return dg::launch_status();
}
}  // namespace

extern "C" int dg_gcn_epilogue_tab_f32(const dg_epi_row_desc* rows, int32_t n_rows, int32_t d, int32_t flags,
                                       const dg_peer_xchg* xchg, void* stream) {
    if (n_rows < 0 || (d != 32 && d != 64)) return DG_EINVAL;
    if (flags & ~(DG_EPI_L2NORM | DG_EPI_RELU | DG_EPI_CHUNK_RELU)) return DG_EINVAL;
    if (n_rows > 0 && (!rows || (reinterpret_cast<uintptr_t>(rows) & 63))) return rows ? DG_EALIGN : DG_EINVAL;
    int64_t blocks = dg::ceil_div(n_rows, 4);
    if (blocks == 0) {
        if (!xchg) return DG_OK;
        blocks = 1;  // no rows here: one workgroup still takes part in the exchange
    }
    dg::PeerK P{};
    if (xchg) {
        const int rc = dg::peer_convert(xchg, P);
        if (rc != DG_OK) return rc;
    }
    dim3 grid(static_cast<unsigned>(blocks)), block(256);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (d == 64) {
        if (xchg)
            hipLaunchKernelGGL((epilogue_tab_kernel<16, true>), grid, block, 0, st, rows, n_rows, flags, P);
        else
            hipLaunchKernelGGL((epilogue_tab_kernel<16, false>), grid, block, 0, st, rows, n_rows, flags, P);
    } else {
        if (xchg)
            hipLaunchKernelGGL((epilogue_tab_kernel<8, true>), grid, block, 0, st, rows, n_rows, flags, P);
        else
            hipLaunchKernelGGL((epilogue_tab_kernel<8, false>), grid, block, 0, st, rows, n_rows, flags, P);
    }
    return dg::launch_status();
}

extern "C" int dg_gcn_epilogue_multi_f32(const dg_epi_target* targets, int32_t n_targets, int32_t d,
                                         int32_t flags, void* stream) {
    return epilogue_launch(targets, n_targets, d, flags, nullptr, stream);
}

extern "C" int dg_gcn_epilogue_peer_f32(const dg_epi_target* targets, int32_t n_targets, int32_t d, int32_t flags,
                                        const dg_peer_xchg* xchg, void* stream) {
    if (!xchg) return DG_EINVAL;
    return epilogue_launch(targets, n_targets, d, flags, xchg, stream);
}

extern "C" int dg_gcn_epilogue_f32(const dg_epi_group* groups, int32_t n_groups, float* out,
                                   int32_t n_rows, int32_t d, int32_t flags, void* stream) {
    if (n_groups < 1 || groups == nullptr) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
    if (d < 4 || d > 256 || (d & 3) || n_rows < 0) return DG_EINVAL;
    if (flags & ~(DG_EPI_L2NORM | DG_EPI_RELU | DG_EPI_CHUNK_RELU)) return DG_EINVAL;
    if (n_rows == 0) return DG_OK;
    if (!out || !dg::aligned16(out)) return out ? DG_EALIGN : DG_EINVAL;
    const dg_epi_target t{groups, n_groups, 0, out, n_rows, 0, {0, 0}};
    return dg_gcn_epilogue_multi_f32(&t, 1, d, flags, stream);
}

extern "C" int dg_spmm_groups_lds_f32(const dg_rel_group* groups, int32_t n_groups, int32_t d, void* stream) {
    if (n_groups < 0 || (n_groups > 0 && groups == nullptr)) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
    if (d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    LdsArgs a{};
    a.d = d;
    a.n_slices = dg::ceil_div(d, kLdsSlice);
    int64_t blocks = 0, total_items = 0;
    int max_rows = 0;
    for (int i = 0; i < n_groups; ++i) {
        const dg_rel_group& s = groups[i];
        if (s.n_rows == 0) continue;
        SpmmGroupK k;
        const int rc = convert_group(s, d, true, k);
        if (rc != DG_OK) return rc;
        if (s.x_rows > kLdsRowsMax || !dg::aligned16(s.out)) return s.x_rows > kLdsRowsMax ? DG_EINVAL : DG_EALIGN;
        const int64_t items = (int64_t)s.n_chunks * s.n_rows;
        if (items > 0x7fffffff) return DG_EINVAL;
        LdsGroupK& g = a.g[a.n_groups++];
        g.rowptr = k.rowptr;
        g.vcol = k.vcol;
        g.val = k.val;
        g.x = k.x;
        g.out = k.out;
        g.x_ld = k.x_ld;
        g.x_rows = s.x_rows;
        g.n_items = static_cast<int32_t>(items);
        // items per wave: ~2048 item blocks of 16 waves for balance over the resident
        // workgroups, 16..128 items per wave
        int pw = static_cast<int>((items + 2048 * 16 - 1) / (2048 * 16));
        pw = pw < 16 ? 16 : (pw > kLdsItemsMax ? kLdsItemsMax : (pw + 15) / 16 * 16);
        g.per_wave = pw;
        g.item_blocks = dg::ceil_div(items, 16 * pw);
        total_items += items;
        max_rows = s.x_rows > max_rows ? s.x_rows : max_rows;
    }
    if (a.n_groups == 0) return DG_OK;
    const int lds = max_rows * kLdsRowF4 * 16;
    // persistent workgroups: as many as are resident at once (two 1024-thread workgroups per CU
    // at most, fewer when the staged slice is large), shared by the groups in proportion to
    // their items, so each slice is staged once per resident workgroup instead of once per
    // item block
    const int per_cu = lds > 0 ? (160 * 1024 / lds < 2 ? 1 : 2) : 2;
    const int64_t resident = 256LL * per_cu;
    for (int i = 0; i < a.n_groups; ++i) {
        LdsGroupK& g = a.g[i];
        int64_t share = (resident * g.n_items + total_items - 1) / total_items;
        share = (share + a.n_slices - 1) / a.n_slices;
        g.persist = static_cast<int32_t>(share < 1 ? 1 : (share > g.item_blocks ? g.item_blocks : share));
        g.block_begin = static_cast<int32_t>(blocks);
        blocks += (int64_t)g.persist * a.n_slices;
    }
    if (blocks > 0x7fffffff) return DG_EINVAL;
    static std::atomic<uint64_t> configured{0};
    dg::lds_optin(reinterpret_cast<const void*>(&spmm_lds_kernel), 160 * 1024, configured);
    hipLaunchKernelGGL(spmm_lds_kernel, dim3(static_cast<unsigned>(blocks)), dim3(1024), lds,
                       reinterpret_cast<hipStream_t>(stream), a);
    return dg::launch_status();
}
