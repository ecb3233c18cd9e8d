// Training-step kernels for gfx950 (MI355X): the backward of the hinge cost through the
// edge decoder and the row L2 normalisation, and TF 1.8's Adam update.
//
// Replaces (paths relative to the reference root):
//   tf.train.AdamOptimizer(lr).minimize(cost)            decagon/deep/optimizer.py:108-114
//     - the gradient of DecagonOptimizer._hinge_loss      optimizer.py:116-120
//       through batch_predict's u·L·G·L·v                 optimizer.py:51-57, :63-85
//       and the gathers from the embeddings               optimizer.py:66-76
//     - the gradient of tf.nn.l2_normalize(dim=1)         layers.py:93, :117
//       and of relu(add_n(.))                              model.py:75
//     - ApplyAdam on every variable                       (TF 1.8 training_ops)
// The SpMM / GEMM pieces of the backward (Âᵀ·G, Hᵀ·dP, Σ_k dP_k·W_kᵀ) reuse
// dg_spmm_groups_f32 and dg_gemm_f32 (spmm.hip, gemm.hip).
//
// Sums run in a fixed order (no float atomics): results are bitwise reproducible.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kPairChunk = 64;   // pairs per dM partial

// ---------------------------------------------------------------- decoder, per pair
// One wave per pair p.  With a_p = [neg_p - (pos_p - margin) > 0] (relu's gradient mask)
// the cost's gradient w.r.t. the positive score is -a_p and w.r.t. the negative one +a_p,
// and with M = L·G·L (L = diag(l)):
//   grad_rows[p]     = -a_p · M·v_p          (the positive row u_p)
//   grad_rows[n + p] = +a_p · M·v_p          (the negative row un_p)
//   grad_cols[p]     =  a_p · Mᵀ·(un_p - u_p)
//   xw[p] = a_p·(un_p - u_p),  vw[p] = v_p   (operands of dM = Σ_p xw[p]·vw[p]ᵀ)
struct PairArgs {
    const float* row_table;
    const float* col_table;
    const int32_t* rows;
    const int32_t* cols;
    const int32_t* negs;
    const float* pos;
    const float* neg;
    const float* G;
    const float* l;
    float* grad_rows;
    float* grad_cols;
    float* xw;
    float* vw;
    int64_t ld_row;
    int64_t ld_col;
    int32_t n;
    int32_t d;
    float margin;
    int32_t pad;
};

__global__ __launch_bounds__(256) void decoder_grad_pairs_kernel(const PairArgs a) {
    __shared__ float lv_s[4][256];
    __shared__ float dd_s[4][256];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int p = blockIdx.x * 4 + w;
    if (p >= a.n) return;  // wave-uniform; no block barriers below
    const int d = a.d;
    const float z = a.neg[p] - (a.pos[p] - a.margin);
    const bool act = z > 0.f;
    const float* u = a.row_table + (int64_t)a.rows[p] * a.ld_row;
    const float* un = a.row_table + (int64_t)a.negs[p] * a.ld_row;
    const float* v = a.col_table + (int64_t)a.cols[p] * a.ld_col;
    for (int c = lane; c < d; c += 64) {
        const float lc = a.l ? a.l[c] : 1.0f;
        const float vc = v[c];
        const float dc = act ? un[c] - u[c] : 0.f;
        lv_s[w][c] = lc * vc;
        dd_s[w][c] = lc * dc;
        a.xw[(int64_t)p * d + c] = dc;
        a.vw[(int64_t)p * d + c] = vc;
    }
    __builtin_amdgcn_wave_barrier();  // LDS of this wave written (one wave: program order)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int c = lane; c < d; c += 64) {
        float mv = 0.f, mtd = 0.f;
        if (act) {
            const float* gr = a.G + (int64_t)c * d;  // row c of G
#pragma unroll 4
            for (int b = 0; b < d; ++b) mv = fmaf(gr[b], lv_s[w][b], mv);
#pragma unroll 4
            for (int b = 0; b < d; ++b) mtd = fmaf(a.G[(int64_t)b * d + c], dd_s[w][b], mtd);
            const float lc = a.l ? a.l[c] : 1.0f;
            mv *= lc;
            mtd *= lc;
        }
        a.grad_rows[(int64_t)p * d + c] = act ? -mv : 0.f;
        a.grad_rows[((int64_t)a.n + p) * d + c] = act ? mv : 0.f;
        a.grad_cols[(int64_t)p * d + c] = mtd;
    }
}

// dM partials: one wave per (32x32 tile of dM, chunk of kPairChunk pairs) on the exact-fp32
// MFMA: part[ch][a][b] = Σ_{p in chunk} xw[p][a]·vw[p][b], pairs in order.
__global__ __launch_bounds__(256) void decoder_grad_dm_kernel(const float* xw, const float* vw, int n, int d,
                                                              float* part) {
    const int lane = threadIdx.x & 63;
    const int i = lane & 31, h = lane >> 5;
    const int tiles = d / 32;
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nch = (n + kPairChunk - 1) / kPairChunk;
    if (wid >= tiles * tiles * nch) return;
    const int ch = wid / (tiles * tiles);
    const int t = wid - ch * tiles * tiles;
    const int ta = t / tiles, tb = t - ta * tiles;
    const int p0 = ch * kPairChunk;
    f32x16 acc = {};
    // every row load of the chunk issued before the MFMA chain: unconditional loads (a pair past
    // n reads pair n - 1, then contributes zeros) — conditional ones were each waited for in turn
    constexpr int kSteps = kPairChunk / 2;
    float av[kSteps], bv[kSteps];
#pragma unroll
    for (int s2 = 0; s2 < kSteps; ++s2) {
        const int p = p0 + 2 * s2 + h;
        const int pc = p < n ? p : n - 1;
        av[s2] = xw[(int64_t)pc * d + ta * 32 + i];
        bv[s2] = vw[(int64_t)pc * d + tb * 32 + i];
    }
#pragma unroll
    for (int s2 = 0; s2 < kSteps; ++s2) {
        const bool ok = p0 + 2 * s2 + h < n;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ok ? av[s2] : 0.f, ok ? bv[s2] : 0.f, acc, 0, 0, 0);
    }
    float* out = part + (int64_t)ch * d * d;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = ta * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(int64_t)row * d + tb * 32 + i] = acc[r];
    }
}

// dM = Σ_chunks part (chunk order); dG = L·dM·L (written if dG != NULL).
__global__ __launch_bounds__(256) void decoder_grad_reduce_kernel(const float* part, int nch, int d,
                                                                  const float* l, float* dM, float* dG) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= d * d) return;
    float s = 0.f;
#pragma unroll 16
    for (int c = 0; c < nch; ++c) s += part[(int64_t)c * d * d + e];  // (loads ahead of the adds)
    dM[e] = s;
    if (dG) {
        const int ra = e / d, cb = e - ra * d;
        dG[e] = l ? l[ra] * s * l[cb] : s;
    }
}

// dl[a] = Σ_b dM[a][b]·G[a][b]·l[b] + Σ_c dM[c][a]·G[c][a]·l[c]   (M = L·G·L, L = diag(l));
// diag[a] = dG[a][a] (the DistMult relation vector's gradient: G = diag(r), L = I).
__global__ __launch_bounds__(256) void decoder_grad_vec_kernel(const float* dM, const float* G, const float* l,
                                                               int d, float* dl, float* dgdiag) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a >= d) return;
    if (dl) {
        float s = 0.f;  // (unrolled: the loads run ahead of the dependent fma chain)
#pragma unroll 16
        for (int b = 0; b < d; ++b) s = fmaf(dM[(int64_t)a * d + b] * G[(int64_t)a * d + b], l[b], s);
#pragma unroll 16
        for (int c = 0; c < d; ++c) s = fmaf(dM[(int64_t)c * d + a] * G[(int64_t)c * d + a], l[c], s);
        dl[a] = s;
    }
    if (dgdiag) {
        const float la = l ? l[a] : 1.0f;
        dgdiag[a] = la * dM[(int64_t)a * d + a] * la;
    }
}

// ---------------------------------------------------------------- scatter of row gradients
// out[idx[q]] += Σ_{q': idx[q'] == idx[q]} src[q'] — the gradient of the embedding gathers
// (optimizer.py:75-76).  One wave per q; the wave of a row's first occurrence sums every
// occurrence in order and owns the read-modify-write, so rows are updated once, race-free.
__global__ __launch_bounds__(256) void scatter_rows_kernel(const int32_t* idx, int n, const float* src, int d,
                                                           float* out, int64_t ld_out, int n_out) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= n) return;
    const int r = idx[q];
    if (r < 0 || r >= n_out) return;  // outside the table: no row to update (wave-uniform)
    // idx scanned 16 chunks of 64 at a time, their loads all in flight (one chunk per round
    // trip before: n / 64 dependent round trips for every wave); chunks in order, so a wave
    // returns on an earlier occurrence before it adds anything, and adds its occurrences in
    // index order as before
    constexpr int kScanU = 16;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};  // columns lane + 64t, d <= 256
    for (int q0 = 0; q0 < n; q0 += 64 * kScanU) {
        int v[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const int j = q0 + 64 * u + lane;
            v[u] = idx[j < n ? j : n - 1];  // unconditional (clamped) loads
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const int c0 = q0 + 64 * u;
            if (c0 >= n) break;  // wave-uniform
            const int j = c0 + lane;
            const bool hit = j < n && v[u] == r;
            if (__any(hit && j < q)) return;  // an earlier occurrence owns the row
            uint64_t m = __ballot(hit && j >= q);
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                const float* s = src + (int64_t)(c0 + b) * d;
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (lane + 64 * t < d) acc[t] += s[lane + 64 * t];
            }
        }
    }
    float* o = out + (int64_t)r * ld_out;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        if (lane + 64 * t < d) o[lane + 64 * t] += acc[t];
}

// ---------------------------------------------------------------- l2_normalize backward
struct L2gArgs {
    const float* s[DG_MAX_GROUPS];
    float* ds[DG_MAX_GROUPS];
    const float* dy;
    const float* mask;
    int32_t n_groups;
    int32_t n_rows;
    int32_t d;
    int32_t pad;
};

// One wave per row; LP lanes hold the row (a float4 each).  dy' = dy ∘ [mask > 0] (relu's
// gradient, model.py:75) when mask != NULL; per group g:
//   ds = dy'·inv − s·inv³·(s·dy')·[Σs² >= 1e-12],  inv = rsqrt(max(Σs², 1e-12)).
template <int LP>
__global__ __launch_bounds__(256) void l2norm_grad_kernel(const L2gArgs a) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= a.n_rows) return;
    const int q = lane % LP;
    const bool ok = lane < LP && q * 4 < a.d;
    const int64_t off = (int64_t)r * a.d + q * 4;
    float4 dy = ok ? *reinterpret_cast<const float4*>(a.dy + off) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.mask && ok) {
        const float4 m = *reinterpret_cast<const float4*>(a.mask + off);
        dy.x = m.x > 0.f ? dy.x : 0.f;
        dy.y = m.y > 0.f ? dy.y : 0.f;
        dy.z = m.z > 0.f ? dy.z : 0.f;
        dy.w = m.w > 0.f ? dy.w : 0.f;
    }
    // every group's S row loaded before the first group's sums (one round trip, not one a group)
    float4 sv[DG_MAX_GROUPS];
#pragma unroll
    for (int g = 0; g < DG_MAX_GROUPS; ++g)
        sv[g] = ok && g < a.n_groups ? *reinterpret_cast<const float4*>(a.s[g] + off) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int g = 0; g < DG_MAX_GROUPS; ++g) {
        if (g >= a.n_groups) break;  // wave-uniform
        const float4 s = sv[g];
        float ss = s.x * s.x + s.y * s.y + s.z * s.z + s.w * s.w;
        float dot = s.x * dy.x + s.y * dy.y + s.z * dy.z + s.w * dy.w;
#pragma unroll
        for (int m = 1; m < LP; m <<= 1) {
            ss += __shfl_xor(ss, m);
            dot += __shfl_xor(dot, m);
        }
        const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
        const float coef = ss >= 1e-12f ? dot * inv * inv * inv : 0.f;
        if (ok)
            *reinterpret_cast<float4*>(a.ds[g] + off) =
                make_float4(dy.x * inv - s.x * coef, dy.y * inv - s.y * coef, dy.z * inv - s.z * coef,
                            dy.w * inv - s.w * coef);
    }
}

// ---------------------------------------------------------------- Adam
struct AdamSegK {
    float* p;
    const float* g;
    float* m;
    float* v;
    int64_t n;
    int32_t block_begin;
    int32_t pad;
};

struct AdamArgs {
    AdamSegK s[DG_MAX_ADAM_SEGS];
    const float* state;  // device {β1^t, β2^t, alpha} or NULL (then `alpha`)
    int32_t n_segs;
    float alpha;
    float beta1;
    float beta2;
    float eps;
    int32_t pad;
};

constexpr int kAdamF4PerBlock = 256 * 4;  // float4s per block (4 per thread)

// TF 1.8 ApplyAdam (use_nesterov = false), element-wise in fp32:
//   m += (g − m)(1 − β1);  v += (g² − v)(1 − β2);  p −= alpha·m / (sqrt(v) + ε)
// alpha = lr·sqrt(1 − β2^t)/(1 − β1^t) is computed by the caller as TF does (fp32).
__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float alpha, const AdamArgs& a) {
    m += (g - m) * (1.0f - a.beta1);
    v += (g * g - v) * (1.0f - a.beta2);
    p -= (m * alpha) / (sqrtf(v) + a.eps);
}

__global__ __launch_bounds__(256) void adam_kernel(const AdamArgs a) {
    const int b = blockIdx.x;
    int si = 0;
#pragma unroll 1
    while (si + 1 < a.n_segs && b >= a.s[si + 1].block_begin) ++si;
    const AdamSegK& s = a.s[si];
    const float alpha = a.state ? a.state[2] : a.alpha;
    const int64_t f0 = (int64_t)(b - s.block_begin) * kAdamF4PerBlock;
    const int64_t nf4 = s.n >> 2;
    // every load of the block's four float4 rounds first (clamped indices, no branch: 16
    // loads in flight per lane), then the updates and the predicated stores
    if (nf4 > 0) {
        float4 p[4], m[4], v[4], g[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t f = min(f0 + u * 256 + threadIdx.x, nf4 - 1);
            p[u] = reinterpret_cast<const float4*>(s.p)[f];
            m[u] = reinterpret_cast<const float4*>(s.m)[f];
            v[u] = reinterpret_cast<const float4*>(s.v)[f];
            g[u] = s.g ? reinterpret_cast<const float4*>(s.g)[f] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t f = f0 + u * 256 + threadIdx.x;
            adam1(p[u].x, g[u].x, m[u].x, v[u].x, alpha, a);
            adam1(p[u].y, g[u].y, m[u].y, v[u].y, alpha, a);
            adam1(p[u].z, g[u].z, m[u].z, v[u].z, alpha, a);
            adam1(p[u].w, g[u].w, m[u].w, v[u].w, alpha, a);
            if (f < nf4) {
                reinterpret_cast<float4*>(s.p)[f] = p[u];
                reinterpret_cast<float4*>(s.m)[f] = m[u];
                reinterpret_cast<float4*>(s.v)[f] = v[u];
            }
        }
    }
    // the tail (n % 4 elements) by the segment's last block
    const int64_t tail0 = nf4 << 2;
    if (tail0 < s.n && f0 <= nf4 && nf4 < f0 + kAdamF4PerBlock && threadIdx.x < s.n - tail0) {
        const int64_t e = tail0 + threadIdx.x;
        adam1(s.p[e], s.g ? s.g[e] : 0.f, s.m[e], s.v[e], alpha, a);
    }
}

// TF's _finish: β1^t, β2^t ← ·β1, ·β2 (float32 variables), then the next step's
// alpha = lr·sqrt(1 − β2^t)/(1 − β1^t).
__global__ void adam_advance_kernel(float* state, float lr, float beta1, float beta2) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const float b1p = state[0] * beta1, b2p = state[1] * beta2;
        state[0] = b1p;
        state[1] = b2p;
        state[2] = lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
    }
}

}  // namespace

extern "C" int64_t dg_decoder_grad_workspace(int32_t n, int32_t d) {
    if (n < 1 || d < 32) return 0;
    const int64_t nch = dg::ceil_div(n, kPairChunk);
    return 4 * (2 * (int64_t)n * d + nch * d * d + (int64_t)d * d);
}

extern "C" int dg_decoder_grad_f32(const float* row_table, int64_t ld_row, const float* col_table,
                                   int64_t ld_col, const int32_t* rows, const int32_t* cols,
                                   const int32_t* neg_rows, int32_t n, const float* pos, const float* neg,
                                   const float* G, const float* l, int32_t d, float margin,
                                   float* grad_rows, float* grad_cols, float* dG, float* dl,
                                   float* dG_diag, void* workspace, int64_t workspace_bytes, void* stream) {
    if (n < 0 || d < 32 || d > 256 || (d & 31)) return DG_EINVAL;
    if (n == 0) return DG_OK;
    if (!row_table || !col_table || !rows || !cols || !neg_rows || !pos || !neg || !G || !grad_rows ||
        !grad_cols || !workspace)
        return DG_EINVAL;
    if (ld_row < d || ld_col < d) return DG_EINVAL;
    if (dl && !l) return DG_EINVAL;
    if (workspace_bytes < dg_decoder_grad_workspace(n, d) || !dg::aligned16(workspace)) return DG_EINVAL;
    float* xw = static_cast<float*>(workspace);
    float* vw = xw + (int64_t)n * d;
    float* part = vw + (int64_t)n * d;
    const int nch = dg::ceil_div(n, kPairChunk);
    float* dM = part + (int64_t)nch * d * d;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    PairArgs pa{row_table, col_table, rows, cols, neg_rows, pos, neg, G, l, grad_rows, grad_cols, xw, vw,
                ld_row, ld_col, n, d, margin, 0};
    hipLaunchKernelGGL(decoder_grad_pairs_kernel, dim3(dg::ceil_div(n, 4)), dim3(256), 0, st, pa);
    if (!dG && !dl && !dG_diag) return dg::launch_status();
    const int tiles = d / 32;
    hipLaunchKernelGGL(decoder_grad_dm_kernel, dim3(dg::ceil_div((int64_t)tiles * tiles * nch, 4)), dim3(256), 0,
                       st, xw, vw, n, d, part);
    hipLaunchKernelGGL(decoder_grad_reduce_kernel, dim3(dg::ceil_div((int64_t)d * d, 256)), dim3(256), 0, st,
                       part, nch, d, l, dM, dG);
    if (dl || dG_diag)
        hipLaunchKernelGGL(decoder_grad_vec_kernel, dim3(1), dim3(256), 0, st, dM, G, l, d, dl, dG_diag);
    return dg::launch_status();
}

extern "C" int dg_scatter_rows_f32(const int32_t* idx, int32_t n, const float* src, int32_t d, float* out,
                                   int64_t ld_out, int32_t n_out_rows, void* stream) {
    if (n < 0 || d < 1 || d > 256 || ld_out < d || n_out_rows < 0) return DG_EINVAL;
    if (n == 0) return DG_OK;
    if (!idx || !src || !out) return DG_EINVAL;
    hipLaunchKernelGGL(scatter_rows_kernel, dim3(dg::ceil_div(n, 4)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), idx, n, src, d, out, ld_out, n_out_rows);
    return dg::launch_status();
}

extern "C" int dg_l2norm_grad_f32(const dg_l2g_group* groups, int32_t n_groups, const float* dy,
                                  const float* mask, int32_t n_rows, int32_t d, void* stream) {
    if (n_groups < 1 || !groups) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
    if (d < 4 || d > 256 || (d & 3) || n_rows < 0) return DG_EINVAL;
    if (n_rows == 0) return DG_OK;
    if (!dy || !dg::aligned16(dy) || (mask && !dg::aligned16(mask))) return dy ? DG_EALIGN : DG_EINVAL;
    L2gArgs a{};
    for (int i = 0; i < n_groups; ++i) {
        if (!groups[i].s || !groups[i].ds) return DG_EINVAL;
        if (!dg::aligned16(groups[i].s) || !dg::aligned16(groups[i].ds)) return DG_EALIGN;
        a.s[i] = groups[i].s;
        a.ds[i] = groups[i].ds;
    }
    a.dy = dy;
    a.mask = mask;
    a.n_groups = n_groups;
    a.n_rows = n_rows;
    a.d = d;
    const int lp = dg::lanes_per_row(d);
    dim3 grid(dg::ceil_div(n_rows, 4)), block(256);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define DG_LAUNCH_L2G(L) hipLaunchKernelGGL(l2norm_grad_kernel<L>, grid, block, 0, st, a)
    switch (lp) {
        case 1: DG_LAUNCH_L2G(1); break;
        case 2: DG_LAUNCH_L2G(2); break;
        case 4: DG_LAUNCH_L2G(4); break;
        case 8: DG_LAUNCH_L2G(8); break;
        case 16: DG_LAUNCH_L2G(16); break;
        case 32: DG_LAUNCH_L2G(32); break;
        case 64: DG_LAUNCH_L2G(64); break;
        default: return DG_EINVAL;
    }
#undef DG_LAUNCH_L2G
    return dg::launch_status();
}

extern "C" int dg_adam_f32(const dg_adam_seg* segs, int32_t n_segs, float alpha, float beta1, float beta2,
                           float eps, const float* state, void* stream) {
    if (n_segs < 0 || (n_segs > 0 && !segs)) return DG_EINVAL;
    if (n_segs > DG_MAX_ADAM_SEGS) return DG_ETOOMANY;
    AdamArgs a{};
    a.state = state;
    a.alpha = alpha;
    a.beta1 = beta1;
    a.beta2 = beta2;
    a.eps = eps;
    int64_t blocks = 0;
    for (int i = 0; i < n_segs; ++i) {
        const dg_adam_seg& s = segs[i];
        if (s.n < 0) return DG_EINVAL;
        if (s.n == 0) continue;
        if (!s.param || !s.m || !s.v) return DG_EINVAL;
        if (!dg::aligned16(s.param) || !dg::aligned16(s.m) || !dg::aligned16(s.v) || (s.grad && !dg::aligned16(s.grad)))
            return DG_EALIGN;
        AdamSegK& k = a.s[a.n_segs++];
        k.p = s.param;
        k.g = s.grad;
        k.m = s.m;
        k.v = s.v;
        k.n = s.n;
        k.block_begin = static_cast<int32_t>(blocks);
        blocks += dg::ceil_div(dg::ceil_div(s.n, 4), kAdamF4PerBlock);
        if (blocks > 0x7fffffff) return DG_EINVAL;
    }
    if (blocks == 0) return DG_OK;
    hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), a);
    return dg::launch_status();
}

extern "C" int dg_adam_advance(float* state, float lr, float beta1, float beta2, void* stream) {
    if (!state) return DG_EINVAL;
    hipLaunchKernelGGL(adam_advance_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), state, lr,
                       beta1, beta2);
    return dg::launch_status();
}
