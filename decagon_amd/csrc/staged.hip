// LDS-staged relation SpMM for gfx950 (MI355X): groups with many relations over a narrow
// column space (polypharmacy drug×drug: 1,928 relations of 645×645).
//
// Reference ops replaced: tf.sparse_tensor_dense_matmul(adj_mats[edge_type][k], x) and
// tf.add_n (decagon/deep/layers.py:90-92, :114-116) for such groups.
//
// Why: gathering 16-byte pieces of random 256-byte X rows through L1/L2/Infinity Cache runs at
// ~11 TB/s of gathered bytes on MI355X whatever the L2 hit rate (measured: profiles/),
// and every nonzero gathers a full row.  Here a workgroup streams one relation's dense operand
// slab X_k[:, slice] into LDS with coalesced 16-byte loads (each HBM byte of X read once), then
// every row's nonzeros gather from LDS — ds_read_b128 at ~256 B/clk/CU — and accumulate in
// registers across the relations of an output chunk.
//
// Workgroup = 1024 threads, one per (output chunk c, column slice s):
//   for k in chunk c:   issue at once: the CSR of every row this thread owns (LPW*NPF
//                       nonzeros per row in registers), the slab X_slab(k)[:, s*W .. s*W+W)
//                       and relation k+1's row pointers; barrier; slab -> LDS (rows padded
//                       by 16 B); barrier; rows r = pass*RP + wave*(64/LPW) + lane/LPW, LPW
//                       lanes per row, (vcol, val) handed out with ds_bpermute, 16-byte LDS
//                       gathers, fmaf into acc[pass]
//   write out[c][r][s*W .. s*W+W)
// Fixed summation order, no atomics.
#include "common.h"

namespace {

struct StagedGroupK {
    const int32_t* rowptr;
    const int32_t* vcol;
    const float* val;
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
    int32_t pad;
};

struct StagedArgs {
    StagedGroupK g[DG_MAX_GROUPS];
    int32_t n_groups;
    int32_t d;
};

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;

// LPW lanes per row (slice = 4*LPW floats); MAXP passes of RP rows; NPF nonzeros per lane
// prefetched per row and relation (rows longer than LPW*NPF finish in a tail loop); SR
// 16-byte staging loads per thread.
template <int LPW, int MAXP, int NPF, int SR>
__global__ __launch_bounds__(kThreads) void spmm_staged_kernel(const StagedArgs a) {
    extern __shared__ float4 xs[];  // [n_cols][LPW + 1] float4 (one float4 of padding per row)
    constexpr int RPW = 64 / LPW;          // rows per wave per pass
    constexpr int RP = kWaves * RPW;       // rows per pass
    constexpr int LDR = LPW + 1;           // LDS row stride in float4
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int q = lane % LPW;
    const int gbase = lane - q;            // first lane of this lane group
    const int b = blockIdx.x;
    int gi = 0;
#pragma unroll 1
    while (gi + 1 < a.n_groups && b >= a.g[gi + 1].block_begin) ++gi;
    const StagedGroupK& g = a.g[gi];
    // XCD-contiguous item map (see spmm.hip): the slices of one chunk run on one XCD, so the
    // chunk's CSR is fetched from HBM once and re-read from that XCD's L2.
    const int lb = b - g.block_begin;
    const int per = g.n_blocks >> 3;
    const int item = (lb & 7) * per + (lb >> 3);
    if (item >= g.n_out_chunks * g.n_slices) return;  // block-uniform, before any barrier
    const int c = item / g.n_slices;
    const int s = item - c * g.n_slices;
    const int d = a.d;
    const int col0 = s * (4 * LPW);
    const bool qact = col0 + q * 4 < d;
    const int n_rows = g.n_rows;
    const int n_cols = g.n_cols;
    const int row0 = wave * RPW + lane / LPW;  // this lane group's row in pass 0
    const int k0 = c * g.out_chunk;
    const int k1 = min(k0 + g.out_chunk, g.n_rels);

    float4 acc[MAXP];
#pragma unroll
    for (int p = 0; p < MAXP; ++p) acc[p] = make_float4(0.f, 0.f, 0.f, 0.f);

    // row extents of relation k for every pass (prefetched one relation ahead)
    int beg[MAXP], len[MAXP];
    auto load_rows = [&](int k, int (&bg)[MAXP], int (&ln)[MAXP]) {
        const int32_t* __restrict__ rp = g.rowptr + (int64_t)k * n_rows;
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
            const int r = p * RP + row0;
            bg[p] = 0;
            ln[p] = 0;
            if (k < k1 && r < n_rows) {
                bg[p] = rp[r];
                ln[p] = rp[r + 1] - bg[p];
            }
        }
    };
    load_rows(k0, beg, len);

#pragma unroll 1
    for (int k = k0; k < k1; ++k) {
        const int slab = g.slab ? g.slab[k] : k;
        const int vbase = slab * n_cols;
        // ---- 1. issue every load of relation k: its CSR for this thread's rows ----
        int vc[MAXP][NPF];
        float vv[MAXP][NPF];
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
#pragma unroll
            for (int i = 0; i < NPF; ++i) {
                const int o = q + LPW * i;
                vc[p][i] = 0;
                vv[p][i] = 0.f;
                if (o < len[p]) {
                    vc[p][i] = g.vcol[beg[p] + o];
                    vv[p][i] = g.val[beg[p] + o];
                }
            }
        }
        // ---- ... its dense slab X_slab[:, col0 .. col0+4*LPW) ----
        const float* __restrict__ xk = g.x + (int64_t)vbase * g.x_ld + col0;
        float4 st[SR];
#pragma unroll
        for (int j = 0; j < SR; ++j) {
            const int idx = tid + j * kThreads;
            const int v = idx / LPW;
            const int qq = idx - v * LPW;
            st[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (v < n_cols && col0 + qq * 4 < d)
                st[j] = *reinterpret_cast<const float4*>(xk + (int64_t)v * g.x_ld + qq * 4);
        }
        // ---- ... and the next relation's row extents ----
        int nbeg[MAXP], nlen[MAXP];
        load_rows(k + 1, nbeg, nlen);
        __syncthreads();  // the previous relation's gathers are done with the slab buffer
#pragma unroll
        for (int j = 0; j < SR; ++j) {
            const int idx = tid + j * kThreads;
            const int v = idx / LPW;
            if (v < n_cols) xs[v * LDR + (idx - v * LPW)] = st[j];
        }
        __syncthreads();
        // ---- 2. gather from LDS: lane group walks its row, LPW nonzeros per round ----
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
            if (p * RP >= n_rows) break;  // uniform
#pragma unroll
            for (int i = 0; i < NPF; ++i) {
#pragma unroll
                for (int t = 0; t < LPW; ++t) {
                    const int vct = __shfl(vc[p][i], gbase + t) - vbase;
                    const float vvt = __shfl(vv[p][i], gbase + t);
                    if (LPW * i + t < len[p]) dg::fma4(acc[p], vvt, xs[vct * LDR + q]);
                }
            }
            // rows longer than the prefetch: finish from global memory (rare)
            int maxlen = len[p];
#pragma unroll
            for (int m = LPW; m < 64; m <<= 1) maxlen = max(maxlen, __shfl_xor(maxlen, m));
#pragma unroll 1
            for (int o = LPW * NPF; o < maxlen; o += LPW) {
                int vcl = 0;
                float vvl = 0.f;
                if (o + q < len[p]) {
                    vcl = g.vcol[beg[p] + o + q] - vbase;
                    vvl = g.val[beg[p] + o + q];
                }
#pragma unroll
                for (int t = 0; t < LPW; ++t) {
                    const int vct = __shfl(vcl, gbase + t);
                    const float vvt = __shfl(vvl, gbase + t);
                    if (o + t < len[p]) dg::fma4(acc[p], vvt, xs[vct * LDR + q]);
                }
            }
        }
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
            beg[p] = nbeg[p];
            len[p] = nlen[p];
        }
    }
    // ---- write the chunk partial ----
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
        const int r = p * RP + row0;
        if (p * RP >= n_rows) break;
        if (r < n_rows && qact)
            *reinterpret_cast<float4*>(g.out + ((int64_t)c * n_rows + r) * d + col0 + q * 4) = acc[p];
    }
}

template <int LPW, int MAXP, int NPF, int SR>
int launch_staged(const StagedArgs& a, int64_t blocks, int lds_bytes, hipStream_t st) {
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&spmm_staged_kernel<LPW, MAXP, NPF, SR>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        configured = true;
    }
    hipLaunchKernelGGL((spmm_staged_kernel<LPW, MAXP, NPF, SR>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kThreads), lds_bytes, st, a);
    return dg::launch_status();
}

}  // namespace

extern "C" int dg_spmm_staged_f32(const dg_staged_group* groups, int32_t n_groups, int32_t d,
                                  int32_t slice, void* stream) {
    if (n_groups < 1 || !groups) return DG_EINVAL;
    if (n_groups > DG_MAX_GROUPS) return DG_ETOOMANY;
    if (d < 4 || d > 256 || (d & 3)) return DG_EINVAL;
    if (slice != 16 && slice != 32) return DG_EINVAL;
    const int lpw = slice / 4;
    const int rows_per_pass = kWaves * (64 / lpw);
    StagedArgs a{};
    a.d = d;
    int64_t blocks = 0;
    int max_cols = 0, max_rows = 0;
    for (int i = 0; i < n_groups; ++i) {
        const dg_staged_group& s = groups[i];
        if (s.n_rows < 0 || s.n_cols < 0 || s.n_rels < 0 || s.out_chunk < 1) return DG_EINVAL;
        if (s.n_rows == 0 || s.n_rels == 0) continue;
        if (!s.rowptr || !s.x || !s.out) return DG_EINVAL;
        if (!dg::aligned16(s.x) || !dg::aligned16(s.out) || (s.x_ld & 3) || s.x_ld < d) return DG_EALIGN;
        if ((int64_t)s.x_rows * s.x_ld > 0x7fffffffLL) return DG_EINVAL;
        StagedGroupK& k = a.g[a.n_groups++];
        k.rowptr = s.rowptr;
        k.vcol = s.vcol;
        k.val = s.val;
        k.slab = s.slab;
        k.x = s.x;
        k.out = s.out;
        k.x_ld = static_cast<int32_t>(s.x_ld);
        k.n_rows = s.n_rows;
        k.n_cols = s.n_cols;
        k.n_rels = s.n_rels;
        k.out_chunk = s.out_chunk;
        k.n_out_chunks = dg::ceil_div(s.n_rels, s.out_chunk);
        k.n_slices = dg::ceil_div(d, slice);
        const int64_t items = (int64_t)k.n_out_chunks * k.n_slices;
        k.n_blocks = static_cast<int32_t>(8 * ((items + 7) / 8));
        k.block_begin = static_cast<int32_t>(blocks);
        blocks += k.n_blocks;
        max_cols = s.n_cols > max_cols ? s.n_cols : max_cols;
        max_rows = s.n_rows > max_rows ? s.n_rows : max_rows;
    }
    if (blocks == 0) return DG_OK;
    if (blocks > 0x7fffffff) return DG_EINVAL;
    const int64_t lds = (int64_t)max_cols * (lpw + 1) * 16;
    if (lds > 160 * 1024) return DG_EINVAL;           // the slab must fit in LDS
    const int passes = dg::ceil_div(max_rows, rows_per_pass);
    const int sr = dg::ceil_div((int64_t)max_cols * lpw, kThreads);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int L = static_cast<int>(lds);
    // register budget: passes x prefetch and staging loads per thread are compile-time
    // (every variant below stays within 128 VGPRs without scratch)
    if (lpw == 4 && sr <= 4) {
        if (passes <= 4) return launch_staged<4, 4, 4, 4>(a, blocks, L, st);
        if (passes <= 8) return launch_staged<4, 8, 1, 4>(a, blocks, L, st);
    } else if (lpw == 8 && sr <= 8 && passes <= 4) {
        return launch_staged<8, 4, 2, 8>(a, blocks, L, st);
    }
    return DG_EINVAL;  // too many rows or columns for one workgroup
}
