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
//   for k in chunk c:   stage X_slab(k)[:, s*W .. s*W+W) → LDS (rows padded by 16 B)
//                       rows r = pass*RP + wave*(64/LPW) + lane/LPW, LPW lanes per row:
//                       8 nonzeros (vcol, val) loaded per lane-group round, handed out with
//                       ds_bpermute, 16-byte LDS gathers, fmaf into acc[pass]
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

template <int LPW, int MAXP>
__global__ __launch_bounds__(kThreads) void spmm_staged_kernel(const StagedArgs a) {
    extern __shared__ float4 xs[];  // [n_cols][LPW + 1] float4 (one float4 of padding per row)
    constexpr int RPW = 64 / LPW;          // rows per wave per pass
    constexpr int RP = kWaves * RPW;       // rows per pass
    constexpr int LDR = LPW + 1;           // LDS row stride in float4
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int q = lane % LPW;
    const int gsub = lane / LPW;           // row slot of this lane group within the wave
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

    float4 acc[MAXP];
#pragma unroll
    for (int p = 0; p < MAXP; ++p) acc[p] = make_float4(0.f, 0.f, 0.f, 0.f);

    const int k0 = c * g.out_chunk;
    const int k1 = min(k0 + g.out_chunk, g.n_rels);
#pragma unroll 1
    for (int k = k0; k < k1; ++k) {
        const int slab = g.slab ? g.slab[k] : k;
        const int vbase = slab * n_cols;
        // ---- stage X_slab[:, col0 .. col0+4*LPW) into LDS ----
        __syncthreads();  // the previous relation's gathers are done
        const float* __restrict__ xk = g.x + (int64_t)vbase * g.x_ld + col0;
        for (int idx = tid; idx < n_cols * LPW; idx += kThreads) {
            const int v = idx / LPW;
            const int qq = idx - v * LPW;
            float4 val4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (col0 + qq * 4 < d) val4 = *reinterpret_cast<const float4*>(xk + (int64_t)v * g.x_ld + qq * 4);
            xs[v * LDR + qq] = val4;
        }
        __syncthreads();
        // ---- every row's nonzeros of relation k, gathered from LDS ----
        const int32_t* __restrict__ rp = g.rowptr + (int64_t)k * n_rows;
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
            const int r = p * RP + wave * RPW + gsub;
            if (p * RP >= n_rows) break;  // uniform
            int beg = 0, end = 0;
            if (r < n_rows) {
                beg = rp[r];
                end = rp[r + 1];
            }
            // lane groups of one wave walk their rows in lock-step, LPW nonzeros per round
            int len = end - beg;
            int maxlen = len;
#pragma unroll
            for (int m = LPW; m < 64; m <<= 1) maxlen = max(maxlen, __shfl_xor(maxlen, m));
#pragma unroll 1
            for (int o = 0; o < maxlen; o += LPW) {
                const int e = beg + o + q;
                int vc = 0;
                float vv = 0.f;
                if (o + q < len) {
                    vc = g.vcol[e] - vbase;
                    vv = g.val[e];
                }
#pragma unroll
                for (int t = 0; t < LPW; ++t) {
                    const int src = (lane - q) + t;  // lane t of this lane group
                    const int vct = __shfl(vc, src);
                    const float vvt = __shfl(vv, src);
                    if (o + t < len) {
                        const float4 xv = xs[vct * LDR + q];
                        dg::fma4(acc[p], vvt, xv);
                    }
                }
            }
        }
    }
    // ---- write the chunk partial ----
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
        const int r = p * RP + wave * RPW + gsub;
        if (p * RP >= n_rows) break;
        if (r < n_rows && qact)
            *reinterpret_cast<float4*>(g.out + ((int64_t)c * n_rows + r) * d + col0 + q * 4) = acc[p];
    }
}

template <int LPW, int MAXP>
int launch_staged(const StagedArgs& a, int64_t blocks, int lds_bytes, hipStream_t st) {
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&spmm_staged_kernel<LPW, MAXP>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        configured = true;
    }
    hipLaunchKernelGGL((spmm_staged_kernel<LPW, MAXP>), dim3(static_cast<unsigned>(blocks)),
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
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int L = static_cast<int>(lds);
    if (lpw == 8) {
        if (passes <= 4) return launch_staged<8, 4>(a, blocks, L, st);
        if (passes <= 8) return launch_staged<8, 8>(a, blocks, L, st);
    } else {
        if (passes <= 4) return launch_staged<4, 4>(a, blocks, L, st);
        if (passes <= 8) return launch_staged<4, 8>(a, blocks, L, st);
    }
    return DG_EINVAL;  // too many rows for one workgroup's registers
}
