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
// Layout (decagon_amd/sparse.py: staged_layout): per relation, rows are split into virtual
// rows of at most L nonzeros (L the smallest leaving ≤ 1024 of them), sorted by length, and
// the nonzeros stored diagonal-major: the m-th nonzero of every virtual row that has one, in
// sorted order.  Thread i owns sorted virtual row i, so at diagonal m the 64 threads of a
// wave read 64 consecutive (col, value) pairs — one coalesced 512-byte load straight from
// global memory, prefetched four diagonals ahead in registers — and no thread walks a long
// row while the others wait.  Each row's nonzeros are ordered on the host (layout.cpp) so the
// 16 lanes of a ds_read_b128 group mostly gather from distinct bank slots.
//
// Workgroup = 1024 threads, one per (output chunk c, 16-float column slice s):
//   for relation k of the chunk:
//     barrier; the slab slice X_slab(k)[:, 16s .. +16) and k's tables (vinfo, doff), both
//     prefetched into registers during relation k-1, → LDS (columns 80 B apart: the bank slot
//     of float4 j of column v is (5v+j) mod 16); barrier; prefetch relation k+1's
//     thread i: part = Σ_{m < len[i]} val · xs[col]   (pairs from global, 4 × ds_read_b128 per nonzero)
//     acc[row[i]] += part, in rounds by segment index (a row's segments in order)
//   out[c][r][16s .. +16) = acc[r]
// Fixed summation order, no atomics: bitwise reproducible.
#include "common.h"

namespace {

constexpr int kMaxThreads = 1024;
constexpr int kLdsBytes = 160 * 1024;
constexpr int kMetaInts = 256;  // a chunk's tables: jm offsets (nk + 1) and slabs (nk), nk <= 64
constexpr int kJmRegs = 3;      // jm words per thread: 4 + 1024 + (n_cols + 1) + pad <= 3 * 1024

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
    int32_t pad;
};

struct StagedArgs {
    StagedGroupK g[DG_MAX_GROUPS];
    int32_t n_groups;
    int32_t d;
    int32_t xs_f4;     // float4 slots of the slab slice (+ the zero column)
    int32_t acc_f4;    // float4 slots of the accumulator
    int32_t jm_ints;   // ints of the jm buffer
#ifdef DG_STAGED_PROF
    unsigned long long* prof;  // per block: [relation start, gather, accumulate, relations] cycles
#endif
};

// float4 j = q & 3 of column v = q >> 2 of the slab slice (zero past the slice; a partial last
// slice loads any valid float4); it lives at xs[5v + j] — columns 80 B apart, so the 16-byte
// bank slot of float4 j of column v is (5v + j) mod 16, a bijection of v & 15 for every j
__device__ __forceinline__ float4 slab_slot(const float* xk, int q, int n_cols, int x_ld, int col0, int d) {
    if (q >= n_cols * 4) return make_float4(0.f, 0.f, 0.f, 0.f);
    const int v = q >> 2;
    const int cj = min(col0 + 4 * (q & 3), d - 4) - col0;
    return *reinterpret_cast<const float4*>(xk + (int64_t)v * x_ld + cj);
}

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
    const int k0 = c * g.out_chunk;
    const int nk = min(g.out_chunk, g.n_rels - k0);  // relations of this chunk

    // LDS: xs (columns 0..n_cols-1, then the zero column n_cols) | meta | acc | jm
    float4* xs = lds;  // at offset 0: gather addresses need no base
    int* jof = reinterpret_cast<int*>(xs + a.xs_f4);
    int* slb = jof + (nk + 1);
    float4* acc = reinterpret_cast<float4*>(jof + kMetaInts);
    int* jm = reinterpret_cast<int*>(acc + a.acc_f4);

    for (int i = tid; i <= nk; i += T) jof[i] = g.jmoff[k0 + i];
    for (int i = tid; i < nk; i += T) slb[i] = g.slab ? g.slab[k0 + i] : k0 + i;
    for (int i = tid; i < n_rows * 4; i += T) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < 4) xs[n_cols * 5 + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();

    // relation i's slab slice and tables into registers (T >= n_cols: 4 slots per thread)
    float4 xr0, xr1, xr2, xr3;
    int jr[kJmRegs];
    auto prefetch = [&](int i) {
        const float* xk = g.x + (int64_t)slb[i] * n_cols * g.x_ld + col0;
        xr0 = slab_slot(xk, tid, n_cols, g.x_ld, col0, d);
        xr1 = slab_slot(xk, tid + T, n_cols, g.x_ld, col0, d);
        xr2 = slab_slot(xk, tid + 2 * T, n_cols, g.x_ld, col0, d);
        xr3 = slab_slot(xk, tid + 3 * T, n_cols, g.x_ld, col0, d);
        const int j0 = jof[i], jn = jof[i + 1] - j0;
#pragma unroll
        for (int u = 0; u < kJmRegs; ++u) jr[u] = tid + u * T < jn ? g.jm[j0 + tid + u * T] : 0;
    };
    prefetch(0);

#ifdef DG_STAGED_PROF
    unsigned long long c_start = 0, c_gather = 0, c_acc = 0, c0 = __builtin_readcyclecounter(), c1;
#define DG_TICK(acc_) (c1 = __builtin_readcyclecounter(), acc_ += c1 - c0, c0 = c1)
#else
#define DG_TICK(acc_) ((void)0)
#endif
    const int2 zero_pair = make_int2(n_cols, 0);  // the zero column, value 0: adds +0
#pragma unroll 1
    for (int i = 0; i < nk; ++i) {
        __syncthreads();  // relation i-1's gathers and accumulation are done with xs / jm
        {
            const int n4 = n_cols * 4;
            auto put = [&](int q, float4 v) {
                if (q < n4) xs[(q >> 2) * 5 + (q & 3)] = v;
            };
            put(tid, xr0);
            put(tid + T, xr1);
            put(tid + 2 * T, xr2);
            put(tid + 3 * T, xr3);
            const int jn = jof[i + 1] - jof[i];
#pragma unroll
            for (int u = 0; u < kJmRegs; ++u)
                if (tid + u * T < jn) jm[tid + u * T] = jr[u];
        }
        __syncthreads();
        const int n_virt = jm[0], rounds = jm[1];
        const int vi = tid < n_virt ? jm[4 + tid] : 0;  // row | seg << 10 | len << 16
        const int rl = vi >> 16;
        const int* doff = jm + 4 + n_virt;
        // the wave's longest virtual row is its first (sorted descending)
        const int rlw = __builtin_amdgcn_readfirstlane(rl);
        const int2* pr = g.pairs + tid;
        auto pairs4 = [&](int m, int2 (&u)[4]) {
#pragma unroll
            for (int q = 0; q < 4; ++q) u[q] = m + q < rl ? pr[doff[m + q]] : zero_pair;
        };
        int2 un[4];
        pairs4(0, un);  // issued before the next relation's prefetch: waiting for it does not
        if (i + 1 < nk) prefetch(i + 1);  // wait for those
        DG_TICK(c_start);
        float4 part[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) part[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
        for (int m = 0; m < rlw; m += 4) {
            int2 u[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) u[q] = un[q];
            if (m + 4 < rlw) pairs4(m + 4, un);
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
        // a row's segments meet in the accumulator in segment order, one round each
        float4* ar = acc + (vi & 1023) * 4;
#pragma unroll 1
        for (int rd = 0; rd < rounds; ++rd) {
            if (rl > 0 && ((vi >> 10) & 63) == rd) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float4 o = ar[j];
                    o.x += part[j].x;
                    o.y += part[j].y;
                    o.z += part[j].z;
                    o.w += part[j].w;
                    ar[j] = o;
                }
            }
            if (rd + 1 < rounds) __syncthreads();
        }
        DG_TICK(c_acc);
    }
#ifdef DG_STAGED_PROF
    if (tid == 0) {
        a.prof[4 * b + 0] = c_start;
        a.prof[4 * b + 1] = c_gather;
        a.prof[4 * b + 2] = c_acc;
        a.prof[4 * b + 3] = nk;
    }
#endif
#undef DG_TICK
    __syncthreads();
    for (int q = tid; q < n_rows * 4; q += T) {
        const int r = q >> 2, j = q & 3;
        if (col0 + 4 * j < d)
            *reinterpret_cast<float4*>(g.out + ((int64_t)c * n_rows + r) * d + col0 + 4 * j) = acc[q];
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
    (void)hipMemcpy(host, dg_staged_prof_last, n * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    return n;
}
#endif

extern "C" int dg_spmm_staged_f32(const dg_staged_group* groups, int32_t n_groups, int32_t d,
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
        if (s.n_rows < 0 || s.n_cols < 0 || s.n_rels < 0 || s.out_chunk < 1 || s.out_chunk > 64) return DG_EINVAL;
        if (s.n_rows >= kMaxThreads || s.n_cols > kMaxThreads) return DG_EINVAL;  // rows fit 10 bits
        if (s.n_rows == 0 || s.n_rels == 0) continue;
        if (!s.pairs || !s.jm || !s.jmoff || !s.x || !s.out) return DG_EINVAL;
        if (!dg::aligned16(s.x) || !dg::aligned16(s.out) || !dg::aligned16(s.pairs) || (s.x_ld & 3) || s.x_ld < d)
            return DG_EALIGN;
        if ((int64_t)s.x_rows * s.x_ld > 0x7fffffffLL) return DG_EINVAL;
        StagedGroupK& k = a.g[a.n_groups++];
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
        k.n_slices = dg::ceil_div(d, 16);
        const int64_t items = (int64_t)k.n_out_chunks * k.n_slices;
        k.n_blocks = static_cast<int32_t>(8 * ((items + 7) / 8));
        k.block_begin = static_cast<int32_t>(blocks);
        blocks += k.n_blocks;
        max_cols = s.n_cols > max_cols ? s.n_cols : max_cols;
        max_rows = s.n_rows > max_rows ? s.n_rows : max_rows;
    }
    if (blocks == 0) return DG_OK;
    if (blocks > 0x7fffffff) return DG_EINVAL;
    const int threads = kMaxThreads;  // one thread per virtual row (staged_layout: at most 1024)
    a.xs_f4 = (max_cols + 1) * 5;     // + the zero column
    a.acc_f4 = max_rows * 4;
    a.jm_ints = kJmRegs * kMaxThreads;
    const int64_t lds = (int64_t)a.xs_f4 * 16 + kMetaInts * 4 + (int64_t)a.acc_f4 * 16 + (int64_t)a.jm_ints * 4;
    if (lds > kLdsBytes) return DG_EINVAL;
#ifdef DG_STAGED_PROF
    {
        static unsigned long long* buf = nullptr;
        static int64_t have_blocks = 0;
        if (have_blocks < blocks) {
            if (buf) (void)hipFree(buf);
            (void)hipMalloc(&buf, blocks * 4 * sizeof(unsigned long long));
            have_blocks = blocks;
        }
        (void)hipMemset(buf, 0, blocks * 4 * sizeof(unsigned long long));
        a.prof = buf;
        dg_staged_prof_last = buf;
        dg_staged_prof_blocks = blocks;
    }
#endif
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&spmm_staged_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
        configured = true;
    }
    hipLaunchKernelGGL(spmm_staged_kernel, dim3(static_cast<unsigned>(blocks)), dim3(threads),
                       static_cast<int>(lds), st, a);
    return dg::launch_status();
}
