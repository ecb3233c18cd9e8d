// Edge decoders, losses and the unigram negative sampler for gfx950 (MI355X).
//
// Replaces (paths relative to the reference root):
//   DecagonOptimizer.batch_predict + tf.diag_part     decagon/deep/optimizer.py:51-57, :63-85
//   DecagonOptimizer._hinge_loss / _xent_loss          decagon/deep/optimizer.py:116-127
//   tf.nn.fixed_unigram_candidate_sampler(0.75)        decagon/deep/optimizer.py:40-47
//
// Decoder: the reference forms the full B×B matrix U·L·G·L·Vᵀ and keeps its diagonal.  Here
// one wave scores 32 pairs: T = (U∘l)·G runs on the exact-fp32 MFMA (32 pairs × 32 output
// features per v_mfma_f32_32x32x2_f32 tile, d/32 tiles), then each lane multiplies its
// accumulator column by l[j]·V[p][j] and the 32 lanes of a half-wave fold the row sums with
// a shuffle butterfly.  Nothing of size B×B is formed.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct DecArgs {
    const float* row_table;
    const float* col_table;
    const int32_t* row_idx;
    const int32_t* col_idx;
    const float* G;
    const float* l;
    float* out;
    int64_t ld_row;
    int64_t ld_col;
    int32_t n_pairs;
    int32_t d;
};

__global__ __launch_bounds__(256) void decoder_score_kernel(const DecArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int p0 = (blockIdx.x * 4 + wave) * 32;
    if (p0 >= a.n_pairs) return;
    const int i = lane & 31;
    const int h = lane >> 5;
    const int d = a.d;
    const int p = p0 + i;
    const bool pvalid = p < a.n_pairs;
    const float* u = a.row_table + (int64_t)(pvalid ? a.row_idx[p] : 0) * a.ld_row;
    const int cidx_mine = pvalid ? a.col_idx[p] : 0;

    float part[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) part[r] = 0.f;

#pragma unroll 1
    for (int n0 = 0; n0 < d; n0 += 32) {
        f32x16 acc = {};
#pragma unroll 4
        for (int k0 = 0; k0 < d; k0 += 2) {
            const int kk = k0 + h;
            float av = 0.f;
            if (pvalid) {
                av = u[kk];
                if (a.l) av *= a.l[kk];
            }
            const float bv = a.G[(int64_t)kk * d + n0 + i];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
        const int j = n0 + i;
        const float lj = a.l ? a.l[j] : 1.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int prow = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int cidx = __shfl(cidx_mine, prow);  // lane prow holds pair p0+prow
            if (p0 + prow < a.n_pairs) {
                const float v = a.col_table[(int64_t)cidx * a.ld_col + j];
                part[r] = fmaf(acc[r] * lj, v, part[r]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
        for (int m = 1; m < 32; m <<= 1) part[r] += __shfl_xor(part[r], m);
    }
    if (i == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int pp = p0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (pp < a.n_pairs) a.out[pp] = part[r];
        }
    }
}

// Fixed-order block reduction (deterministic): thread t sums t, t+256, ... then a tree.
template <typename F>
__device__ float block_sum_256(int n, F term) {
    __shared__ float red[256];
    float s = 0.f;
    for (int idx = threadIdx.x; idx < n; idx += 256) s += term(idx);
    __syncthreads();  // a previous call's readers of red[0] are done
    red[threadIdx.x] = s;
    __syncthreads();
#pragma unroll
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    return red[0];
}

__global__ __launch_bounds__(256) void hinge_kernel(const float* pos, const float* neg, int n,
                                                    float margin, float* loss) {
    const float s = block_sum_256(n, [&](int p) { return fmaxf(neg[p] - (pos[p] - margin), 0.f); });
    if (threadIdx.x == 0) loss[0] = s;
}

__device__ __forceinline__ float softplus_neg_abs(float x) { return log1pf(expf(-fabsf(x))); }

__global__ __launch_bounds__(256) void xent_kernel(const float* pos, const float* neg, int n,
                                                   float w, float* loss) {
    // sigmoid_cross_entropy_with_logits(z, x) = max(x,0) - x*z + log(1 + exp(-|x|))
    const float sp = block_sum_256(n, [&](int p) {
        const float x = pos[p];
        return fmaxf(x, 0.f) - x + softplus_neg_abs(x);
    });
    const float sn = block_sum_256(n, [&](int p) {
        const float x = neg[p];
        return fmaxf(x, 0.f) + softplus_neg_abs(x);
    });
    if (threadIdx.x == 0) loss[0] = sp + w * sn;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void unigram_sample_kernel(const float* cdf, int range, int n,
                                                             uint64_t seed, uint64_t offset,
                                                             int32_t* out) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= n) return;
    const uint64_t h = splitmix64(seed ^ splitmix64(offset + (uint64_t)idx));
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);  // [0,1), 24 bits
    const float target = u * cdf[range - 1];
    // first c with cdf[c] > target
    int lo = 0, hi = range - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] > target)
            hi = mid;
        else
            lo = mid + 1;
    }
    out[idx] = lo;
}

}  // namespace

extern "C" int dg_decoder_score_f32(const float* row_table, int64_t ld_row, const float* col_table,
                                    int64_t ld_col, const int32_t* row_idx, const int32_t* col_idx,
                                    int32_t n_pairs, const float* G, const float* l, int32_t d,
                                    float* out, void* stream) {
    if (n_pairs < 0 || d <= 0 || (d % 32) || d > 256) return DG_EINVAL;
    if (n_pairs == 0) return DG_OK;
    if (!row_table || !col_table || !row_idx || !col_idx || !G || !out) return DG_EINVAL;
    if (ld_row < d || ld_col < d) return DG_EINVAL;
    DecArgs a{row_table, col_table, row_idx, col_idx, G, l, out, ld_row, ld_col, n_pairs, d};
    dim3 grid(dg::ceil_div(n_pairs, 128)), block(256);
    hipLaunchKernelGGL(decoder_score_kernel, grid, block, 0, reinterpret_cast<hipStream_t>(stream), a);
    return dg::launch_status();
}

extern "C" int dg_hinge_loss_f32(const float* pos, const float* neg, int32_t n, float margin,
                                 float* loss, void* stream) {
    if (n < 0 || !loss || (n > 0 && (!pos || !neg))) return DG_EINVAL;
    hipLaunchKernelGGL(hinge_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       pos, neg, n, margin, loss);
    return dg::launch_status();
}

extern "C" int dg_xent_loss_f32(const float* pos, const float* neg, int32_t n, float neg_weight,
                                float* loss, void* stream) {
    if (n < 0 || !loss || (n > 0 && (!pos || !neg))) return DG_EINVAL;
    hipLaunchKernelGGL(xent_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       pos, neg, n, neg_weight, loss);
    return dg::launch_status();
}

extern "C" int dg_unigram_sample(const float* cdf, int32_t range, int32_t n, uint64_t seed,
                                 uint64_t offset, int32_t* out, void* stream) {
    if (range < 1 || n < 0 || !cdf || (n > 0 && !out)) return DG_EINVAL;
    if (n == 0) return DG_OK;
    hipLaunchKernelGGL(unigram_sample_kernel, dim3(dg::ceil_div(n, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), cdf, range, n, seed, offset, out);
    return dg::launch_status();
}
