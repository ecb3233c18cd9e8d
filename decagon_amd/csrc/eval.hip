// Link-prediction accuracy metrics on the device (the evaluation path):
// AUROC, AUPRC and AP@k of positive vs negative edge scores.
//
// Replaces (paths relative to the reference root):
//   metrics.roc_auc_score / metrics.average_precision_score (sklearn) and
//   rank_metrics.apk(actual, predicted, k=50)         main.py:38-80 (get_accuracy_scores),
//                                                     decagon/utility/rank_metrics.py:4-40,
//                                                     main/AccuracyEvaluators/Tensorflow/
//                                                     DecagonAccuracyEvaluator.py:58-120
// Every metric is a sum over the positives of counts against all scores, so no sort is needed:
// for positive i with score s (list order: positives, then negatives, as get_accuracy_scores
// builds `predicted`),
//   AUROC term  #neg < s + ½·#neg == s                      (Mann–Whitney = roc_auc_score)
//   AP term     #pos >= s / #all >= s                        (= average_precision_score)
//   rank        #all > s + #pos before i with == s           (Python's stable sort, reverse=True)
//   AP@k term   (hits before i + 1)/(rank + 1) if rank < k,  hits = #pos > s + #pos before i ==
// One workgroup per positive counts in integers (exact); the terms are summed in double, in
// positive order, by one workgroup: deterministic.
#include "common.h"

namespace {



__device__ __forceinline__ int block_sum_int(int v, int* red) {
    for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    int s = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += red[k];
    return s;
}

// The score each edge is ranked by (mode, dg_rank_metrics_ex_f32), from its logit x:
//   DG_RANK_LOGIT      x itself (float)
//   DG_RANK_SIGMOID64  main.py:51-52,60,70,81 under numpy 1.14 (requirements.txt:14): rec is
//                      TF's float32, so np.exp(-x) runs in float32 (glibc expf: correctly
//                      rounded — computed here as (float)exp((double)-x)), `1 + e` and `1. / …`
//                      promote to float64, then np.nan_to_num.  Saturates: x > ≈36.7 → 1.0,
//                      x < ≈-88.7 → 0.0 (float32 exp overflows), so large logits tie.
//   DG_RANK_SIGMOID32  MathUtils.sigmoid on the float32 decoder output array
//                      (DecagonAccuracyEvaluator.py:123): every step float32 (x > ≈16.6 → 1.0)
__global__ __launch_bounds__(256) void score_key_kernel(const float* x, int n, int mode, double* key) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    double k = v;
    if (mode != DG_RANK_LOGIT) {
        const float e = (float)exp(-(double)v);
        if (mode == DG_RANK_SIGMOID64) {
            k = 1.0 / (1.0 + (double)e);
        } else {
            const float one = 1.0f;
            k = (double)(one / (one + e));
        }
        if (k != k) k = 0.0;  // np.nan_to_num (only a NaN logit gets here)
    }
    key[i] = k;
}

// counts[i] = {lt_neg, eq_neg, ge_pos, ge_all, gt_all, gt_pos, eq_pos_before}
template <typename T>
__global__ __launch_bounds__(256) void rank_counts_kernel(const T* pos, int P, const T* neg, int N,
                                                          int* counts) {
    __shared__ int red[4];
    const int i = blockIdx.x;
    const T s = pos[i];
    int lt_neg = 0, eq_neg = 0, ge_pos = 0, gt_pos = 0, eq_before = 0, gt_neg = 0;
    for (int j = threadIdx.x; j < P; j += blockDim.x) {
        const T v = pos[j];
        ge_pos += v >= s;
        gt_pos += v > s;
        eq_before += (v == s) && (j < i);
    }
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
        const T v = neg[j];
        lt_neg += v < s;
        eq_neg += v == s;
        gt_neg += v > s;
    }
    int c[6] = {lt_neg, eq_neg, ge_pos, gt_pos, eq_before, gt_neg};
#pragma unroll
    for (int q = 0; q < 6; ++q) c[q] = block_sum_int(c[q], red);
    if (threadIdx.x == 0) {
        int* o = counts + (int64_t)i * 8;
        o[0] = c[0];                   // #neg < s
        o[1] = c[1];                   // #neg == s
        o[2] = c[2];                   // #pos >= s
        o[3] = c[2] + c[1] + c[5];     // #all >= s
        o[4] = c[3] + c[5];            // #all > s
        o[5] = c[3];                   // #pos > s
        o[6] = c[4];                   // #pos before i with == s
    }
}

__global__ __launch_bounds__(256) void rank_reduce_kernel(const int* counts, int P, int N, int k, double* out) {
    __shared__ double red[3][256];
    double au = 0.0, ap = 0.0, apk = 0.0;
    for (int i = threadIdx.x; i < P; i += 256) {
        const int* c = counts + (int64_t)i * 8;
        au += (double)c[0] + 0.5 * (double)c[1];
        ap += (double)c[2] / (double)c[3];
        const int rank = c[4] + c[6];
        if (rank < k) apk += ((double)(c[5] + c[6]) + 1.0) / ((double)rank + 1.0);
    }
    red[0][threadIdx.x] = au;
    red[1][threadIdx.x] = ap;
    red[2][threadIdx.x] = apk;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int q = 0; q < 3; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = N > 0 && P > 0 ? red[0][0] / ((double)P * (double)N) : __builtin_nan("");
        out[1] = P > 0 ? red[1][0] / (double)P : __builtin_nan("");
        out[2] = P > 0 ? red[2][0] / (double)(P < k ? P : k) : 0.0;
    }
}

}  // namespace

extern "C" int64_t dg_rank_metrics_workspace(int32_t n_pos) { return n_pos > 0 ? 32LL * n_pos : 0; }

extern "C" int64_t dg_rank_metrics_ex_workspace(int32_t n_pos, int32_t n_neg) {
    return 32LL * n_pos + 8LL * ((int64_t)n_pos + n_neg) + 16;
}

extern "C" int dg_rank_metrics_f32(const float* pos, int32_t n_pos, const float* neg, int32_t n_neg, int32_t k,
                                   double* out, void* workspace, int64_t workspace_bytes, void* stream) {
    if (n_pos < 0 || n_neg < 0 || k < 1 || !out) return DG_EINVAL;
    if (n_pos > 0 && (!pos || !workspace || workspace_bytes < dg_rank_metrics_workspace(n_pos))) return DG_EINVAL;
    if (n_neg > 0 && !neg) return DG_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int* counts = static_cast<int*>(workspace);
    if (n_pos > 0)
        hipLaunchKernelGGL(rank_counts_kernel<float>, dim3(n_pos), dim3(256), 0, st, pos, n_pos, neg, n_neg,
                           counts);
    hipLaunchKernelGGL(rank_reduce_kernel, dim3(1), dim3(256), 0, st, counts, n_pos, n_neg, k, out);
    return dg::launch_status();
}

extern "C" int dg_rank_metrics_ex_f32(const float* pos, int32_t n_pos, const float* neg, int32_t n_neg,
                                      int32_t k, int32_t mode, double* out, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
    if (n_pos < 0 || n_neg < 0 || k < 1 || !out || !workspace) return DG_EINVAL;
    if (mode != DG_RANK_LOGIT && mode != DG_RANK_SIGMOID64 && mode != DG_RANK_SIGMOID32) return DG_EINVAL;
    if (workspace_bytes < dg_rank_metrics_ex_workspace(n_pos, n_neg)) return DG_EINVAL;
    if ((n_pos > 0 && !pos) || (n_neg > 0 && !neg)) return DG_EINVAL;
    if (!dg::aligned16(workspace)) return DG_EALIGN;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    double* kp = static_cast<double*>(workspace);
    double* kn = kp + n_pos;
    int* counts = reinterpret_cast<int*>(kp + n_pos + n_neg + 1);
    if (n_pos > 0)
        hipLaunchKernelGGL(score_key_kernel, dim3(dg::ceil_div(n_pos, 256)), dim3(256), 0, st, pos, n_pos, mode, kp);
    if (n_neg > 0)
        hipLaunchKernelGGL(score_key_kernel, dim3(dg::ceil_div(n_neg, 256)), dim3(256), 0, st, neg, n_neg, mode, kn);
    if (n_pos > 0)
        hipLaunchKernelGGL(rank_counts_kernel<double>, dim3(n_pos), dim3(256), 0, st, kp, n_pos, kn, n_neg,
                           counts);
    hipLaunchKernelGGL(rank_reduce_kernel, dim3(1), dim3(256), 0, st, counts, n_pos, n_neg, k, out);
    return dg::launch_status();
}
