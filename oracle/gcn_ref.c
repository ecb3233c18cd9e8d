/*
 * ORACLE — test infrastructure only.  Scalar C restatement (fp32, one thread) of the
 * reference's per-op GCN forward, used as the timed CPU baseline ("port") in bench.py and
 * as a second checker in tests/.  Never linked into the product.
 *
 * It follows TF 1.8's CPU op sequence of one GCN layer (paths relative to the reference):
 *   Y_k = sparse_tensor_dense_matmul(A_k, X_k)   decagon/deep/layers.py:90, :114
 *         (zeroed output, nonzeros visited in order: out[row] += val * X[col])
 *   S   = add_n(Y_1..Y_K)                        decagon/deep/layers.py:92, :116
 *   S   = S * rsqrt(max(sum(S^2), 1e-12))        decagon/deep/layers.py:93, :117
 *   H   = relu(add_n over edge types)            decagon/deep/model.py:75
 *   X_k = H_j · W_k (layer 2 projection)         decagon/deep/layers.py:113
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

void oracle_spmm_f32(const int32_t* rowptr, const int32_t* col, const float* val, int32_t n_rows,
                     const float* x, int64_t ldx, int32_t d, float* y) {
    memset(y, 0, sizeof(float) * (size_t)n_rows * (size_t)d);
    for (int32_t r = 0; r < n_rows; ++r) {
        float* yr = y + (int64_t)r * d;
        for (int32_t p = rowptr[r]; p < rowptr[r + 1]; ++p) {
            const float v = val[p];
            const float* xr = x + (int64_t)col[p] * ldx;
            for (int32_t c = 0; c < d; ++c) yr[c] += v * xr[c];
        }
    }
}

void oracle_add_f32(float* acc, const float* y, int64_t n) {
    for (int64_t i = 0; i < n; ++i) acc[i] += y[i];
}

void oracle_l2norm_rows_f32(float* x, int32_t n_rows, int32_t d) {
    for (int32_t r = 0; r < n_rows; ++r) {
        float* xr = x + (int64_t)r * d;
        float ss = 0.f;
        for (int32_t c = 0; c < d; ++c) ss += xr[c] * xr[c];
        const float inv = 1.0f / sqrtf(ss > 1e-12f ? ss : 1e-12f);
        for (int32_t c = 0; c < d; ++c) xr[c] *= inv;
    }
}

void oracle_relu_f32(float* x, int64_t n) {
    for (int64_t i = 0; i < n; ++i) x[i] = x[i] > 0.f ? x[i] : 0.f;
}

/* C[m][n] = A[m][k] · B[k][n], row-major, k-ordered sums. */
void oracle_gemm_f32(const float* a, const float* b, float* c, int32_t m, int32_t k, int32_t n) {
    for (int32_t i = 0; i < m; ++i) {
        float* ci = c + (int64_t)i * n;
        for (int32_t j = 0; j < n; ++j) ci[j] = 0.f;
        for (int32_t t = 0; t < k; ++t) {
            const float av = a[(int64_t)i * k + t];
            const float* bt = b + (int64_t)t * n;
            for (int32_t j = 0; j < n; ++j) ci[j] += av * bt[j];
        }
    }
}
