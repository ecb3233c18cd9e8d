// Dropout masks for gfx950 (MI355X): the training path's dropout_sparse / tf.nn.dropout.
//
// Replaces (paths relative to the reference root):
//   dropout_sparse(inputs, 1 - dropout, nonzero_feat)   decagon/deep/layers.py:23-31, :88
//   tf.nn.dropout(inputs, 1 - dropout)                  decagon/deep/layers.py:112
//
// TF draws its masks from its own stateful RNG, which cannot be reproduced; the distribution is
// what is restated: every element kept independently with probability keep and scaled by
// 1/keep, a fresh draw per relation k and per run.  Here a mask bit is a counter-based hash of
// (seed, step, stream tag, element index) — dg_keep() below — so the forward, the backward and
// the test oracle (oracle/decagon_oracle.dropout_keep) regenerate identical masks, and the step
// counter lives on the device (advanced by dg_dropout_advance), which keeps a training step
// capturable into one hipGraph.
//
// Identity features make layer 1's dropout a row mask on the relation-stacked operand W1
// (X_j·W1_k with X_j = diag(m_k)/keep is W1_k with rows scaled): dg_dropout_rows_f32 writes the
// masked copy the SpMM reads, and scales the rows of dW1 in the backward.  Layer 2's dropout is
// an element mask on H1_j per relation: dg_dropout_elems_f32 writes H_k = M_k∘H1_j/keep for the
// projection GEMM; the backward's Σ_k M_k∘(dP_k·W2_kᵀ) applies the same bits inside
// dg_gemm_f32 (batch-reduce mode with a dropout descriptor).
#include "common.h"
#include "dropout.h"

namespace {

__global__ __launch_bounds__(256) void dropout_rows_kernel(const float* in, float* out, int64_t n_rows, int d,
                                                           const uint64_t* state, uint32_t tag, float keep) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const uint32_t key = dg::drop_key(state, tag);
    const float s = dg::keep_scale(key, static_cast<uint32_t>(r), keep);
    const float* src = in + r * d;
    float* dst = out + r * d;
    for (int c = lane; c < d; c += 64) dst[c] = src[c] * s;
}

// out[k][r][f] = src[r][f] · s(k·n_rows·d + r·d + f) for k < K (element index in 32 bits)
__global__ __launch_bounds__(256) void dropout_elems_kernel(const float* src, float* out, int K, int n_rows, int d,
                                                            const uint64_t* state, uint32_t tag, float keep) {
    const int64_t total = (int64_t)K * n_rows * d;
    const uint32_t key = dg::drop_key(state, tag);
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t rf = e % ((int64_t)n_rows * d);
        out[e] = src[rf] * dg::keep_scale(key, static_cast<uint32_t>(e), keep);
    }
}

// Relation-mapped forms (a rank's relation shard, sharding.py): local slab b is global relation
// rel_map[b] and carries THAT relation's mask bits — the same bits the unmapped kernels draw for
// it — so every rank, and the one-GPU run, mask a relation identically.
// Rows: slab b = rows_per_slab rows; in / out addressed at slab rel_map[b] (flags bit 1 / 2) or b.
__global__ __launch_bounds__(256) void dropout_rows_map_kernel(const float* in, float* out, const int32_t* rel_map,
                                                               int64_t n_rows, int64_t rows_per_slab, int d,
                                                               int flags, const uint64_t* state, uint32_t tag,
                                                               float keep) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // local row: slab b, row j
    if (r >= n_rows) return;
    const int64_t b = r / rows_per_slab, j = r - b * rows_per_slab;
    const int64_t gr = (int64_t)rel_map[b] * rows_per_slab + j;     // global row: the mask bit
    const uint32_t key = dg::drop_key(state, tag);
    const float s = dg::keep_scale(key, static_cast<uint32_t>(gr), keep);
    const float* src = in + ((flags & 1) ? gr : r) * d;
    float* dst = out + ((flags & 2) ? gr : r) * d;
    for (int c = lane; c < d; c += 64) dst[c] = src[c] * s;
}

// out[b][r][f] = src[r][f] · s(rel_map[b]·n_rows·d + r·d + f)
__global__ __launch_bounds__(256) void dropout_elems_map_kernel(const float* src, float* out, const int32_t* rel_map,
                                                                int K, int n_rows, int d, const uint64_t* state,
                                                                uint32_t tag, float keep) {
    const int64_t plane = (int64_t)n_rows * d, total = (int64_t)K * plane;
    const uint32_t key = dg::drop_key(state, tag);
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t b = e / plane, rf = e - b * plane;
        out[e] = src[rf] * dg::keep_scale(key, static_cast<uint32_t>(rel_map[b] * plane + rf), keep);
    }
}

__global__ void dropout_advance_kernel(uint64_t* state) {
    if (threadIdx.x == 0 && blockIdx.x == 0) state[1] += 1;
}

}  // namespace

extern "C" int dg_dropout_rows_f32(const float* in, float* out, int64_t n_rows, int32_t d, const uint64_t* state,
                                   uint32_t tag, float keep, void* stream) {
    if (n_rows < 0 || d < 1 || !(keep > 0.f && keep <= 1.f)) return DG_EINVAL;
    if (n_rows == 0) return DG_OK;
    if (!in || !out || !state) return DG_EINVAL;
    if (n_rows * d >= 0xFFFFFFFFLL) return DG_EINVAL;
    hipLaunchKernelGGL(dropout_rows_kernel, dim3(static_cast<unsigned>((n_rows + 3) / 4)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), in, out, n_rows, d, state, tag, keep);
    return dg::launch_status();
}

extern "C" int dg_dropout_elems_f32(const float* src, float* out, int32_t K, int32_t n_rows, int32_t d,
                                    const uint64_t* state, uint32_t tag, float keep, void* stream) {
    if (K < 0 || n_rows < 0 || d < 1 || !(keep > 0.f && keep <= 1.f)) return DG_EINVAL;
    const int64_t total = (int64_t)K * n_rows * d;
    if (total == 0) return DG_OK;
    if (!src || !out || !state) return DG_EINVAL;
    if (total >= 0xFFFFFFFFLL) return DG_EINVAL;  // element indices are 32-bit
    const int64_t blocks = (total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096;
    hipLaunchKernelGGL(dropout_elems_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), src, out, K, n_rows, d, state, tag, keep);
    return dg::launch_status();
}

extern "C" int dg_dropout_rows_map_f32(const float* in, float* out, const int32_t* rel_map, int32_t n_map,
                                       int64_t rows_per_slab, int32_t d, int32_t flags, const uint64_t* state,
                                       uint32_t tag, float keep, void* stream) {
    if (n_map < 0 || rows_per_slab < 0 || d < 1 || (flags & ~3) || !(keep > 0.f && keep <= 1.f)) return DG_EINVAL;
    const int64_t n_rows = (int64_t)n_map * rows_per_slab;
    if (n_rows == 0) return DG_OK;
    if (!in || !out || !state || !rel_map) return DG_EINVAL;
    hipLaunchKernelGGL(dropout_rows_map_kernel, dim3(static_cast<unsigned>((n_rows + 3) / 4)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), in, out, rel_map, n_rows, rows_per_slab, d, flags,
                       state, tag, keep);
    return dg::launch_status();
}

extern "C" int dg_dropout_elems_map_f32(const float* src, float* out, const int32_t* rel_map, int32_t K,
                                        int32_t n_rows, int32_t d, const uint64_t* state, uint32_t tag, float keep,
                                        void* stream) {
    if (K < 0 || n_rows < 0 || d < 1 || !(keep > 0.f && keep <= 1.f)) return DG_EINVAL;
    const int64_t total = (int64_t)K * n_rows * d;
    if (total == 0) return DG_OK;
    if (!src || !out || !state || !rel_map) return DG_EINVAL;
    const int64_t blocks = (total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096;
    hipLaunchKernelGGL(dropout_elems_map_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), src, out, rel_map, K, n_rows, d, state, tag, keep);
    return dg::launch_status();
}

extern "C" int dg_dropout_advance(uint64_t* state, void* stream) {
    if (!state) return DG_EINVAL;
    hipLaunchKernelGGL(dropout_advance_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), state);
    return dg::launch_status();
}
