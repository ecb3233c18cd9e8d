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
#include "decoder_tile.h"

namespace {

using dg::DecTab;
using dg::f32x16;
using dg::score_tile;
using dg::splitmix64;
using dg::unigram_draw;

struct DecArgs {
    DecTab t;
    const int32_t* row_idx;
    const int32_t* col_idx;
    float* out;
    int32_t n_pairs;
};

__global__ __launch_bounds__(256) void decoder_score_kernel(const DecArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int p0 = (blockIdx.x * 4 + wave) * 32;
    if (p0 >= a.n_pairs) return;
    const int i = lane & 31;
    const int h = lane >> 5;
    const int p = p0 + i;
    const bool valid = p < a.n_pairs;
    float part[16];
    score_tile(a.t, valid ? a.row_idx[p] : 0, valid ? a.col_idx[p] : 0, valid, part);
    if ((i & 1) == 0) {  // lane 2r holds score r of its half
        const int r = i >> 1;
        const int pp = p0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (pp < a.n_pairs) a.out[pp] = part[0];
    }
}

// Fused decoder step (optimizer.py:37-57 + :116-120): for the batch pairs b < n,
//   neg_row[b] = given[b] or draw (offset + b) of the alias sampler,
//   pos[b] = score(rows[b], cols[b]),  neg[b] = score(neg_row[b], cols[b]),
//   loss   = sum_b relu(neg[b] - (pos[b] - margin))
// One workgroup of two waves per 32 pairs (wave 0 the positive tile, wave 1 the negative
// tile).  Each workgroup folds its 32 hinge terms into a partial, and the partials meet in one
// launch without float atomics:
//  - PACKED (at most 255 workgroups): one returning 64-bit atomic add per workgroup on a word
//    that holds the arrival count (bits 56-63), the count of partials outside the fixed-point
//    range (48-55) and the sum of the others as fixed point, 2^-32 units (0-47: a partial below
//    256 is < 2^40, 255 of them < 2^48), each partial rounded to the nearest 2^-32 — so the
//    reported loss is within 255·2^-33 ≈ 3e-8 (absolute) of the exact sum of the fp32 partials,
//    and unbiased.  Integer sums do not depend on the order, so the result is bitwise
//    reproducible; the workgroup that sees count = grid − 1 has the whole sum in
//    hand (no partial store, drain or read-back).  A partial ≥ 256 (or NaN / inf) is stored
//    write-through, drained and counted in bits 48-55 instead; the last workgroup then adds those
//    in block order (they are rare: the others' stores are never read).
//  - otherwise: each workgroup publishes its partial (a write-through sc1 store, drained) and
//    takes a ticket; the last one reads every partial with sc1 loads (cdna_hip_programming.md
//    Guideline 16; no L2 write-back or invalidate) and adds them in block order.
// The last workgroup resets what it used for the next launch.
#ifdef DG_DEC_PROF
extern "C" int64_t dg_dec_prof_copy(unsigned long long* host) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(dg::g_dec_prof), sizeof(dg::g_dec_prof), 0, hipMemcpyDeviceToHost) !=
        hipSuccess)
        return -1;
    return 256;
}
#endif

struct HingeArgs {
    DecTab t;
    const int32_t* rows;
    const int32_t* cols;
    const int32_t* neg_given;
    const uint2* alias;
    float* pos;
    float* neg;
    int32_t* neg_rows_out;
    float* loss;        // [1]
    float* partial;     // [gridDim.x]
    uint32_t* ticket;   // zero before the first launch; the last block resets it
    unsigned long long* word;  // PACKED: count | out-of-range count | fixed-point sum (zero between launches)
    uint64_t seed;
    uint64_t offset;
    int32_t range;
    int32_t n;
    float margin;
};

template <bool PACKED>
__global__ __launch_bounds__(128) void decoder_hinge_kernel(const HingeArgs a) {
    __shared__ float sc[2][32];
    __shared__ float red[128];
    __shared__ int last;
    __shared__ unsigned long long total;
    const int lane = threadIdx.x & 63;
    const int side = threadIdx.x >> 6;  // 0: positives, 1: negatives
    const int i = lane & 31;
    const int h = lane >> 5;
    const int b0 = blockIdx.x * 32;
    const int b = b0 + i;
    const bool valid = b < a.n;
    DG_DEC_STAMP(0);  // (profiling build: wave start)
    int ridx = 0, cidx = 0;
    if (valid) {
        cidx = a.cols[b];
        if (side == 0)
            ridx = a.rows[b];
        else if (a.neg_given)
            ridx = a.neg_given[b];
        else
            ridx = unigram_draw(a.alias, a.range, a.seed, a.offset + (uint64_t)b);
        if (side == 1 && a.neg_rows_out && h == 0) a.neg_rows_out[b] = ridx;
    }
    DG_DEC_STAMP(1);  // indices (and the negatives' draws) landed
    float part[16];
    score_tile(a.t, ridx, cidx, valid, part);
    if ((i & 1) == 0) {  // lane 2r holds score r of its half
        const int r = i >> 1;
        const int q = (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = (b0 + q < a.n) ? part[0] : 0.f;
        sc[side][q] = v;
        if (b0 + q < a.n) (side == 0 ? a.pos : a.neg)[b0 + q] = v;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        float term = 0.f;
        if (lane < 32 && b0 + lane < a.n) term = fmaxf(sc[1][lane] - (sc[0][lane] - a.margin), 0.f);
        term = dg::xor_add<1>(dg::xor_add<2>(dg::xor_add<4>(dg::xor_add<8>(dg::xor_add<16>(dg::xor_add<32>(term))))));
        if (lane == 0 && PACKED) {
            unsigned long long add = 1ull << 56;
            if (term < 256.0f) {  // (false for NaN and inf too)
                add += static_cast<unsigned long long>(static_cast<double>(term) * 4294967296.0 + 0.5);  // nearest
            } else {
                __hip_atomic_store(a.partial + blockIdx.x, term, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                add += 1ull << 48;
            }
            const unsigned long long old =
                __hip_atomic_fetch_add(a.word, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = (old >> 56) == gridDim.x - 1 ? 1 : 0;
            total = old + add;
        } else if (lane == 0) {
            // hand-off without L2 write-back / invalidate (MI355X_MICROARCH.md "Valid forms",
            // first row): the partial is stored write-through (sc1) and drained before the
            // ticket add; the last block reads every partial with sc1 loads
            __hip_atomic_store(a.partial + blockIdx.x, term, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = (t == gridDim.x - 1) ? 1 : 0;
        }
    }
    __syncthreads();
    DG_DEC_STAMP(5);  // the block's ticket returned
    if (!last) return;  // block-uniform
    if constexpr (PACKED) {
        if (threadIdx.x == 0) {
            double s = static_cast<double>(total & ((1ull << 48) - 1)) * (1.0 / 4294967296.0);
            if ((total >> 48) & 0xFF) {  // partials outside the fixed-point range, in block order
                for (int k = 0; k < (int)gridDim.x; ++k) {
                    const float v = __hip_atomic_load(a.partial + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (v != 0.f) {
                        s += static_cast<double>(v);
                        __hip_atomic_store(a.partial + k, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
            a.loss[0] = static_cast<float>(s);
            __hip_atomic_store(a.word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        DG_DEC_STAMP(6);  // loss stored (last block)
        return;
    }
    float s = 0.f;
    for (int k = threadIdx.x; k < (int)gridDim.x; k += 128)
        s += __hip_atomic_load(a.partial + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    red[threadIdx.x] = s;
    __syncthreads();
#pragma unroll
    for (int w = 64; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    for (int k = threadIdx.x; k < (int)gridDim.x; k += 128) a.partial[k] = 0.f;  // (read above; the PACKED
    if (threadIdx.x == 0) {                                                      //  form reads zeros there)
        a.loss[0] = red[0];
        atomicExch(a.ticket, 0u);
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

// Many-block hinge (config 5: 10^6 pairs): block b sums its contiguous chunk in a fixed
// order, publishes the partial and takes a ticket; the last block adds the partials in block
// order and resets the ticket (the decoder_hinge_kernel pattern) — deterministic for a given n.
__global__ __launch_bounds__(256) void hinge_multi_kernel(const float* pos, const float* neg, int n,
                                                          float margin, float* loss, float* partial,
                                                          uint32_t* ticket) {
    __shared__ int last;
    const int chunk = (n + (int)gridDim.x - 1) / (int)gridDim.x;
    const int p0 = blockIdx.x * chunk;
    const int cnt = max(0, min(n, p0 + chunk) - p0);
    const float s = block_sum_256(cnt, [&](int q) {
        return fmaxf(neg[p0 + q] - (pos[p0 + q] - margin), 0.f);
    });
    if (threadIdx.x == 0) {  // sc1 partial, drained, then the ticket (decoder_hinge_kernel)
        __hip_atomic_store(partial + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;  // block-uniform
    const float t = block_sum_256((int)gridDim.x, [&](int b) {
        return __hip_atomic_load(partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    });
    if (threadIdx.x == 0) {
        loss[0] = t;
        atomicExch(ticket, 0u);
    }
}

// log1p in double: the float log1pf's double-float arithmetic is vectorised by the compiler into
// packed adds whose low result reads src1's high dword, the form this library keeps out of
// every kernel (tests/test_cpu_isa.py); the double result rounds to within an ulp
__device__ __forceinline__ float softplus_neg_abs(float x) { return (float)log1p((double)expf(-fabsf(x))); }

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

__global__ __launch_bounds__(256) void unigram_sample_kernel(const uint2* table, int range, int n,
                                                             uint64_t seed, uint64_t offset,
                                                             int32_t* out) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= n) return;
    out[idx] = unigram_draw(table, range, seed, offset + (uint64_t)idx);
}

// one table per relation slot: draw i is draw slot0*batch + i of slot (slot0 + i / batch)'s table
__global__ __launch_bounds__(256) void unigram_sample_slots_kernel(const uint2* table, int range, int64_t stride,
                                                                   int slot0, int batch, int n, uint64_t seed,
                                                                   int32_t* out) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= n) return;
    const int slot = slot0 + idx / batch;
    out[idx] = unigram_draw(table + (int64_t)slot * stride, range, seed,
                            (uint64_t)slot0 * (uint64_t)batch + (uint64_t)idx);
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
    DecArgs a{};
    a.t = DecTab{row_table, col_table, G, l, ld_row, ld_col, d,
                 dg::aligned16(row_table) && (ld_row & 3) == 0 && (!l || dg::aligned16(l))};
    a.row_idx = row_idx;
    a.col_idx = col_idx;
    a.out = out;
    a.n_pairs = n_pairs;
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

extern "C" int dg_hinge_loss_ws_f32(const float* pos, const float* neg, int32_t n, float margin,
                                    float* loss, void* workspace, void* stream) {
    if (n < 0 || !loss || !workspace || (n > 0 && (!pos || !neg))) return DG_EINVAL;
    if (!dg::aligned16(workspace)) return DG_EALIGN;
    const int blocks = max(1, min(DG_HINGE_WS_BLOCKS, dg::ceil_div(n, 4096)));
    hipLaunchKernelGGL(hinge_multi_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       pos, neg, n, margin, loss, reinterpret_cast<float*>(workspace) + 4,
                       reinterpret_cast<uint32_t*>(workspace));
    return dg::launch_status();
}

extern "C" int dg_xent_loss_f32(const float* pos, const float* neg, int32_t n, float neg_weight,
                                float* loss, void* stream) {
    if (n < 0 || !loss || (n > 0 && (!pos || !neg))) return DG_EINVAL;
    hipLaunchKernelGGL(xent_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       pos, neg, n, neg_weight, loss);
    return dg::launch_status();
}

extern "C" int dg_unigram_sample(const uint32_t* alias_table, int32_t range, int32_t n,
                                 uint64_t seed, uint64_t offset, int32_t* out, void* stream) {
    if (range < 1 || n < 0 || !alias_table || (n > 0 && !out)) return DG_EINVAL;
    if (n == 0) return DG_OK;
    hipLaunchKernelGGL(unigram_sample_kernel, dim3(dg::ceil_div(n, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const uint2*>(alias_table), range, n, seed, offset, out);
    return dg::launch_status();
}

extern "C" int dg_unigram_sample_slots(const uint32_t* alias_table, int32_t range, int64_t alias_stride,
                                       int32_t slot0, int32_t batch, int32_t n, uint64_t seed, int32_t* out,
                                       void* stream) {
    if (range < 1 || n < 0 || batch < 1 || slot0 < 0 || alias_stride < 0 || !alias_table || (n > 0 && !out))
        return DG_EINVAL;
    if (alias_stride > 0 && alias_stride < range) return DG_EINVAL;
    if (n == 0) return DG_OK;
    hipLaunchKernelGGL(unigram_sample_slots_kernel, dim3(dg::ceil_div(n, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint2*>(alias_table), range,
                       alias_stride, slot0, batch, n, seed, out);
    return dg::launch_status();
}

extern "C" int dg_decoder_hinge_f32(const float* row_table, int64_t ld_row, const float* col_table,
                                    int64_t ld_col, const int32_t* rows, const int32_t* cols,
                                    const int32_t* neg_rows, const uint32_t* alias_table,
                                    int32_t range, uint64_t seed, uint64_t offset, int32_t n,
                                    const float* G, const float* l, int32_t d, float margin,
                                    float* pos, float* neg, int32_t* neg_rows_out, float* loss,
                                    void* workspace, void* stream) {
    if (n < 1 || d <= 0 || (d % 32) || d > 256) return DG_EINVAL;
    if (!row_table || !col_table || !rows || !cols || !G || !pos || !neg || !loss || !workspace)
        return DG_EINVAL;
    if (!neg_rows && (!alias_table || range < 1)) return DG_EINVAL;
    if (ld_row < d || ld_col < d) return DG_EINVAL;
    if (!dg::aligned16(workspace)) return DG_EALIGN;
    const int blocks = dg::ceil_div(n, 32);
    HingeArgs a{};
    a.t = DecTab{row_table, col_table, G, l, ld_row, ld_col, d,
                 dg::aligned16(row_table) && (ld_row & 3) == 0 && (!l || dg::aligned16(l))};
    a.rows = rows;
    a.cols = cols;
    a.neg_given = neg_rows;
    a.alias = reinterpret_cast<const uint2*>(alias_table);
    a.pos = pos;
    a.neg = neg;
    a.neg_rows_out = neg_rows_out;
    a.loss = loss;
    a.ticket = reinterpret_cast<uint32_t*>(workspace);
    a.word = reinterpret_cast<unsigned long long*>(workspace) + 1;
    a.partial = reinterpret_cast<float*>(workspace) + 4;
    a.seed = seed;
    a.offset = offset;
    a.range = range;
    a.n = n;
    a.margin = margin;
    // ≤ 255 workgroups: one returning 64-bit atomic per block (PACKED); more: the sc1 ticket
    if (blocks <= 255)
        hipLaunchKernelGGL(decoder_hinge_kernel<true>, dim3(blocks), dim3(128), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
    else
        hipLaunchKernelGGL(decoder_hinge_kernel<false>, dim3(blocks), dim3(128), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
    return dg::launch_status();
}
