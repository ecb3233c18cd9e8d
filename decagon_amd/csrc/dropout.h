// Counter-based dropout masks shared by the kernels that apply them (dropout.hip, gemm.hip).
// A mask element is kept iff the top 24 bits of h = lowbias32(key ^ idx) are below keep·2^24,
// key = lowbias32(lowbias32(seed_lo ^ tag·0x9E3779B9) ^ (seed_hi + step·0x85EBCA6B)) with
// (seed, step) = state[0..1] on the device; a kept element is scaled by 1/keep.  The numpy
// restatement (oracle/decagon_oracle.dropout_keep) regenerates the same bits.
#pragma once

#include <stdint.h>

namespace dg {

__host__ __device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t drop_key(const uint64_t* state, uint32_t tag) {
    const uint64_t seed = state[0], step = state[1];
    return lowbias32(lowbias32(static_cast<uint32_t>(seed) ^ (tag * 0x9E3779B9U)) ^
                     (static_cast<uint32_t>(seed >> 32) + static_cast<uint32_t>(step) * 0x85EBCA6BU));
}

__device__ __forceinline__ float keep_scale(uint32_t key, uint32_t idx, float keep) {
    const uint32_t thr = static_cast<uint32_t>(keep * 16777216.0f);
    return (lowbias32(key ^ idx) >> 8) < thr ? 1.0f / keep : 0.0f;
}

}  // namespace dg
