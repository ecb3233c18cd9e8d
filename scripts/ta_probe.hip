// Load-path probe (config 5): does the lane arrangement of a 16-B-per-lane row gather change
// its cost when the bytes and cache lines touched are identical?
//   A ("pair-minor", the 16x16x32 MFMA operand layout): lane l reads row r[l & 15] at byte
//     16 (l >> 4) + 64 q — consecutive lanes (a quad) read four different rows
//   B ("pair-major"): lane l reads row r[l >> 2] at byte 16 (l & 3) + 64 q — a quad reads 64
//     contiguous bytes of one row
//   C: as B with the quad's four chunks in rotated order (2, 3, 0, 1)
//   E: as B with a quad's 4 lanes XOR-permuted by the row (chunk (l & 3) ^ (row & 3))
//   S: the staged kernel's slab copy: 5 lanes per row (chunks 0-3 and a pad lane re-reading
//     chunk 3), so 3 of every 5 quads straddle two rows
// Both read 16 rows x 64 B per instruction from a 645-row x 512-B bf16 table (L2-resident),
// 12 waves per CU on every CU, rows drawn by a hash per (wave, iteration).
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/ta_probe scripts/ta_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int MODE, int ROWS_IN_FLIGHT>
__global__ __launch_bounds__(768) void probe(const uint16_t* table, int n_rows, int iters, float* out) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 12 + (threadIdx.x >> 6);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(table), 0, 0x7fffffff, 0x00020000);
    float acc = 0.f;
    const int pr = MODE == 0 ? (lane & 15) : MODE == 4 ? lane / 5 : (lane >> 2);
    int ch = MODE == 0 ? (lane >> 4) : MODE == 2 ? ((lane & 3) + 2) & 3 : MODE == 4 ? min(lane % 5, 3) : (lane & 3);
    for (int it = 0; it < iters; ++it) {
        const int row = (int)(hash32((uint32_t)(wave * 131071 + it * 16 + pr)) % (uint32_t)n_rows);
        const int c2 = MODE == 3 ? ch ^ (row & 3) : ch;
        const int base = row * 512 + 16 * c2;
        uint4 v[ROWS_IN_FLIGHT];
#pragma unroll
        for (int q = 0; q < ROWS_IN_FLIGHT; ++q)
            v[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, base + 64 * q, 0, 0));
#pragma unroll
        for (int q = 0; q < ROWS_IN_FLIGHT; ++q)
            acc += __uint_as_float(v[q].x) + __uint_as_float(v[q].y) + __uint_as_float(v[q].z) +
                   __uint_as_float(v[q].w);
    }
    if (acc == 1234.5f) out[wave * 64 + lane] = acc;
}

int main() {
    const int n_rows = 645, iters = 2000, blocks = 256;
    std::vector<uint16_t> h((size_t)n_rows * 256);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint16_t)(0x3f80 + (i % 7));
    uint16_t* d = nullptr;
    float* out = nullptr;
    hipMalloc(&d, h.size() * 2);
    hipMalloc(&out, (size_t)blocks * 12 * 64 * 4);
    hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, const char* name, int per_iter) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(blocks), dim3(768), 0, 0, d, n_rows, iters, out);
        hipEventRecord(e0);
        const int reps = 10;
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(768), 0, 0, d, n_rows, iters, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / reps;
        const double insns = (double)blocks * 12 * iters * per_iter;
        printf("{\"mode\": \"%s\", \"us\": %.2f, \"load_insns\": %.0f, \"ns_per_insn_per_cu\": %.3f, \"TBps\": %.2f}\n",
               name, us, insns, us * 1e3 / (insns / 256), insns * 1024 / (us * 1e-6) / 1e12);
    };
    run(probe<0, 8>, "A_pair_minor_x8", 8);
    run(probe<1, 8>, "B_pair_major_x8", 8);
    run(probe<0, 2>, "A_pair_minor_x2", 2);
    run(probe<1, 2>, "B_pair_major_x2", 2);
    run(probe<0, 8>, "A_pair_minor_x8", 8);
    run(probe<1, 8>, "B_pair_major_x8", 8);
    run(probe<2, 8>, "C_pair_major_rotated_x8", 8);
    run(probe<3, 8>, "E_pair_major_xor_by_row_x8", 8);
    run(probe<4, 8>, "S_slab_copy_5_lanes_per_row_x8", 8);
    hipFree(d);
    hipFree(out);
    return 0;
}
