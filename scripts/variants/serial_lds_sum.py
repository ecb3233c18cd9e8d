# A/B: the one-wave relation / group sums of the tab kernels as the serial loop of round 5
# (one LDS round trip per row) instead of lds_ordered_sum's batched reads — the same bits.
EDITS = [("segspmm.hip", """    float4 s = rows[0][q];
#pragma unroll 1
    for (int u0 = 1; u0 < K; u0 += 8) {
        float4 z[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) z[j] = rows[u0 + j < K ? u0 + j : 0][q];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (u0 + j < K) dg::add4(s, z[j]);
    }
    return s;""", """    float4 s = rows[0][q];
#pragma unroll 1
    for (int u = 1; u < K; ++u) dg::add4(s, rows[u][q]);
    return s;""")]
