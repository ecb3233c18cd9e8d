# A/B: the reassociated layer 2 of the tab kernels loads its W slab slice (8 float4 a lane)
# before the first gathers instead of after the last (+32 VGPRs through the gather loop; the
# slice's L2 round trip then overlaps the gathers' instead of trailing them).
EDITS = [("segspmm.hip", """        const uint2* nx = ovf + D.ovf;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
        for (int base = 0; base < D.cnt; base += 64) {""", """        const uint2* nx = ovf + D.ovf;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        float4 wv[8];
        if constexpr (PROJ) {
            const float4* w = reinterpret_cast<const float4*>(D.w) + (8 * (lane >> 3)) * 8 + (lane & 7);
#pragma unroll
            for (int i = 0; i < 8; ++i) wv[i] = w[8 * i];
        }
#pragma unroll 1
        for (int base = 0; base < D.cnt; base += 64) {"""),
         ("segspmm.hip", """            const int ms = lane >> 3;
            const float4* w = reinterpret_cast<const float4*>(D.w) + (8 * ms) * 8 + (lane & 7);
            float4 wv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) wv[i] = w[8 * i];
            if (lane < 16) ybuf[lane] = acc;""", """            const int ms = lane >> 3;
            if (lane < 16) ybuf[lane] = acc;""")]
