// Peer memory for the xGMI exchange: IPC export / import of exchange regions, the uncached
// flag blocks, and the stand-alone peer-store all-gather kernel (peer.h has the protocol).
//
// Reference op replaced: none directly — the reference runs on one CPU process.  This is the
// exchange step of the sharded forward (sharding.py), the all-gather of the row-split blocks
// that the per-(i,j) normalisation of layers.py:92-93 makes necessary once per layer.
#include <cstring>

#include "common.h"
#include "peer.h"

namespace {

// One workgroup per 16 KB of the pushed bytes: each thread copies 16-B pieces of this rank's
// block(s) into every peer's copy (write-through, system scope), then peer_arrive.
struct PushSeg {
    int64_t off;    // byte offset of the block in the region (16-B aligned)
    int64_t bytes;  // multiple of 16
    int32_t block_begin;
    int32_t pad;
};

struct PushArgs {
    PushSeg s[DG_MAX_GROUPS];
    const char* base;  // this rank's region
    int32_t n_seg;
    int32_t pad;
    dg::PeerK P;
};

constexpr int kPushThreads = 256;
constexpr int kPushBytes = 16384;  // per workgroup: 4 pieces of 16 B per thread

__global__ __launch_bounds__(kPushThreads) void peer_push_kernel(const PushArgs a) {
    int si = 0;
#pragma unroll 1
    while (si + 1 < a.n_seg && (int)blockIdx.x >= a.s[si + 1].block_begin) ++si;
    const PushSeg& S = a.s[si];
    const int64_t b0 = (int64_t)(blockIdx.x - S.block_begin) * kPushBytes;
    const float* base = reinterpret_cast<const float*>(a.base + S.off);  // workgroup-uniform
    if (b0 < S.bytes) {
        float4 v[kPushBytes / (16 * kPushThreads)];
#pragma unroll
        for (int u = 0; u < kPushBytes / (16 * kPushThreads); ++u) {
            const int64_t o = b0 + (int64_t)(u * kPushThreads + threadIdx.x) * 16;
            v[u] = o < S.bytes ? *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + o)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < kPushBytes / (16 * kPushThreads); ++u) {
            const int64_t o = b0 + (int64_t)(u * kPushThreads + threadIdx.x) * 16;
            if (o < S.bytes) dg::peer_store4(a.P, base, (uint32_t)S.bytes, (uint32_t)o, v[u]);
        }
    }
    dg::peer_arrive(a.P);
}

}  // namespace

extern "C" int dg_peer_alloc(int64_t bytes, int32_t kind, void** ptr) {
    if (!ptr || bytes <= 0 || kind < 0 || kind > 2) return DG_EINVAL;
    *ptr = nullptr;
    const unsigned flags = kind == 0 ? hipDeviceMallocDefault
                                     : (kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
    hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, flags);
    if (e != hipSuccess) {
        *ptr = nullptr;
        (void)hipGetLastError();
        return static_cast<int>(e);
    }
    e = hipMemset(*ptr, 0, (size_t)bytes);
    if (e != hipSuccess) {
        (void)hipFree(*ptr);
        *ptr = nullptr;
        return static_cast<int>(e);
    }
    return DG_OK;
}

extern "C" int dg_peer_read(const void* device, void* host, int64_t bytes) {
    if (!device || !host || bytes <= 0) return DG_EINVAL;
    const hipError_t e = hipMemcpy(host, device, (size_t)bytes, hipMemcpyDeviceToHost);
    return e == hipSuccess ? DG_OK : static_cast<int>(e);
}

extern "C" int dg_peer_free(void* ptr) {
    if (!ptr) return DG_OK;
    const hipError_t e = hipFree(ptr);
    return e == hipSuccess ? DG_OK : static_cast<int>(e);
}

extern "C" int dg_ipc_get_handle(void* ptr, void* handle, int64_t* offset) {
    if (!ptr || !handle || !offset) return DG_EINVAL;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, ptr);
    if (e != hipSuccess) return static_cast<int>(e);
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, base);
    if (e != hipSuccess) return static_cast<int>(e);
    static_assert(sizeof(h) == DG_IPC_HANDLE_BYTES, "hipIpcMemHandle_t size");
    memcpy(handle, &h, sizeof(h));
    *offset = static_cast<int64_t>(reinterpret_cast<char*>(ptr) - reinterpret_cast<char*>(base));
    return DG_OK;
}

extern "C" int dg_ipc_open(const void* handle, void** ptr) {
    if (!handle || !ptr) return DG_EINVAL;
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    *ptr = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        *ptr = nullptr;
        (void)hipGetLastError();
        return static_cast<int>(e);
    }
    return DG_OK;
}

extern "C" int dg_ipc_close(void* ptr) {
    if (!ptr) return DG_OK;
    const hipError_t e = hipIpcCloseMemHandle(ptr);
    return e == hipSuccess ? DG_OK : static_cast<int>(e);
}

extern "C" int dg_peer_allgather(const dg_peer_xchg* xchg, const void* region, const int64_t* offsets,
                                 const int64_t* sizes, int32_t n_seg, void* stream) {
    if (!xchg || !region || n_seg < 1 || n_seg > DG_MAX_GROUPS || !offsets || !sizes) return DG_EINVAL;
    PushArgs a{};
    const int rc = dg::peer_convert(xchg, a.P);
    if (rc != DG_OK) return rc;
    if (!dg::aligned16(region)) return DG_EALIGN;
    a.base = reinterpret_cast<const char*>(region);
    int64_t blocks = 0;
    for (int i = 0; i < n_seg; ++i) {
        if (offsets[i] < 0 || sizes[i] < 0 || (offsets[i] & 15) || (sizes[i] & 15)) return DG_EINVAL;
        if (sizes[i] > 0x7fffffffLL) return DG_EINVAL;  // 32-bit buffer offsets
        a.s[i].off = offsets[i];
        a.s[i].bytes = sizes[i];
        a.s[i].block_begin = static_cast<int32_t>(blocks);
        blocks += sizes[i] ? (sizes[i] + kPushBytes - 1) / kPushBytes : 0;
    }
    a.n_seg = n_seg;
    if (blocks == 0) blocks = 1;  // nothing to push: one workgroup still raises and waits
    if (blocks > 0x7fffffff) return DG_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(peer_push_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kPushThreads), 0, st, a);
    return dg::launch_status();
}
