// Peer-store exchange over xGMI (device side): a rank's finishing kernel stores its finished
// rows straight into every peer's copy of the row-split output (IPC-mapped peer memory), and
// the kernel's last workgroup raises an arrival flag at every peer, then waits for every
// peer's flag before the kernel ends — so the next kernel on this rank starts with the
// all-gathered rows in place.  It replaces the RCCL all-gather of the
// row-split blocks (sharding.py) for the small exchanges of config S.
//
// Memory protocol (system scope: the peers are other GPUs):
//   payload  every 16-B piece stored WRITE-THROUGH at system scope (buffer_store_dwordx4 ...
//            sc0 sc1) into the peer's buffer; every storing wave then `s_waitcnt vmcnt(0)`
//            (the stores are complete at the peer's memory), a workgroup barrier, and ONE lane
//            adds to this rank's arrival counter (agent scope) — in launches of >= 128
//            workgroups through one of 8 sub-counters first, whose last arriver adds to it;
//   flag     the workgroup whose add returns grid-1 (the last) stores epoch into word
//            [slot][rank] of every peer's flag block (lane p: peer p) (a system-scope relaxed atomic store:
//            global_store ... sc0 sc1) — the flag blocks live in uncached device memory
//            (hipDeviceMallocUncached), so polls never hit a stale cache line;
//   wait     the same wave polls this rank's own block, words [slot][0..world) (lane s: source
//            s), relaxed at system scope with s_sleep, until every peer's epoch arrived — BOUNDED: after
//            timeout ticks of s_memrealtime (100 MHz) it sets the error word and gives up; a
//            set error word poisons the exchange: later launches raise no flag and wait for
//            none (fail fast), so the peers' waits time out as well and every host raises;
//   consume  the kernels that read the gathered rows start after this kernel ends: the
//            dispatch's acquire makes the bytes the peers wrote into this GPU's memory visible
//            as it does for any earlier kernel's stores.
// Epochs: state[2·slot] counts a launch's arrivals (the last arriver resets it; sub-counters at
// state[DG_PEER_SUB_BASE + (8·slot + s)·DG_PEER_SUB_STRIDE], reset by their last arriver), state[2·slot+1]
// is the slot's epoch (launches completed), so no flag is ever reset and a graph replay needs
// no memset.  Reuse is safe with ONE buffer per slot: a rank can only overwrite a peer's copy
// of step t's rows after passing a later wait that needs that peer's next exchange, which the
// peer raises only after its kernels that read step t's rows have ended (stream order).
#pragma once

#include "common.h"

#ifndef DG_PEER_FENCES
#define DG_PEER_FENCES 1
#endif

namespace dg {

struct PeerK {
    int64_t delta[DG_PEER_MAX];     // bytes from this rank's region to rank p's, as mapped here
    uint32_t* flags[DG_PEER_MAX];   // rank p's flag block [DG_PEER_SLOTS][DG_PEER_MAX], mapped here
    uint32_t* state;                // this rank's {arrivals, epoch} per slot, then the error word
    int64_t timeout;                // s_memrealtime ticks a wait may spin
    int32_t rank, world, slot, loopback;
    int32_t on;                     // 0: no exchange (the kernel runs as without a descriptor)
    int32_t pad;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// launches of at least this many workgroups count their arrivals in two levels (peer_arrive)
constexpr uint32_t kPeerSubMin = 128;

// Validate a host descriptor and copy it into the kernel form.
inline int peer_convert(const dg_peer_xchg* x, PeerK& k) {
    k = PeerK{};
    if (!x) return DG_OK;
    if (x->world < 1 || x->world > DG_PEER_MAX || x->rank < 0 || x->rank >= x->world || x->slot < 0 ||
        x->slot >= DG_PEER_SLOTS || !x->state || x->timeout_ticks <= 0)
        return DG_EINVAL;
    for (int p = 0; p < x->world; ++p) {
        if (!x->flags[p] || (x->delta[p] & 15)) return DG_EINVAL;
        k.delta[p] = x->delta[p];
        k.flags[p] = x->flags[p];
    }
    if (x->delta[x->rank] != 0) return DG_EINVAL;
    k.state = x->state;
    k.timeout = x->timeout_ticks;
    k.rank = x->rank;
    k.world = x->world;
    k.slot = x->slot;
    k.loopback = x->loopback ? 1 : 0;
    k.on = 1;
    return DG_OK;
}

// Store v (16 B) at byte offset `off` of the row block that starts at `base` (this rank's
// copy) into every peer's copy, write-through at system scope.  base must be wave-uniform.
__device__ __forceinline__ void peer_store4(const PeerK& P, const float* base, uint32_t bytes, uint32_t off,
                                            const float4& v) {
    const u32x4 w = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
#pragma unroll 1
    for (int p = 0; p < P.world; ++p) {
        if (p == P.rank) continue;
        const char* pb = reinterpret_cast<const char*>(base) + P.delta[p];
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pb), 0, (int)bytes, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(w, rs, (int)off, 0, 17);  // aux 17 = sc0 sc1
    }
}

__device__ __forceinline__ void diag_store(const PeerK& P, int word, uint32_t v) {
    __hip_atomic_store(P.state + DG_PEER_DIAG_BASE + word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave-level bounded wait: lane s polls word [slot][s] of this rank's block (one round trip per
// poll for every source) until all of [0, world) reached epoch; on timeout the wait record
// (decagon_hip.h, DG_PEER_DIAG_BASE: slot, expected epoch, each source's last flag word, the
// start / give-up / flag-raise ticks) is written, then lane 0 sets the error word
// (0x10000 | slot << 8 | the first late source).  t_raise: when this rank raised its flags.
__device__ __forceinline__ void peer_poll(const PeerK& P, uint32_t epoch, int lane, uint64_t t_raise) {
    const bool mine = lane < P.world;
    const uint32_t* own = P.flags[P.rank] + P.slot * DG_PEER_MAX + lane;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (;;) {
        const uint32_t v = mine ? __hip_atomic_load(own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : epoch;
        const uint64_t who = __ballot((int32_t)(v - epoch) < 0);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (!who) {
            // system-scope acquire after the flags matched (buffer_inv sc0 sc1): this wave's
            // later loads see what the peers released before raising them; the launches that
            // read the gathered rows start after this one ends, behind their own acquire
#if DG_PEER_FENCES
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#endif
            if (now - t0 > (uint64_t)DG_PEER_SLOW_TICKS && lane == 0) {  // a slow wait: count it, keep its max
                __hip_atomic_fetch_add(P.state + DG_PEER_DIAG_BASE + 16, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_max(P.state + DG_PEER_DIAG_BASE + 17, (uint32_t)min(now - t0, (uint64_t)0xffffffffu),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }
        if (now - t0 > (uint64_t)P.timeout) {
            if (mine) diag_store(P, 2 + lane, v);  // each source's flag word as last read
            if (lane == 0) {
                diag_store(P, 0, (uint32_t)P.slot);
                diag_store(P, 1, epoch);
                diag_store(P, 10, (uint32_t)t0);
                diag_store(P, 11, (uint32_t)(t0 >> 32));
                diag_store(P, 12, (uint32_t)now);
                diag_store(P, 13, (uint32_t)(now >> 32));
                diag_store(P, 14, (uint32_t)t_raise);
                diag_store(P, 15, (uint32_t)(t_raise >> 32));
                __hip_atomic_store(P.state + 2 * DG_PEER_SLOTS,
                                   0x10000u | ((uint32_t)P.slot << 8) | ((uint32_t)__ffsll((long long)who) - 1u),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Called by EVERY thread of EVERY workgroup of the launch after its peer stores: drain, meet,
// count; wave 0 of the last workgroup raises this rank's flag at every peer (lane p stores to
// peer p) and waits for theirs (lane s polls source s: one round trip per poll for all ranks),
// bounded.
__device__ __forceinline__ void peer_arrive(const PeerK& P) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc0 sc1 stores complete
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    uint32_t* arrivals = P.state + 2 * P.slot;
    uint32_t old = 0;
    if (gridDim.x >= kPeerSubMin) {
        // two-level count: workgroup b arrives on sub-counter b & 7 of the slot (one 64-B line
        // each, so the ≈ gridDim / 8 returning adds of each proceed beside the others' instead of
        // queueing on one word); the last of each sub-group arrives on the slot's counter.
        // Loopback A/B (scripts/sim_ab.sh): config P at N = 8 (≈ 760 workgroups a pushing
        // epilogue) 122 → 112.7 µs a rank, config S at N = 2 (≈ 450) 26.0 → 24.5; config S at
        // N = 8 (29) 25.9 → 26.6, hence the threshold
        const uint32_t sub = blockIdx.x & 7u;
        const uint32_t n_sub = (gridDim.x - sub + 7u) / 8u;  // workgroups b with b & 7 == sub
        uint32_t* sc = P.state + DG_PEER_SUB_BASE + (P.slot * 8 + sub) * DG_PEER_SUB_STRIDE;
        if (lane == 0) old = __hip_atomic_fetch_add(sc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __shfl(old, 0);
        if (old + 1u != n_sub) return;
        if (lane == 0) {
            __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch counts anew
            old = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        old = __shfl(old, 0);
        if (old + 1u != 8u) return;
    } else {
        if (lane == 0) old = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __shfl(old, 0);
        if (old + 1u != gridDim.x) return;
    }
    uint32_t* ep = P.state + 2 * P.slot + 1;
    const uint32_t* err = P.state + 2 * DG_PEER_SLOTS;
    uint32_t epoch = 0, failed = 0;
    if (lane == 0) {
        __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch counts anew
        epoch = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    epoch = __shfl(epoch, 0);
    failed = __shfl(failed, 0);
    // A set error word poisons the exchange: this rank raises no flag and waits for none, so
    // every peer's next wait times out too and every rank's host raises at its next check
    // (PeerExchange.check, Session.run) instead of computing on rows that never arrived.
    if (failed) return;
    // System-scope release before the flags (AMDGPU memory model, gfx942/gfx950: a release at
    // system scope is buffer_wbl2 sc0 sc1 + s_waitcnt vmcnt(0)): every byte this agent wrote
    // before — the other workgroups' payload stores, each drained before its arrival add — is
    // visible to the other agents before any flag store is.  The asm wait keeps the write-back
    // ahead of the flag store even where the compiler drops the fence's own wait
    // (MI355X_MICROARCH.md, "Compiler hazard").
#if DG_PEER_FENCES
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    // lane p < world: rank p's flag block (a select chain over the kernel arguments: no scratch)
    uint32_t* fp = nullptr;
#pragma unroll
    for (int p = 0; p < DG_PEER_MAX; ++p)
        if (lane == p) fp = P.flags[p];
    const uint64_t t_raise = __builtin_amdgcn_s_memrealtime();
    if (lane < P.world)
        __hip_atomic_store(fp + P.slot * DG_PEER_MAX + (P.loopback ? lane : P.rank), epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    peer_poll(P, epoch, lane, t_raise);
    if (lane == 0) __hip_atomic_store(ep, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dg
