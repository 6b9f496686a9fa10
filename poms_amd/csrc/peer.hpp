// The peer transport of the slab ghost exchange (csrc/comm.hip): the mailbox block
// layout, the argument block of one exchange and the device code that runs it.
// (Run by extra workgroups inside the v5 interior launch instead, it doubled the
// SGPR spills of the Jacobi build -- 64 -> 245 lane moves per 7 planes in its march
// -- and was slower on the loopback proxy: DESIGN.md section 4.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace poms {

// Block layout (u64 words): [0, 256) arrive_from_prev, [256, 512) arrive_from_next,
// [512, 768) ack_from_prev, [768, 1024) ack_from_next -- one slot per workgroup of
// the WRITING rank's kernel, each holding the last exchange number that workgroup
// finished -- then the rank's own exchange count, a done counter and a status word;
// the two mailbox sides (side 0: planes from prev, side 1: from next) from byte
// kPeerHdr.  Slots are plain stores of monotonic numbers: no remote atomics.

constexpr int kPeerMaxWgs = 256;
constexpr int kArrPrev = 0, kArrNext = 256, kAckPrev = 512, kAckNext = 768, kSeq = 1024, kDone = 1032,
              kStatus = 1040;
constexpr size_t kPeerHdr = 16384;
constexpr int64_t kPeerTimeoutTicks = 2000000000ll;   // 20 s of the 100 MHz wall clock

struct PeerArgs {
    const double* send_lo;   // my first `width` owned planes
    const double* send_hi;   // my last `width` owned planes
    double* ghost_lo;
    double* ghost_hi;
    int64_t cnt;             // doubles per side
    uint64_t* own;
    // per link (lo: with prev, hi: with next; nullptr: no such neighbour): where the
    // boundary planes go and the arrival slots to set there, and where this rank's
    // acknowledgement of the neighbour's planes goes.  Between ranks the lo link
    // writes prev's side 1 / arrive_from_next and acks into prev's ack_from_next; on
    // a one-rank loopback it writes this rank's own side 0 / arrive_from_prev (the
    // ghosts then hold the slab's own boundary planes, as with RCCL's self-send).
    double* out_lo;
    uint64_t* arr_lo;
    uint64_t* ack_lo;
    double* out_hi;
    uint64_t* arr_hi;
    uint64_t* ack_hi;
    int64_t cap;             // doubles per mailbox side
    int G;                   // exchange workgroups (0: no exchange in this launch)
    // set to 1 (system scope) when a wait times out: pinned, device-mapped HOST memory,
    // which every host-synchronising communicator call reads (poms_comm_wait fails
    // loudly on it, so a timed-out exchange is never consumed silently)
    uint64_t* status;
};

#ifdef __HIPCC__
__device__ __forceinline__ double* peer_side(uint64_t* blk, int side, int64_t cap) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(blk) + kPeerHdr) + (int64_t)side * cap;
}

// Memory ordering without cache maintenance.  A release / acquire fence at agent or
// system scope writes back / invalidates the whole L2 of the XCD: one per workgroup
// and spin iteration cost the first version 147 us per headline exchange, and the
// interior launch beside it its cached lines.  Instead every access to a mailbox or
// a flag slot is a relaxed SYSTEM-scope atomic (the scope bits make the store write
// through and the load read coherently; no fence is emitted), a writer waits for its
// stores to complete (vmcnt 0) before the flag store, and a reader issues its
// mailbox loads only after it saw the flag (workgroup barrier in between).
__device__ __forceinline__ uint64_t sys_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void stores_done() { __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// threads t < nwg wait until slot[t] >= v; bounded: on timeout the status word is
// set and the wait gives up, so a lost peer can never hang the GPU
__device__ __forceinline__ void peer_wait(const uint64_t* slots, uint64_t v, int nwg, uint64_t* status,
                                          uint64_t t_end) {
    const int t = threadIdx.x;
    if (t < nwg) {
        while (sys_load(slots + t) < v) {
            if (wall_clock64() > t_end) {
                sys_store(status, 1ull);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

// this workgroup's share [lo, hi) of `cnt` doubles, U loads in flight per thread:
// into a mailbox (system-scope stores) or out of one (system-scope loads)
template <bool TO_MAILBOX>
__device__ __forceinline__ void peer_copy(double* __restrict__ dst, const double* __restrict__ src, int64_t lo,
                                          int64_t hi) {
    constexpr int U = 8;
    const int64_t step = blockDim.x;
    auto* d = reinterpret_cast<uint64_t*>(dst);
    auto* q = reinterpret_cast<const uint64_t*>(src);
    int64_t i = lo + threadIdx.x;
    for (; i + (U - 1) * step < hi; i += U * step) {
        uint64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = TO_MAILBOX ? q[i + u * step] : sys_load(q + i + u * step);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (TO_MAILBOX) sys_store(d + i + u * step, v[u]);
            else d[i + u * step] = v[u];
        }
    }
    for (; i < hi; i += step) {
        if (TO_MAILBOX) sys_store(d + i, q[i]);
        else d[i] = sys_load(q + i);
    }
}

// One exchange, run by workgroup w of the G exchange workgroups (all of blockDim.x
// threads; G == PeerArgs::G on every rank).
__device__ __forceinline__ void peer_exchange_body(const PeerArgs& a, const int w, const int G) {
    uint64_t* status = a.status;
    const uint64_t s = sys_load(a.own + kSeq) + 1;
    const uint64_t t_end = wall_clock64() + kPeerTimeoutTicks;
    const int64_t per = (a.cnt + G - 1) / G;
    const int64_t lo = min(a.cnt, per * w), hi = min(a.cnt, lo + per);
    const bool L = a.out_lo != nullptr, H = a.out_hi != nullptr;
    // A: the receivers consumed what this rank wrote into their mailboxes last time
    if (L) peer_wait(a.own + kAckPrev, s - 1, G, status, t_end);
    if (H) peer_wait(a.own + kAckNext, s - 1, G, status, t_end);
    // B: boundary planes into the receivers' mailboxes, then this workgroup's slot
    if (L) peer_copy<true>(a.out_lo, a.send_lo, lo, hi);
    if (H) peer_copy<true>(a.out_hi, a.send_hi, lo, hi);
    stores_done();
    __syncthreads();
    if (threadIdx.x == 0) {
        if (L) sys_store(a.arr_lo + w, s);
        if (H) sys_store(a.arr_hi + w, s);
    }
    // C: every workgroup of each sender wrote this exchange's planes here
    if (L) peer_wait(a.own + kArrPrev, s, G, status, t_end);
    if (H) peer_wait(a.own + kArrNext, s, G, status, t_end);
    // D: mailboxes into the ghost planes, then tell the senders (their loads returned)
    if (L) peer_copy<false>(a.ghost_lo, peer_side(a.own, 0, a.cap), lo, hi);
    if (H) peer_copy<false>(a.ghost_hi, peer_side(a.own, 1, a.cap), lo, hi);
    stores_done();
    __syncthreads();
    if (threadIdx.x == 0) {
        if (L) sys_store(a.ack_lo + w, s);
        if (H) sys_store(a.ack_hi + w, s);
        // the last workgroup out counts the exchange (every workgroup has read s by now)
        if (__hip_atomic_fetch_add(a.own + kDone, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ==
            (uint64_t)(G - 1)) {
            sys_store(a.own + kDone, 0ull);
            sys_store(a.own + kSeq, s);
        }
    }
}
#endif

}  // namespace poms
