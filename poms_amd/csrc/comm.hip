// Native RCCL communicator for the slab decomposition (one rank per GPU):
// the p-plane ghost exchange with rank +-1 and the scalar all-reduces of pcg /
// damped Jacobi, issued from C so that a sweep costs the host a few
// microseconds instead of a torch.distributed round trip.
//
// Every RCCL operation goes to ONE communication stream, in the order the host
// issues it (the same on every rank), ordered against the caller's stream with
// events: the exchange waits for the planes to be written, the caller's stream
// waits for the exchange only where the ghosts are read.
//
// Replaces the reference's `_update_ghost_regions_parallel` (Irecv/Isend/Waitall
// per direction, `pyccel/kron_product.py:21-41`) and `comm.allreduce` of the
// solver scalars (`sources/solvers.py:87-124`, `sources/mg_jac.py:95`).
#include "common.hpp"
#include "split_hooks.hpp"
#include "peer.hpp"
#include "../../include/poms_hip.h"

#include <rccl/rccl.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace poms;

struct poms_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
    hipStream_t cs = nullptr;       // the communication stream
    hipEvent_t ev_in = nullptr;     // caller's stream -> cs
    hipEvent_t ev_halo = nullptr;   // exchange done (cs -> caller)
    hipEvent_t ev_red = nullptr;    // all-reduce done (cs -> caller)
    hipEvent_t ev_bnd = nullptr;    // boundary launch on cs done (cs -> caller)
    // Ring of slots for global sums only the host reads (the damped-Jacobi norms,
    // pcg's r.r): a launch's reduction kernel writes the rank's local sum straight
    // into the slot -- pinned, coherent host memory mapped into the device -- and
    // poms_comm_wait sums the ranks' values ON THE HOST (shared memory between the
    // ranks of the node, or the host transport's callback).  No RCCL kernel, no copy
    // and nothing on the communication stream, which then carries the ghost exchange
    // alone: each such kernel used to wait for CUs behind the interior launch and
    // hold up the next exchange (profiles/r03/proxy/).
    static constexpr int kRing = 16;
    double* ring = nullptr;         // kRing x 2 doubles, host-coherent, device-mapped
    hipEvent_t ring_ev[kRing] = {}; // after the launch that writes the slot
    double* ring_dst[kRing] = {};   // where poms_comm_wait leaves the global sums
    int ring_cnt[kRing] = {};
    bool ring_done[kRing] = {};
    int ring_next = 0;
    // node-local shared memory for the host-side sums (nullptr: not all ranks on this
    // node -- the sums then go through RCCL synchronously)
    struct ShmSlot {
        std::atomic<uint64_t> seq;
        double v[2];
        char pad[64 - sizeof(std::atomic<uint64_t>) - 2 * sizeof(double)];
    };
    ShmSlot* shm = nullptr;         // [2][nranks]: round s uses half s & 1
    size_t shm_bytes = 0;
    uint64_t shm_seq = 0;
    char shm_name[64] = {};
    double* dev_tmp = nullptr;      // 2 doubles: the RCCL fall-back of the host sums
    // host transport (poms_comm_create_host): the same schedule with the data moved
    // by caller-supplied host callbacks (e.g. torch.distributed / gloo) instead of
    // RCCL -- every call synchronises the caller's stream, stages the planes or
    // scalars through host memory and runs the callback in line
    bool host = false;
    poms_host_exchange_fn xchg = nullptr;
    poms_host_allreduce_fn ar = nullptr;
    void* user = nullptr;
    std::vector<double> stage;      // 4 x width x plane_elems (send lo / recv lo / send hi / recv hi)
    // peer transport (poms_comm_set_peer): the ghost exchange as ONE kernel on the
    // communication stream that writes the boundary planes straight into the
    // neighbours' mailboxes (IPC-mapped device memory, xGMI peer stores) and copies
    // its own mailboxes into the ghost planes, synchronised by per-workgroup flag
    // slots -- no RCCL call, no host step, capturable into a graph
    bool peer_on = false;
    int peer_wgs = 32;                // exchange workgroups (the same on every rank)
    int peer_prev = -2, peer_next = -2;   // the neighbours the blocks were exchanged with
    int64_t peer_cap = 0;             // doubles per mailbox side
    char* pblk = nullptr;             // own block: flag slots + 2 mailbox sides
    char* pprev = nullptr;            // the neighbours' blocks (IPC-opened; own on a loopback)
    char* pnext = nullptr;
    bool pprev_ipc = false, pnext_ipc = false;
    bool peer_fine = false;           // own block is fine-grained (coherent) device memory
    hipStream_t halo_on = nullptr;    // the stream the last exchange was queued on
    uint64_t* peer_status = nullptr;  // timeout flag of the exchange kernel (pinned, device-mapped host memory)
    uint64_t* peer_status_dev = nullptr;   // its device address (taken once: not a call to make inside a capture)
    // an exchange was queued while a stream was being captured: graphs now hold raw
    // pointers into the mailbox block and its flag slots, so the block may no longer be
    // rebuilt or released (advisor, round 5)
    bool peer_captured = false;
};

#define POMS_NCCL_CHECK(expr)                                                    \
    do {                                                                         \
        ncclResult_t _r = (expr);                                                \
        if (_r != ncclSuccess) {                                                 \
            ::poms::set_error(std::string(#expr) + ": " + ncclGetErrorString(_r)); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

static hipStream_t cstream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// The stream an RCCL call of this communicator goes to: the communication stream, or
// -- while the caller's stream is being captured into a graph -- the capturing stream
// itself.  With the HIP 7.0 runtime torch bundles (the one every library process runs
// on: same SONAME, loaded first), hipStreamEndCapture segfaults when RCCL's grouped
// send / receive was captured on a stream FORKED from the capturing one by an event;
// captured on the capturing stream it works, as does the fork with the ROCm 7.2 runtime
// and a fork around a plain kernel (tools/r06/graph_probe.cpp, profiles/r06/graph_probe/).
static hipStream_t rccl_stream(poms_comm* c, hipStream_t caller) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(caller, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return caller;
    return c->cs;
}

// A call that waits on the host (event / stream synchronisation, a host callback)
// must not run while `s` is being captured into a graph: nothing captured has run,
// so it would wait for work that never starts or read values never written.  Such a
// call fails loudly instead (round-4 verdict: capture of a smoother call with a
// communicator had crashed with no diagnosis).
static int refuse_in_capture(hipStream_t s, const char* what) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) return 0;
    if (cs != hipStreamCaptureStatusNone) {
        ::poms::set_error(std::string(what) + ": host-synchronising call during stream capture");
        return 1;
    }
    return 0;
}

namespace poms {
int op_run_split(poms_op* op, int epilogue, double omega, const double* x, double* y, const double* b,
                 int64_t ib, int64_t ie, int64_t b1s, int64_t b1e, int64_t b2s, int64_t b2e, double* norm_out,
                 double* dot_out, const SplitHooks& h, void* stream);
}

static bool getenv_off(const char* name) {
    const char* e = getenv(name);
    return e && e[0] == '0';
}

// a NaN payload no reduction produces: "this slot has not been written yet"
static constexpr uint64_t kUnset = 0x7ff8dead0000beefull;
static void slot_arm(double* v) {
    std::memcpy(v, &kUnset, sizeof(double));
}
static bool slot_unset(const double* v) {
    uint64_t u;
    std::memcpy(&u, const_cast<const double*>(reinterpret_cast<const volatile double*>(v)), sizeof(u));
    return u == kUnset;
}

// Map the node-local shared-memory block of the communicator named by `id` and mark
// this rank present.  Every rank calls this before ncclCommInitRank (a collective):
// after it, all ranks of THIS node have marked themselves, and poms_comm_create
// agrees over the ranks whether every rank found all the others.
static void shm_open_block(poms_comm* c, const char* id, size_t id_len) {
    uint64_t h = 1469598103934665603ull;   // FNV-1a of the id bytes
    for (size_t i = 0; i < id_len; ++i) h = (h ^ (uint8_t)id[i]) * 1099511628211ull;
    char name[64];
    snprintf(name, sizeof(name), "/poms_comm_%016llx", (unsigned long long)h);
    c->shm_bytes = (size_t)(2 * c->nranks + 1) * sizeof(poms_comm::ShmSlot);
    int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) return;
    if (ftruncate(fd, (off_t)c->shm_bytes) != 0) { close(fd); return; }
    void* p = mmap(nullptr, c->shm_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return;
    c->shm = static_cast<poms_comm::ShmSlot*>(p);
    // the last slot's seq counts the ranks present (zero-filled by the first ftruncate)
    reinterpret_cast<std::atomic<uint64_t>*>(&c->shm[2 * c->nranks].seq)->fetch_add(1);
    snprintf(c->shm_name, sizeof(c->shm_name), "%s", name);
}

// ---- peer transport (csrc/peer.hpp) -------------------------------------------
namespace {
__global__ void __launch_bounds__(256) peer_exchange_kernel(const PeerArgs a) { peer_exchange_body(a, blockIdx.x, gridDim.x); }

double* peer_side_host(uint64_t* blk, int side, int64_t cap) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(blk) + kPeerHdr) + (int64_t)side * cap;
}
}  // namespace

static void peer_release(poms_comm* c) {
    if (c->pprev_ipc && c->pprev) (void)hipIpcCloseMemHandle(c->pprev);
    if (c->pnext_ipc && c->pnext && c->pnext != c->pprev) (void)hipIpcCloseMemHandle(c->pnext);
    if (c->pblk) (void)hipFree(c->pblk);
    c->pblk = c->pprev = c->pnext = nullptr;
    c->pprev_ipc = c->pnext_ipc = false;
    c->peer_cap = 0;
    c->peer_prev = c->peer_next = -2;
}

// Pass `bytes` of host data to prev / next and take theirs (blocking): the host
// callback, or RCCL send/recv on the communication stream.  prev == next (a
// one-rank loopback): nothing to exchange, the caller uses its own block.
static int peer_swap_bytes(poms_comm* c, const void* mine, void* from_prev, void* from_next, int bytes, int prev,
                           int next) {
    const int nd = (bytes + 7) / 8;
    std::vector<double> st(4 * (size_t)nd, 0.0);
    std::memcpy(st.data(), mine, bytes);
    std::memcpy(st.data() + 2 * nd, mine, bytes);
    if (c->host) {
        if (c->xchg(c->user, st.data(), st.data() + nd, st.data() + 2 * nd, st.data() + 3 * nd, nd, prev, next)) {
            set_error("peer transport: handle exchange callback failed");
            return 1;
        }
    } else {
        double* d = nullptr;
        POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d), 4 * (size_t)nd * sizeof(double)));
        bool ok = hipMemcpy(d, st.data(), 4 * (size_t)nd * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && ncclGroupStart() == ncclSuccess;
        if (ok && prev >= 0)
            ok = ncclSend(d, nd, ncclDouble, prev, c->comm, c->cs) == ncclSuccess &&
                 ncclRecv(d + nd, nd, ncclDouble, prev, c->comm, c->cs) == ncclSuccess;
        if (ok && next >= 0)
            ok = ncclSend(d + 2 * nd, nd, ncclDouble, next, c->comm, c->cs) == ncclSuccess &&
                 ncclRecv(d + 3 * nd, nd, ncclDouble, next, c->comm, c->cs) == ncclSuccess;
        ok = (ncclGroupEnd() == ncclSuccess) && ok;
        ok = ok && hipStreamSynchronize(c->cs) == hipSuccess &&
             hipMemcpy(st.data(), d, 4 * (size_t)nd * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
        (void)hipFree(d);
        if (!ok) { set_error("peer transport: handle exchange over RCCL failed"); return 1; }
    }
    if (prev >= 0) std::memcpy(from_prev, st.data() + nd, bytes);
    if (next >= 0) std::memcpy(from_next, st.data() + 3 * nd, bytes);
    return 0;
}

// Blocks of `cnt` doubles per side with the neighbours prev / next, (re)built when
// missing, too small or exchanged with other neighbours.  Collective over the two
// neighbours (every rank issues the same exchanges in the same order, so all of
// them rebuild at the same call); never inside a capture.
// A timed-out exchange (a neighbour lagged by more than 20 s) left stale or partly
// written mailbox contents in the ghost planes: every later result is invalid.
static int peer_check(poms_comm* c) {
    if (c->peer_status && __atomic_load_n(c->peer_status, __ATOMIC_ACQUIRE) != 0) {
        set_error("peer transport: a ghost exchange timed out waiting for a neighbour (> 20 s); "
                  "its ghost planes, and every result computed from them, are invalid");
        return 1;
    }
    return 0;
}

static int peer_ensure(poms_comm* c, int64_t cnt, int prev, int next, hipStream_t st) {
    if (c->pblk && cnt <= c->peer_cap && prev == c->peer_prev && next == c->peer_next) return 0;
    if (refuse_in_capture(st, "peer transport setup (first exchange of this size)")) return 1;
    if (c->pblk && c->peer_captured) {
        set_error("peer transport: the mailboxes would be rebuilt (a larger exchange or other neighbours) after "
                  "an exchange was captured into a graph, whose replays would then write freed memory; "
                  "reserve the largest exchange (poms_comm_peer_reserve) before capturing");
        return 1;
    }
    if (!c->peer_status) {
        void* h = nullptr;
        POMS_HIP_CHECK(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
        c->peer_status = static_cast<uint64_t*>(h);
        *c->peer_status = 0;
        void* sd = nullptr;
        POMS_HIP_CHECK(hipHostGetDevicePointer(&sd, c->peer_status, 0));
        c->peer_status_dev = static_cast<uint64_t*>(sd);
    }
    // every earlier exchange of this rank is complete, hence every neighbour's store
    // into the old block (the neighbours, in turn, finish theirs before answering the
    // handle exchange below)
    POMS_HIP_CHECK(hipStreamSynchronize(c->cs));
    POMS_HIP_CHECK(hipStreamSynchronize(st));
    const bool loop = c->nranks == 1;   // a one-rank loopback: the neighbours are this rank
    char* old = c->pblk;
    char* old_prev = c->pprev;
    char* old_next = c->pnext;
    const bool old_prev_ipc = c->pprev_ipc, old_next_ipc = c->pnext_ipc;
    const int64_t cap = (std::max<int64_t>(cnt, 1 << 16) + 31) & ~(int64_t)31;   // (keeps side 1 16-B aligned)
    const size_t bytes = kPeerHdr + 2 * (size_t)cap * sizeof(double);
    char* blk = nullptr;
    // fine-grained (coherent between devices and XCDs) unless POMS_PEER_FINE=0 (tuning)
    const char* fe = getenv("POMS_PEER_FINE");
    const bool want_fine = fe ? fe[0] != '0' : true;
    bool fine = want_fine &&
                hipExtMallocWithFlags(reinterpret_cast<void**>(&blk), bytes, hipDeviceMallocFinegrained) == hipSuccess;
    hipIpcMemHandle_t mine{};
    if (fine && !loop && hipIpcGetMemHandle(&mine, blk) != hipSuccess) {   // not exportable: plain device memory
        (void)hipFree(blk);
        blk = nullptr;
        fine = false;
    }
    (void)hipGetLastError();
    if (!blk) {
        POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&blk), bytes));
        if (!loop && hipIpcGetMemHandle(&mine, blk) != hipSuccess) {
            (void)hipFree(blk);
            set_error("peer transport: hipIpcGetMemHandle of the mailboxes failed");
            return 1;
        }
    }
    if (hipMemset(blk, 0, kPeerHdr) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(blk);
        set_error("peer transport: clearing the flag slots failed");
        return 1;
    }
    char* np = nullptr;
    char* nn = nullptr;
    bool pi = false, ni = false;
    // on any failure below: nothing of the new block stays mapped or allocated (the old
    // one, if any, stays in use)
    auto fail = [&](const std::string& msg) {
        if (pi && np) (void)hipIpcCloseMemHandle(np);
        if (ni && nn) (void)hipIpcCloseMemHandle(nn);
        (void)hipFree(blk);
        if (!msg.empty()) set_error(msg);
        return 1;
    };
    if (loop) {
        np = prev >= 0 ? blk : nullptr;
        nn = next >= 0 ? blk : nullptr;
    } else {
        // each rank sends its handle and the capacity, so that a mismatch fails loudly
        // ... and its exchange workgroup count: each workgroup waits for the slots of
        // the neighbour's G workgroups, so unequal counts could only end in the timeout
        struct Msg { hipIpcMemHandle_t h; int64_t cap; int64_t wgs; } m{mine, cap, c->peer_wgs}, fp{}, fn{};
        if (peer_swap_bytes(c, &m, &fp, &fn, (int)sizeof(Msg), prev, next)) return fail("");
        if ((prev >= 0 && fp.cap != cap) || (next >= 0 && fn.cap != cap))
            return fail("peer transport: neighbours disagree on the mailbox size");
        if ((prev >= 0 && fp.wgs != c->peer_wgs) || (next >= 0 && fn.wgs != c->peer_wgs))
            return fail("peer transport: neighbours use different exchange workgroup counts "
                        "(poms_comm_set_peer wgs / POMS_PEER_WGS must be equal on every rank)");
        if (prev >= 0) {
            if (hipIpcOpenMemHandle(reinterpret_cast<void**>(&np), fp.h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
                return fail("peer transport: hipIpcOpenMemHandle of the previous rank's mailboxes failed");
            pi = true;
        }
        if (next >= 0) {
            if (hipIpcOpenMemHandle(reinterpret_cast<void**>(&nn), fn.h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
                return fail("peer transport: hipIpcOpenMemHandle of the next rank's mailboxes failed");
            ni = true;
        }
    }
    if (old_prev_ipc && old_prev) (void)hipIpcCloseMemHandle(old_prev);
    if (old_next_ipc && old_next && old_next != old_prev) (void)hipIpcCloseMemHandle(old_next);
    if (old) (void)hipFree(old);
    c->pblk = blk;
    c->pprev = np;
    c->pnext = nn;
    c->pprev_ipc = pi;
    c->pnext_ipc = ni;
    c->peer_cap = cap;
    c->peer_prev = prev;
    c->peer_next = next;
    c->peer_fine = fine;
    return 0;
}

// The argument block of one exchange of `data` (mailboxes built if needed).
static int peer_fill(poms_comm* c, double* data, int64_t plane_elems, int64_t n_local, int pad, int width, int prev,
                     int next, hipStream_t st, PeerArgs& a) {
    const int64_t cnt = (int64_t)width * plane_elems;
    if (peer_ensure(c, cnt, prev, next, st)) return 1;
    a.send_lo = data + (int64_t)pad * plane_elems;
    a.send_hi = data + (int64_t)(pad + n_local - width) * plane_elems;
    a.ghost_lo = data + (int64_t)(pad - width) * plane_elems;
    a.ghost_hi = data + (int64_t)(pad + n_local) * plane_elems;
    a.cnt = cnt;
    a.cap = c->peer_cap;
    auto* own = reinterpret_cast<uint64_t*>(c->pblk);
    a.own = own;
    a.out_lo = a.out_hi = nullptr;
    a.arr_lo = a.arr_hi = a.ack_lo = a.ack_hi = nullptr;
    const bool loop = c->nranks == 1;
    if (prev >= 0) {
        auto* pb = loop ? own : reinterpret_cast<uint64_t*>(c->pprev);
        a.out_lo = peer_side_host(pb, loop ? 0 : 1, a.cap);
        a.arr_lo = pb + (loop ? kArrPrev : kArrNext);
        a.ack_lo = pb + (loop ? kAckPrev : kAckNext);
    }
    if (next >= 0) {
        auto* nb = loop ? own : reinterpret_cast<uint64_t*>(c->pnext);
        a.out_hi = peer_side_host(nb, loop ? 1 : 0, a.cap);
        a.arr_hi = nb + (loop ? kArrNext : kArrPrev);
        a.ack_hi = nb + (loop ? kAckNext : kAckPrev);
    }
    a.G = c->peer_wgs;
    a.status = c->peer_status_dev;
    return 0;
}

// The exchange as its own kernel on the communication stream
static int peer_exchange(poms_comm* c, double* data, int64_t plane_elems, int64_t n_local, int pad, int width,
                         int prev, int next, hipStream_t st) {
    PeerArgs a;
    if (peer_fill(c, data, plane_elems, n_local, pad, width, prev, next, st, a)) return 1;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    POMS_HIP_CHECK(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone) c->peer_captured = true;
    POMS_HIP_CHECK(hipEventRecord(c->ev_in, st));
    POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_in, 0));
    hipLaunchKernelGGL(peer_exchange_kernel, dim3(a.G), dim3(256), 0, c->cs, a);
    POMS_HIP_CHECK(hipGetLastError());
    POMS_HIP_CHECK(hipEventRecord(c->ev_halo, c->cs));
    return 0;
}

extern "C" {

int poms_comm_destroy(poms_comm* c);
static int comm_common_init(poms_comm* c);

int poms_comm_unique_id(char* out, int len) {
    if (!out || len < (int)sizeof(ncclUniqueId)) { set_error("poms_comm_unique_id: buffer too small"); return 1; }
    ncclUniqueId id;
    POMS_NCCL_CHECK(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

int poms_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int poms_comm_create(int device, const char* id, int rank, int nranks, poms_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) { set_error("poms_comm_create: bad argument"); return 1; }
    POMS_HIP_CHECK(hipSetDevice(device));
    auto* c = new poms_comm();
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    if (nranks > 1 && !getenv_off("POMS_COMM_SHM")) shm_open_block(c, uid.internal, sizeof(uid.internal));
    // POMS_COMM_CTAS caps the workgroups of every RCCL kernel of this communicator
    // (ncclConfig_t::maxCTAs): an exchange overlapped with the interior launch takes
    // CUs from it, and the p-plane message needs few of them (tuning knob; unset =
    // RCCL's choice)
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    if (const char* e = getenv("POMS_COMM_CTAS")) {
        const int n = atoi(e);
        if (n > 0) cfg.minCTAs = cfg.maxCTAs = n;
    }
    ncclResult_t r = ncclCommInitRankConfig(&c->comm, nranks, uid, rank, &cfg);
    if (c->shm && c->shm_name[0]) shm_unlink(c->shm_name);   // every rank of the node has it mapped now
    if (r != ncclSuccess) {
        set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        if (c->shm) munmap(c->shm, c->shm_bytes);
        delete c;
        return 1;
    }
    if (nranks > 1 && !getenv_off("POMS_COMM_SHM")) {
        // use the block only if EVERY rank found all nranks in it (one node) -- the
        // same answer on every rank, so the host sums take one path everywhere; every
        // rank added itself before entering the collective init above
        const uint64_t present =
            c->shm ? reinterpret_cast<std::atomic<uint64_t>*>(&c->shm[2 * nranks].seq)->load(std::memory_order_acquire)
                   : 0;
        int local_all = present == (uint64_t)nranks ? 1 : 0;
        int* dflag = nullptr;
        bool ok = hipMalloc(reinterpret_cast<void**>(&dflag), sizeof(int)) == hipSuccess &&
                  hipMemcpy(dflag, &local_all, sizeof(int), hipMemcpyHostToDevice) == hipSuccess &&
                  ncclAllReduce(dflag, dflag, 1, ncclInt32, ncclMin, c->comm, nullptr) == ncclSuccess &&
                  hipMemcpy(&local_all, dflag, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess;
        if (dflag) (void)hipFree(dflag);
        if (!ok) {
            set_error("poms_comm_create: the shared-memory agreement all-reduce failed");
            if (c->shm) munmap(c->shm, c->shm_bytes);
            c->shm = nullptr;
            poms_comm_destroy(c);
            return 1;
        }
        if (!local_all && c->shm) {
            munmap(c->shm, c->shm_bytes);
            c->shm = nullptr;
        }
    }
    if (comm_common_init(c)) {
        poms_comm_destroy(c);
        return 1;
    }
    *out = c;
    return 0;
}

static int comm_common_init(poms_comm* c) {
    // The communication stream gets the highest priority: HIP then gives it a hardware
    // queue of its own.  A normal-priority stream may share the compute stream's
    // queue (GPU_MAX_HW_QUEUES = 4), and a shared queue runs the exchange between
    // the compute launches instead of beside them -- rocprofv3 showed every RCCL
    // kernel serialised with the interior launch it was meant to overlap
    // (profiles/r03/proxy/).
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&c->cs, hipStreamNonBlocking, greatest) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_red, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_bnd, hipEventDisableTiming) != hipSuccess) {
        set_error("poms_comm_create: stream / event creation failed");
        return 1;
    }
    bool ok = hipHostMalloc(reinterpret_cast<void**>(&c->ring), poms_comm::kRing * 2 * sizeof(double),
                            hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&c->dev_tmp), 2 * sizeof(double)) == hipSuccess;
    for (int i = 0; ok && i < poms_comm::kRing; ++i)
        ok = hipEventCreateWithFlags(&c->ring_ev[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        set_error("poms_comm_create: ring allocation failed");
        return 1;
    }
    return 0;
}

int poms_comm_create_host(int device, int rank, int nranks, poms_host_exchange_fn xchg,
                          poms_host_allreduce_fn ar, void* user, poms_comm** out) {
    if (!xchg || !ar || !out || nranks < 1 || rank < 0 || rank >= nranks) {
        set_error("poms_comm_create_host: bad argument");
        return 1;
    }
    POMS_HIP_CHECK(hipSetDevice(device));
    auto* c = new poms_comm();
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    c->host = true;
    c->xchg = xchg;
    c->ar = ar;
    c->user = user;
    if (comm_common_init(c)) {
        poms_comm_destroy(c);
        return 1;
    }
    *out = c;
    return 0;
}

// Host transport: attach the node-local shared-memory block named by `id` (id_len
// bytes, the same on every rank), so that host-read sums take shm_allsum exactly as
// on the RCCL path of a one-node run.  Collective: the all-reduce callback serves as
// the barrier after which every rank of the node has marked itself present, and
// then as the agreement that every rank found all the others (the same answer
// everywhere; otherwise the block is dropped and the sums keep the callback).
// Lets the gloo tests run shm_allsum and poms_comm_wait's shared-memory branch,
// which the 8-GPU RCCL run depends on (advisor / verdict, round 3).
int poms_comm_host_attach_shm(poms_comm* c, const char* id, int id_len, int* attached) {
    if (!c || !id || id_len < 1 || !attached) { set_error("poms_comm_host_attach_shm: bad argument"); return 1; }
    *attached = 0;
    if (!c->host) { set_error("poms_comm_host_attach_shm: not a host-transport communicator"); return 1; }
    if (c->nranks < 2 || c->shm) {
        *attached = c->shm ? 1 : 0;
        return 0;
    }
    shm_open_block(c, id, (size_t)id_len);
    double v[2] = {1.0, 0.0};
    if (c->ar(c->user, v, 1)) { set_error("host transport: all-reduce callback failed"); return 1; }
    if (c->shm && c->shm_name[0]) shm_unlink(c->shm_name);   // every rank of the node has it mapped now
    const uint64_t present =
        c->shm ? reinterpret_cast<std::atomic<uint64_t>*>(&c->shm[2 * c->nranks].seq)->load(std::memory_order_acquire)
               : 0;
    v[0] = present == (uint64_t)c->nranks ? 1.0 : 0.0;
    if (c->ar(c->user, v, 1)) { set_error("host transport: all-reduce callback failed"); return 1; }
    if (v[0] != (double)c->nranks) {
        if (c->shm) munmap(c->shm, c->shm_bytes);
        c->shm = nullptr;
        return 0;
    }
    *attached = 1;
    return 0;
}

int poms_comm_uses_shm(poms_comm* c, int* yes) {
    if (!c || !yes) { set_error("poms_comm_uses_shm: null argument"); return 1; }
    *yes = c->shm ? 1 : 0;
    return 0;
}

int poms_comm_is_host(poms_comm* c, int* yes) {
    if (!c || !yes) { set_error("poms_comm_is_host: null argument"); return 1; }
    *yes = c->host ? 1 : 0;
    return 0;
}

// host transport: in-place sum of `count` device doubles through the callback
static int host_allreduce(poms_comm* c, double* buf, int64_t count, hipStream_t st) {
    if (refuse_in_capture(st, "host transport all-reduce")) return 1;
    POMS_HIP_CHECK(hipStreamSynchronize(st));
    if (c->stage.size() < (size_t)count) c->stage.resize((size_t)count);
    POMS_HIP_CHECK(hipMemcpy(c->stage.data(), buf, count * sizeof(double), hipMemcpyDeviceToHost));
    if (c->ar(c->user, c->stage.data(), count)) { set_error("host transport: all-reduce callback failed"); return 1; }
    POMS_HIP_CHECK(hipMemcpy(buf, c->stage.data(), count * sizeof(double), hipMemcpyHostToDevice));
    return 0;
}

int poms_comm_destroy(poms_comm* c) {
    if (!c) return 0;
    if (c->cs) (void)hipStreamSynchronize(c->cs);
    peer_release(c);
    if (c->peer_status) (void)hipHostFree(c->peer_status);
    if (c->comm) ncclCommDestroy(c->comm);
    for (hipEvent_t e : {c->ev_in, c->ev_halo, c->ev_red, c->ev_bnd})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ring_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ring) (void)hipHostFree(c->ring);
    if (c->dev_tmp) (void)hipFree(c->dev_tmp);
    if (c->shm) munmap(c->shm, c->shm_bytes);
    if (c->cs) (void)hipStreamDestroy(c->cs);
    delete c;
    return 0;
}

int poms_comm_stream(poms_comm* c, void** stream) {
    if (!c || !stream) { set_error("poms_comm_stream: null argument"); return 1; }
    *stream = c->cs;
    return 0;
}

int poms_comm_set_peer(poms_comm* c, int enable, int wgs) {
    if (!c || wgs < 1 || wgs > kPeerMaxWgs) { set_error("poms_comm_set_peer: bad argument (wgs in 1..256)"); return 1; }
    if (c->peer_on && (!enable || wgs != c->peer_wgs)) {   // blocks are rebuilt at the next exchange
        if (c->pblk && c->peer_captured) {
            set_error("poms_comm_set_peer: an exchange was captured into a graph; its mailboxes cannot be released");
            return 1;
        }
        (void)hipStreamSynchronize(c->cs);
        peer_release(c);
    }
    c->peer_on = enable != 0;
    c->peer_wgs = wgs;
    return 0;
}

int poms_comm_peer_reserve(poms_comm* c, int64_t cnt, int prev, int next) {
    if (!c || cnt < 1) { set_error("poms_comm_peer_reserve: bad argument"); return 1; }
    if (!c->peer_on || (prev < 0 && next < 0)) return 0;
    return peer_ensure(c, cnt, prev, next, c->cs);
}

int poms_comm_check(poms_comm* c) {
    if (!c) { set_error("poms_comm_check: null communicator"); return 1; }
    return peer_check(c);
}

int poms_comm_peer_status(poms_comm* c, int* active, int* fine_grained, int* timed_out) {
    if (!c || !active || !fine_grained || !timed_out) { set_error("poms_comm_peer_status: null argument"); return 1; }
    *active = c->peer_on ? 1 : 0;
    *fine_grained = c->peer_fine ? 1 : 0;
    *timed_out = 0;
    if (c->pblk && c->peer_status) {
        if (refuse_in_capture(c->cs, "poms_comm_peer_status")) return 1;
        POMS_HIP_CHECK(hipStreamSynchronize(c->cs));
        *timed_out = __atomic_load_n(c->peer_status, __ATOMIC_ACQUIRE) != 0 ? 1 : 0;
    }
    return 0;
}

// Ghost exchange of an axis-0 slab: `data` points at plane 0 of the padded local
// array (the first ghost plane), planes are `plane_elems` doubles apart; the
// first / last `width` owned planes go to `prev` / `next` (-1: none) and their
// planes land in this rank's ghost planes.  Starts after the work already queued
// on `stream`; poms_halo_finish makes `stream` wait for it.
int poms_halo_start(poms_comm* c, double* data, int64_t plane_elems, int64_t n_local, int pad, int width,
                    int prev, int next, void* stream) {
    if (!c || !data || plane_elems <= 0 || width < 0 || width > pad || n_local < width) {
        set_error("poms_halo_start: bad argument");
        return 1;
    }
    if (width == 0 || (prev < 0 && next < 0)) return 0;
    if (c->host && !c->peer_on) {   // stage the boundary planes, exchange through the callback, copy back
        hipStream_t st = cstream(stream);
        if (refuse_in_capture(st, "host transport exchange")) return 1;
        POMS_HIP_CHECK(hipStreamSynchronize(st));
        const size_t cnt = (size_t)width * (size_t)plane_elems;
        if (c->stage.size() < 4 * cnt) c->stage.resize(4 * cnt);
        double *slo = c->stage.data(), *rlo = slo + cnt, *shi = rlo + cnt, *rhi = shi + cnt;
        if (prev >= 0)
            POMS_HIP_CHECK(hipMemcpy(slo, data + (int64_t)pad * plane_elems, cnt * 8, hipMemcpyDeviceToHost));
        if (next >= 0)
            POMS_HIP_CHECK(hipMemcpy(shi, data + (int64_t)(pad + n_local - width) * plane_elems, cnt * 8,
                                     hipMemcpyDeviceToHost));
        if (c->xchg(c->user, slo, rlo, shi, rhi, (int64_t)cnt, prev, next)) {
            set_error("host transport: exchange callback failed");
            return 1;
        }
        if (prev >= 0)
            POMS_HIP_CHECK(hipMemcpy(data + (int64_t)(pad - width) * plane_elems, rlo, cnt * 8, hipMemcpyHostToDevice));
        if (next >= 0)
            POMS_HIP_CHECK(hipMemcpy(data + (int64_t)(pad + n_local) * plane_elems, rhi, cnt * 8,
                                     hipMemcpyHostToDevice));
        POMS_HIP_CHECK(hipEventRecord(c->ev_halo, st));
        c->halo_on = st;
        return 0;
    }
    if (c->peer_on) {
        c->halo_on = c->cs;
        return peer_exchange(c, data, plane_elems, n_local, pad, width, prev, next, cstream(stream));
    }
    hipStream_t xs = rccl_stream(c, cstream(stream));
    if (xs != cstream(stream)) {
        POMS_HIP_CHECK(hipEventRecord(c->ev_in, cstream(stream)));
        POMS_HIP_CHECK(hipStreamWaitEvent(xs, c->ev_in, 0));
    }
    const size_t cnt = (size_t)width * (size_t)plane_elems;
    POMS_NCCL_CHECK(ncclGroupStart());
    if (prev >= 0) {
        POMS_NCCL_CHECK(ncclSend(data + (int64_t)pad * plane_elems, cnt, ncclDouble, prev, c->comm, xs));
        POMS_NCCL_CHECK(ncclRecv(data + (int64_t)(pad - width) * plane_elems, cnt, ncclDouble, prev, c->comm, xs));
    }
    if (next >= 0) {
        POMS_NCCL_CHECK(ncclSend(data + (int64_t)(pad + n_local - width) * plane_elems, cnt, ncclDouble, next,
                                 c->comm, xs));
        POMS_NCCL_CHECK(ncclRecv(data + (int64_t)(pad + n_local) * plane_elems, cnt, ncclDouble, next, c->comm, xs));
    }
    POMS_NCCL_CHECK(ncclGroupEnd());
    POMS_HIP_CHECK(hipEventRecord(c->ev_halo, xs));
    c->halo_on = xs;
    return 0;
}

int poms_halo_finish(poms_comm* c, void* stream) {
    if (!c) { set_error("poms_halo_finish: null communicator"); return 1; }
    POMS_HIP_CHECK(hipStreamWaitEvent(cstream(stream), c->ev_halo, 0));
    return 0;
}

// In-place sum over the ranks of `count` doubles, after the work queued on
// `stream`.  wait_back: `stream` waits for the result (device_sum); otherwise the
// result is ready on the communication stream (poms_comm_stream) only, where a
// caller queues its device -> host copy (lazy norms: the next sweep never waits).
int poms_allreduce_sum(poms_comm* c, double* buf, int64_t count, void* stream, int wait_back) {
    if (!c || !buf || count < 0) { set_error("poms_allreduce_sum: bad argument"); return 1; }
    if (c->host) {   // synchronous; the result is then also ordered on the communication stream
        if (host_allreduce(c, buf, count, cstream(stream))) return 1;
        POMS_HIP_CHECK(hipEventRecord(c->ev_in, cstream(stream)));
        POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_in, 0));
        return 0;
    }
    hipStream_t xs = rccl_stream(c, cstream(stream));
    if (xs == cstream(stream)) {   // (captured: on the capturing stream, then ordered on the communication stream)
        POMS_NCCL_CHECK(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, c->comm, xs));
        if (!wait_back) {
            POMS_HIP_CHECK(hipEventRecord(c->ev_red, xs));
            POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_red, 0));
        }
        return 0;
    }
    POMS_HIP_CHECK(hipEventRecord(c->ev_in, cstream(stream)));
    POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_in, 0));
    POMS_NCCL_CHECK(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, c->comm, c->cs));
    if (wait_back) {
        POMS_HIP_CHECK(hipEventRecord(c->ev_red, c->cs));
        POMS_HIP_CHECK(hipStreamWaitEvent(cstream(stream), c->ev_red, 0));
    }
    return 0;
}

// Next ring slot (2 doubles of pinned, device-mapped host memory, armed unset) for
// a global sum only the host reads.  A slot is re-armed only after the launch that
// last wrote it is complete (its event): an abandoned launch may still write it.
int poms_comm_slot(poms_comm* c, double** dev_slot, int* ticket) {
    if (!c || !dev_slot || !ticket) { set_error("poms_comm_slot: null argument"); return 1; }
    const int t = c->ring_next;
    if (refuse_in_capture(c->cs, "poms_comm_slot")) return 1;
    c->ring_next = (t + 1) % poms_comm::kRing;
    POMS_HIP_CHECK(hipEventSynchronize(c->ring_ev[t]));
    slot_arm(c->ring + 2 * t);
    slot_arm(c->ring + 2 * t + 1);
    c->ring_dst[t] = nullptr;
    c->ring_cnt[t] = 0;
    c->ring_done[t] = false;
    *dev_slot = c->ring + 2 * t;
    *ticket = t;
    return 0;
}

// The launch writing ring slot `ticket` (`count` <= 2 local sums) is queued on
// `stream`; poms_comm_wait(ticket) leaves the global sums in host_dst.
int poms_allreduce_to_host(poms_comm* c, int ticket, int count, double* host_dst, void* stream) {
    if (!c || !host_dst || ticket < 0 || ticket >= poms_comm::kRing || count < 1 || count > 2) {
        set_error("poms_allreduce_to_host: bad argument");
        return 1;
    }
    c->ring_dst[ticket] = host_dst;
    c->ring_cnt[ticket] = count;
    POMS_HIP_CHECK(hipEventRecord(c->ring_ev[ticket], cstream(stream)));
    return 0;
}

// Sum `cnt` doubles over the ranks, on the host: every rank publishes its values in
// the half of the block this round uses and adds all ranks' values in rank order
// (the same sum, bit for bit, on every rank).  Two halves suffice: a rank starts
// round s + 2 only after every rank published round s + 1, i.e. finished reading s.
static int shm_allsum(poms_comm* c, double* v, int cnt) {
    const uint64_t s = ++c->shm_seq;
    poms_comm::ShmSlot* half = c->shm + (s & 1) * c->nranks;
    poms_comm::ShmSlot& mine = half[c->rank];
    for (int i = 0; i < cnt; ++i) mine.v[i] = v[i];
    mine.seq.store(s, std::memory_order_release);
    double acc[2] = {0.0, 0.0};
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < c->nranks; ++r) {
        for (long n = 1; half[r].seq.load(std::memory_order_acquire) < s; ++n) {
            __builtin_ia32_pause();
            if ((n & 65535) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
                set_error("poms_comm_wait: a rank did not publish its sum within 120 s");
                return 1;
            }
        }
        for (int i = 0; i < cnt; ++i) acc[i] += half[r].v[i];
    }
    for (int i = 0; i < cnt; ++i) v[i] = acc[i];
    return 0;
}

int poms_comm_wait(poms_comm* c, int ticket) {
    if (!c || ticket < 0 || ticket >= poms_comm::kRing) { set_error("poms_comm_wait: bad argument"); return 1; }
    if (c->ring_done[ticket]) return 0;
    if (refuse_in_capture(c->cs, "poms_comm_wait")) return 1;
    const int cnt = c->ring_cnt[ticket];
    if (cnt < 1 || !c->ring_dst[ticket]) { set_error("poms_comm_wait: ticket has no pending sum"); return 1; }
    double* slot = c->ring + 2 * ticket;
    // spin on the slot (the reduction kernel's store lands ~1 us after it ends; an
    // event wake-up costs ~15 us), checking now and then that the launch is alive
    for (int i = 0; i < cnt; ++i) {
        for (long n = 1; slot_unset(slot + i); ++n) {
            __builtin_ia32_pause();
            if ((n & 4095) == 0 && hipEventQuery(c->ring_ev[ticket]) != hipErrorNotReady) {
                std::atomic_thread_fence(std::memory_order_seq_cst);
                if (slot_unset(slot + i)) { set_error("poms_comm_wait: the launch did not write its sum"); return 1; }
            }
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    // (the launch that wrote the slot read ghost planes of an exchange queued before it)
    if (peer_check(c)) return 1;
    double v[2] = {slot[0], cnt > 1 ? slot[1] : 0.0};
    if (c->nranks > 1) {
        if (c->shm) {   // one node (RCCL ranks, or a host transport with the block attached)
            if (shm_allsum(c, v, cnt)) return 1;
        } else if (c->host) {
            if (c->ar(c->user, v, cnt)) { set_error("host transport: all-reduce callback failed"); return 1; }
        } else {   // ranks on several nodes: through RCCL, synchronously
            POMS_HIP_CHECK(hipMemcpyAsync(c->dev_tmp, v, cnt * sizeof(double), hipMemcpyHostToDevice, c->cs));
            POMS_NCCL_CHECK(ncclAllReduce(c->dev_tmp, c->dev_tmp, (size_t)cnt, ncclDouble, ncclSum, c->comm, c->cs));
            POMS_HIP_CHECK(hipMemcpyAsync(v, c->dev_tmp, cnt * sizeof(double), hipMemcpyDeviceToHost, c->cs));
            POMS_HIP_CHECK(hipStreamSynchronize(c->cs));
        }
    }
    for (int i = 0; i < cnt; ++i) c->ring_dst[ticket][i] = v[i];
    c->ring_done[ticket] = true;
    return 0;
}

// One distributed operator call from a single host call: with `exchange` the
// ghost exchange of x starts, the interior planes [p, n_local - p) run meanwhile,
// then both p-plane boundaries in one launch after the exchange; otherwise one
// launch over all planes.  Reductions (as poms_op_run_reduce2) go to norm_dev /
// dot_dev, or -- lazy_count > 0 -- to a ring slot that is all-reduced and copied
// to host_dst on the communication stream (*ticket for poms_comm_wait; lazy
// order in the slot: [dot, norm] with both, else the one asked for).
int poms_op_run_dist(poms_op* op, poms_comm* c, int epilogue, double omega, const double* x, double* y,
                     const double* b, double* xplanes, int64_t plane_elems, int64_t n_local, int pad, int pmax,
                     int prev, int next, int exchange, int want_norm, int want_dot, double* norm_dev,
                     double* dot_dev, int lazy_count, double* host_dst, int* ticket, void* stream) {
    if (!op || !c) { set_error("poms_op_run_dist: null argument"); return 1; }
    double *nout = want_norm ? norm_dev : nullptr, *dout = want_dot ? dot_dev : nullptr;
    int t = -1;
    if (lazy_count > 0) {
        if (refuse_in_capture(cstream(stream), "poms_op_run_dist (lazy host-read sums)")) return 1;
        if (!host_dst || !ticket || lazy_count != (want_norm ? 1 : 0) + (want_dot ? 1 : 0)) {
            set_error("poms_op_run_dist: bad lazy request");
            return 1;
        }
        double* slot = nullptr;
        if (poms_comm_slot(c, &slot, &t)) return 1;
        dout = want_dot ? slot : nullptr;
        nout = want_norm ? slot + (want_dot ? 1 : 0) : nullptr;
    }
    // the split (interior | boundaries) schedule only when an exchange is actually
    // queued: with no neighbour (a one-rank loopback, a one-rank host transport)
    // poms_halo_start records no event, and the boundary launch on the communication
    // stream would not be ordered after the work on `stream` that wrote x
    // (advisor, round 3)
    const bool queued = exchange && pmax > 0 && (prev >= 0 || next >= 0);
    if (queued && n_local > 2 * pmax) {
        if (poms_halo_start(c, xplanes, plane_elems, n_local, pad, pmax, prev, next, stream)) return 1;
        // the boundary launch runs on the communication stream behind the exchange
        // (POMS_BOUNDARY_ON_CS=0: on the caller's stream after it, as before)
        struct Hooks {
            static int ghosts_on(void* a, void* s) {   // `s` waits for the exchange
                auto* c = static_cast<poms_comm*>(a);
                if (cstream(s) == c->halo_on) return 0;   // queued behind it already
                POMS_HIP_CHECK(hipStreamWaitEvent(cstream(s), c->ev_halo, 0));
                return 0;
            }
            static int join(void* a, void* from, void* to) {
                auto* c = static_cast<poms_comm*>(a);
                POMS_HIP_CHECK(hipEventRecord(c->ev_bnd, cstream(from)));
                POMS_HIP_CHECK(hipStreamWaitEvent(cstream(to), c->ev_bnd, 0));
                return 0;
            }
        };
        static const bool on_cs = !getenv_off("POMS_BOUNDARY_ON_CS");
        const SplitHooks h{on_cs ? static_cast<void*>(c->cs) : nullptr, &Hooks::ghosts_on, &Hooks::join, c};
        if (op_run_split(op, epilogue, omega, x, y, b, pmax, n_local - pmax, 0, pmax, n_local - pmax, n_local, nout,
                         dout, h, stream))
            return 1;
    } else {
        if (exchange) {
            if (poms_halo_start(c, xplanes, plane_elems, n_local, pad, pmax, prev, next, stream)) return 1;
            if (poms_halo_finish(c, stream)) return 1;
        }
        if (poms_op_run_reduce2(op, epilogue, omega, x, y, b, 0, n_local, 0, 0, nout, dout, 0, stream)) return 1;
    }
    if (lazy_count > 0) {
        if (poms_allreduce_to_host(c, t, lazy_count, host_dst, stream)) return 1;
        *ticket = t;
    }
    return 0;
}


}  // extern "C"
