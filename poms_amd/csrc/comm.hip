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
#include "../../include/poms_hip.h"

#include <rccl/rccl.h>

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
    // ring of device scalar slots for lazily read global sums (damped-Jacobi
    // norms): a launch reduces its partials into a slot, the slot is all-reduced
    // and copied to pinned host memory on cs, and the host waits on the slot's event
    static constexpr int kRing = 16;
    double* ring = nullptr;         // kRing x 2 doubles
    hipEvent_t ring_ev[kRing] = {};
    int ring_next = 0;
    // host transport (poms_comm_create_host): the same schedule with the data moved
    // by caller-supplied host callbacks (e.g. torch.distributed / gloo) instead of
    // RCCL -- every call synchronises the caller's stream, stages the planes or
    // scalars through host memory and runs the callback in line
    bool host = false;
    poms_host_exchange_fn xchg = nullptr;
    poms_host_allreduce_fn ar = nullptr;
    void* user = nullptr;
    std::vector<double> stage;      // 4 x width x plane_elems (send lo / recv lo / send hi / recv hi)
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
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        delete c;
        return 1;
    }
    if (comm_common_init(c)) {
        poms_comm_destroy(c);
        return 1;
    }
    *out = c;
    return 0;
}

static int comm_common_init(poms_comm* c) {
    if (hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_red, hipEventDisableTiming) != hipSuccess) {
        set_error("poms_comm_create: stream / event creation failed");
        return 1;
    }
    bool ok = hipMalloc(reinterpret_cast<void**>(&c->ring), poms_comm::kRing * 2 * sizeof(double)) == hipSuccess;
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

int poms_comm_is_host(poms_comm* c, int* yes) {
    if (!c || !yes) { set_error("poms_comm_is_host: null argument"); return 1; }
    *yes = c->host ? 1 : 0;
    return 0;
}

// host transport: in-place sum of `count` device doubles through the callback
static int host_allreduce(poms_comm* c, double* buf, int64_t count, hipStream_t st) {
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
    if (c->comm) ncclCommDestroy(c->comm);
    for (hipEvent_t e : {c->ev_in, c->ev_halo, c->ev_red})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ring_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ring) (void)hipFree(c->ring);
    if (c->cs) (void)hipStreamDestroy(c->cs);
    delete c;
    return 0;
}

int poms_comm_stream(poms_comm* c, void** stream) {
    if (!c || !stream) { set_error("poms_comm_stream: null argument"); return 1; }
    *stream = c->cs;
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
    if (c->host) {   // stage the boundary planes, exchange through the callback, copy back
        hipStream_t st = cstream(stream);
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
        return 0;
    }
    POMS_HIP_CHECK(hipEventRecord(c->ev_in, cstream(stream)));
    POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_in, 0));
    const size_t cnt = (size_t)width * (size_t)plane_elems;
    POMS_NCCL_CHECK(ncclGroupStart());
    if (prev >= 0) {
        POMS_NCCL_CHECK(ncclSend(data + (int64_t)pad * plane_elems, cnt, ncclDouble, prev, c->comm, c->cs));
        POMS_NCCL_CHECK(ncclRecv(data + (int64_t)(pad - width) * plane_elems, cnt, ncclDouble, prev, c->comm, c->cs));
    }
    if (next >= 0) {
        POMS_NCCL_CHECK(ncclSend(data + (int64_t)(pad + n_local - width) * plane_elems, cnt, ncclDouble, next,
                                 c->comm, c->cs));
        POMS_NCCL_CHECK(ncclRecv(data + (int64_t)(pad + n_local) * plane_elems, cnt, ncclDouble, next, c->comm,
                                 c->cs));
    }
    POMS_NCCL_CHECK(ncclGroupEnd());
    POMS_HIP_CHECK(hipEventRecord(c->ev_halo, c->cs));
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
    POMS_HIP_CHECK(hipEventRecord(c->ev_in, cstream(stream)));
    POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_in, 0));
    POMS_NCCL_CHECK(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, c->comm, c->cs));
    if (wait_back) {
        POMS_HIP_CHECK(hipEventRecord(c->ev_red, c->cs));
        POMS_HIP_CHECK(hipStreamWaitEvent(cstream(stream), c->ev_red, 0));
    }
    return 0;
}

// Next ring slot (2 device doubles) for a lazily read global sum; waits for the
// slot's previous use to finish first.
int poms_comm_slot(poms_comm* c, double** dev_slot, int* ticket) {
    if (!c || !dev_slot || !ticket) { set_error("poms_comm_slot: null argument"); return 1; }
    const int t = c->ring_next;
    c->ring_next = (t + 1) % poms_comm::kRing;
    POMS_HIP_CHECK(hipEventSynchronize(c->ring_ev[t]));
    *dev_slot = c->ring + 2 * t;
    *ticket = t;
    return 0;
}

// All-reduce `count` (<= 2) doubles of ring slot `ticket` in place and copy them
// to `host_dst` (pinned), both on the communication stream after the work queued
// on `stream`; poms_comm_wait(ticket) returns when host_dst holds the sums.
int poms_allreduce_to_host(poms_comm* c, int ticket, int count, double* host_dst, void* stream) {
    if (!c || !host_dst || ticket < 0 || ticket >= poms_comm::kRing || count < 1 || count > 2) {
        set_error("poms_allreduce_to_host: bad argument");
        return 1;
    }
    double* slot = c->ring + 2 * ticket;
    if (c->host) {   // synchronous: host_dst holds the sums on return
        if (host_allreduce(c, slot, count, cstream(stream))) return 1;
        POMS_HIP_CHECK(hipMemcpy(host_dst, slot, count * sizeof(double), hipMemcpyDeviceToHost));
        // the ticket's event on the communication stream, ordered after the caller's
        // stream, as on the RCCL path (work queued on poms_comm_stream after this call
        // is then ordered after the result)
        POMS_HIP_CHECK(hipEventRecord(c->ev_in, cstream(stream)));
        POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_in, 0));
        POMS_HIP_CHECK(hipEventRecord(c->ring_ev[ticket], c->cs));
        return 0;
    }
    POMS_HIP_CHECK(hipEventRecord(c->ev_in, cstream(stream)));
    POMS_HIP_CHECK(hipStreamWaitEvent(c->cs, c->ev_in, 0));
    POMS_NCCL_CHECK(ncclAllReduce(slot, slot, (size_t)count, ncclDouble, ncclSum, c->comm, c->cs));
    POMS_HIP_CHECK(hipMemcpyAsync(host_dst, slot, count * sizeof(double), hipMemcpyDeviceToHost, c->cs));
    POMS_HIP_CHECK(hipEventRecord(c->ring_ev[ticket], c->cs));
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
        if (!host_dst || !ticket || lazy_count != (want_norm ? 1 : 0) + (want_dot ? 1 : 0)) {
            set_error("poms_op_run_dist: bad lazy request");
            return 1;
        }
        double* slot = nullptr;
        if (poms_comm_slot(c, &slot, &t)) return 1;
        dout = want_dot ? slot : nullptr;
        nout = want_norm ? slot + (want_dot ? 1 : 0) : nullptr;
    }
    if (exchange && n_local > 2 * pmax) {
        if (poms_halo_start(c, xplanes, plane_elems, n_local, pad, pmax, prev, next, stream)) return 1;
        if (poms_op_run_reduce2(op, epilogue, omega, x, y, b, pmax, n_local - pmax, 0, 0, nout, dout, 0, stream))
            return 1;
        if (poms_halo_finish(c, stream)) return 1;
        if (poms_op_run_reduce2(op, epilogue, omega, x, y, b, 0, pmax, n_local - pmax, n_local, nout, dout, 1,
                                stream))
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

int poms_comm_wait(poms_comm* c, int ticket) {
    if (!c || ticket < 0 || ticket >= poms_comm::kRing) { set_error("poms_comm_wait: bad argument"); return 1; }
    POMS_HIP_CHECK(hipEventSynchronize(c->ring_ev[ticket]));
    return 0;
}

}  // extern "C"
