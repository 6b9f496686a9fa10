// Round 6: which part of an RCCL ghost exchange breaks hipGraph capture?  (round-5
// verdict item 4: the Python probe's control stage captured an empty graph, every stage
// used a one-rank self-send communicator, and the exchange was forked to a second
// stream through events.)  No torch here: capture is driven from the C API, every
// return code is checked and printed, and each stage runs in a process of its own
// (tools/r06/graph_probe.sh), so a crash names its stage and its last completed step.
//
//   stages: ar        in-place ncclAllReduce captured (one rank: a no-op, RCCL records
//                     nothing -- the round-5 control's empty graph)
//           ar_oop    out-of-place ncclAllReduce a -> b captured (the control: a copy)
//           p2p_eager grouped ncclSend / ncclRecv to self, no capture
//           p2p       the same captured directly on the capturing stream
//           p2p_fork  the same on a second stream forked / joined by events (the
//                     library's schedule: the exchange on the communication stream)
//           p2p_fork_prio  p2p_fork with the second stream at the highest priority (the
//                     library's communication stream: its own hardware queue)
//           p2p2 / p2p2_fork_prio  TWO send / receive pairs with the same peer (self) in
//                     one group, as the library's one-rank loopback queues them (its
//                     previous and next neighbour are both rank 0)
//           kern_fork the fork / join with a plain kernel (a -> b copy) on the second
//                     stream instead of RCCL (is the fork alone enough?)
//           send_only one ncclSend captured (no matching receive: expected to fail or hang
//                     -- not run by default)
//   mode:   global | relaxed | thread (hipStreamCaptureMode)
//
//   hipcc -O2 -std=c++17 tools/r06/graph_probe.cpp -o tools/r06/graph_probe.bin -L/opt/rocm/lib -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static void step(const char* what) {
    printf("  step: %s\n", what);
    fflush(stdout);
}
#define HK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("  FAIL %s -> %s (%d)\n", #x, hipGetErrorString(e_), (int)e_);                \
            fflush(stdout);                                                                     \
            return 2;                                                                           \
        }                                                                                       \
        step(#x);                                                                               \
    } while (0)
#define NK(x)                                                                                   \
    do {                                                                                        \
        ncclResult_t r_ = (x);                                                                  \
        if (r_ != ncclSuccess) {                                                                \
            printf("  FAIL %s -> %s (%d)\n", #x, ncclGetErrorString(r_), (int)r_);               \
            fflush(stdout);                                                                     \
            return 3;                                                                           \
        }                                                                                       \
        step(#x);                                                                               \
    } while (0)

__global__ void fill_k(double* p, int64_t n, double base) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = base + (double)i;
}

static int check(const double* d, int64_t n, double base, double scale, const char* what) {
    std::vector<double> h(n);
    if (hipMemcpy(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
        printf("  FAIL readback of %s\n", what);
        return 4;
    }
    for (int64_t i = 0; i < n; ++i)
        if (h[i] != scale * (base + (double)i)) {
            printf("  FAIL %s: element %lld = %.17g, expected %.17g\n", what, (long long)i, h[i], scale * (base + (double)i));
            return 5;
        }
    printf("  %s: %lld values ok\n", what, (long long)n);
    return 0;
}

static int graph_nodes(hipGraph_t g) {
    size_t n = 0;
    if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -1;
    return (int)n;
}

int main(int argc, char** argv) {
    const std::string stage = argc > 1 ? argv[1] : "ar";
    const std::string mode_s = argc > 2 ? argv[2] : "global";
    const int64_t n = argc > 3 ? atoll(argv[3]) : (1 << 20);   // doubles per message (8 MiB)
    const hipStreamCaptureMode mode = mode_s == "relaxed" ? hipStreamCaptureModeRelaxed
                                    : mode_s == "thread" ? hipStreamCaptureModeThreadLocal
                                                         : hipStreamCaptureModeGlobal;
    int ver = 0, rt = 0;
    ncclGetVersion(&ver);
    (void)hipRuntimeGetVersion(&rt);
    printf("stage %s, capture mode %s, %lld doubles, RCCL %d, HIP runtime %d\n", stage.c_str(), mode_s.c_str(),
           (long long)n, ver, rt);
    HK(hipSetDevice(0));
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    ncclComm_t comm;
    // PROBE_CONFIG=1: ncclCommInitRankConfig with the default config (the library's call)
    if (getenv("PROBE_CONFIG") && atoi(getenv("PROBE_CONFIG"))) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        NK(ncclCommInitRankConfig(&comm, 1, id, 0, &cfg));
    } else {
        NK(ncclCommInitRank(&comm, 1, id, 0));
    }
    // PROBE_OFFSET=k: the message buffers start k doubles into their allocations (the
    // library sends planes from inside a padded array: 8-B aligned sub-pointers)
    const int64_t off = getenv("PROBE_OFFSET") ? atoll(getenv("PROBE_OFFSET")) : 0;
    printf("  config %s, buffer offset %lld doubles\n", getenv("PROBE_CONFIG") ? getenv("PROBE_CONFIG") : "0", (long long)off);
    hipStream_t s, s2;
    HK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (stage == "p2p_fork_prio" || stage == "p2p2_fork_prio") {
        int least = 0, greatest = 0;
        HK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, greatest));
    } else {
        HK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    }
    hipEvent_t ev_fork, ev_join;
    HK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    HK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    double *a, *b, *a2, *b2;
    HK(hipMalloc(&a, (n + off) * sizeof(double)));
    HK(hipMalloc(&b, (n + off) * sizeof(double)));
    HK(hipMalloc(&a2, (n + off) * sizeof(double)));
    HK(hipMalloc(&b2, (n + off) * sizeof(double)));
    a += off;
    b += off;
    a2 += off;
    b2 += off;
    hipLaunchKernelGGL(fill_k, dim3((int)((n + 255) / 256)), dim3(256), 0, s, a2, n, 7.0);
    HK(hipGetLastError());
    const int nb = (int)((n + 255) / 256);
    hipLaunchKernelGGL(fill_k, dim3(nb), dim3(256), 0, s, a, n, 1.0);
    HK(hipGetLastError());
    HK(hipMemsetAsync(b, 0, n * sizeof(double), s));
    HK(hipStreamSynchronize(s));

    // the exchange under test, queued on `q` (send a -> self, receive into b)
    auto exchange = [&](hipStream_t q) -> int {
        NK(ncclGroupStart());
        NK(ncclSend(a, (size_t)n, ncclDouble, 0, comm, q));
        NK(ncclRecv(b, (size_t)n, ncclDouble, 0, comm, q));
        if (stage.rfind("p2p2", 0) == 0) {   // the second pair (the other neighbour side)
            NK(ncclSend(a2, (size_t)n, ncclDouble, 0, comm, q));
            NK(ncclRecv(b2, (size_t)n, ncclDouble, 0, comm, q));
        }
        NK(ncclGroupEnd());
        return 0;
    };
    int rc = 0;
    if (stage == "p2p_eager" || stage == "p2p2_eager") {
        if ((rc = exchange(s))) return rc;
        HK(hipStreamSynchronize(s));
        rc = check(b, n, 1.0, 1.0, "eager self-exchange");
        if (!rc && stage == "p2p2_eager") rc = check(b2, n, 7.0, 1.0, "eager second pair");
    } else {
        hipGraph_t g = nullptr;
        HK(hipStreamBeginCapture(s, mode));
        if (stage == "ar") {
            NK(ncclAllReduce(a, a, (size_t)n, ncclDouble, ncclSum, comm, s));
        } else if (stage == "ar_oop") {
            NK(ncclAllReduce(a, b, (size_t)n, ncclDouble, ncclSum, comm, s));
        } else if (stage == "p2p" || stage == "p2p2") {
            if ((rc = exchange(s))) return rc;
        } else if (stage == "p2p_fork" || stage == "p2p_fork_prio" || stage == "p2p2_fork_prio") {
            HK(hipEventRecord(ev_fork, s));
            HK(hipStreamWaitEvent(s2, ev_fork, 0));
            if ((rc = exchange(s2))) return rc;
            HK(hipEventRecord(ev_join, s2));
            HK(hipStreamWaitEvent(s, ev_join, 0));
        } else if (stage == "kern_fork") {
            HK(hipEventRecord(ev_fork, s));
            HK(hipStreamWaitEvent(s2, ev_fork, 0));
            HK(hipMemcpyAsync(b, a, n * sizeof(double), hipMemcpyDeviceToDevice, s2));
            HK(hipEventRecord(ev_join, s2));
            HK(hipStreamWaitEvent(s, ev_join, 0));
        } else if (stage == "send_only") {
            NK(ncclSend(a, (size_t)n, ncclDouble, 0, comm, s));
        } else {
            printf("unknown stage\n");
            return 1;
        }
        HK(hipStreamEndCapture(s, &g));
        const int nn = graph_nodes(g);
        printf("  captured graph: %d nodes\n", nn);
        if (nn <= 0) {
            printf("  FAIL: nothing was captured\n");
            return 6;
        }
        hipGraphExec_t ge = nullptr;
        HK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 3; ++r) {
            HK(hipGraphLaunch(ge, s));
            HK(hipStreamSynchronize(s));
        }
        if (stage == "ar") rc = check(a, n, 1.0, 1.0, "all-reduce (one rank: identity) x3");
        else if (stage == "ar_oop" || stage == "kern_fork") rc = check(b, n, 1.0, 1.0, "out-of-place all-reduce (one rank: a copy) x3");
        else rc = check(b, n, 1.0, 1.0, "captured self-exchange x3");
        if (!rc && stage.rfind("p2p2", 0) == 0) rc = check(b2, n, 7.0, 1.0, "second pair x3");
        HK(hipGraphExecDestroy(ge));
        HK(hipGraphDestroy(g));
    }
    NK(ncclCommDestroy(comm));
    printf("stage %s: %s\n", stage.c_str(), rc ? "FAILED" : "ok");
    return rc;
}
