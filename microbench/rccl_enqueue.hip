// Host cost of one C2 strong-scaling step's exchange on one GPU: a 1-rank RCCL communicator
// sending two 80 KB halos to itself (ncclGroupStart / 2 x ncclSend + 2 x ncclRecv /
// ncclGroupEnd -- the group vip_shard_run enqueues per frame at N > 1, 3840 x 7 rows x 3 B
// per direction), with the event record / stream wait pair around it, against the GPU time
// per step. At 8 GPUs a rank's filter launch is ~25 us, so an enqueue cost near that makes
// the step host-bound.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                     \
    do {                                                                          \
        auto e_ = (x);                                                            \
        if (e_ != 0) {                                                            \
            std::printf("%s failed: %d at line %d\n", #x, (int)e_, __LINE__);     \
            return 1;                                                             \
        }                                                                         \
    } while (0)

__global__ void spin(float* p, int n) {  // a stand-in launch of the filter's size class
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5f + 1.f;
}

int main() {
    const size_t bytes = 3840 * 7 * 3;
    int dev = 0;
    ncclComm_t comm;
    CK(ncclCommInitAll(&comm, 1, &dev));
    hipStream_t s, c;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
    hipEvent_t ev_in, ev_x, t0, t1;
    CK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_x, hipEventDisableTiming));
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    uint8_t *a, *b;
    float* f;
    CK(hipMalloc(&a, 4 * bytes));
    CK(hipMalloc(&b, 4 * bytes));
    CK(hipMalloc(&f, 1 << 20));
    int frames = 1;  // frames whose halos share one group (2 sends + 2 receives each)
    auto exchange = [&]() -> int {
        CK(hipEventRecord(ev_in, s));
        CK(hipStreamWaitEvent(c, ev_in, 0));
        CK(ncclGroupStart());
        for (int fr = 0; fr < frames; ++fr) {
            CK(ncclSend(a + 2 * fr * bytes, bytes, ncclUint8, 0, comm, c));
            CK(ncclRecv(b + 2 * fr * bytes, bytes, ncclUint8, 0, comm, c));
            CK(ncclSend(a + (2 * fr + 1) * bytes, bytes, ncclUint8, 0, comm, c));
            CK(ncclRecv(b + (2 * fr + 1) * bytes, bytes, ncclUint8, 0, comm, c));
        }
        CK(ncclGroupEnd());
        CK(hipEventRecord(ev_x, c));
        CK(hipStreamWaitEvent(s, ev_x, 0));
        return 0;
    };
    for (int mode = 0; mode < 3; ++mode) {  // 0: exchange + launch, 1: exchange only, 2: launch only
        for (int w = 0; w < 50; ++w) {
            if (mode != 2 && exchange()) return 1;
            if (mode != 1) hipLaunchKernelGGL(spin, dim3(256), dim3(1024), 0, s, f, 1 << 18);
        }
        CK(hipStreamSynchronize(s));
        const int n = 2000;
        double host_us = 0;
        CK(hipEventRecord(t0, s));
        for (int i = 0; i < n; ++i) {
            const auto h0 = std::chrono::steady_clock::now();
            if (mode != 2 && exchange()) return 1;
            if (mode != 1) hipLaunchKernelGGL(spin, dim3(256), dim3(1024), 0, s, f, 1 << 18);
            host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
        }
        CK(hipEventRecord(t1, s));
        CK(hipEventSynchronize(t1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t0, t1));
        const char* name[3] = {"exchange (4 p2p ops, events) + launch", "exchange only", "launch only"};
        std::printf("%-40s host enqueue %.2f us per step, device %.2f us per step\n", name[mode], host_us / n,
                    ms * 1e3 / n);
    }
    for (frames = 2; frames <= 4; frames *= 2) {  // one group for several frames' halos
        for (int w = 0; w < 50; ++w)
            if (exchange()) return 1;
        CK(hipStreamSynchronize(s));
        const int n = 1000;
        double host_us = 0;
        CK(hipEventRecord(t0, s));
        for (int i = 0; i < n; ++i) {
            const auto h0 = std::chrono::steady_clock::now();
            if (exchange()) return 1;
            host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
        }
        CK(hipEventRecord(t1, s));
        CK(hipEventSynchronize(t1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t0, t1));
        std::printf("one group for %d frames' halos (%d ops)     host enqueue %.2f us per group, device %.2f us per group\n",
                    frames, 4 * frames, host_us / n, ms * 1e3 / n);
    }
    frames = 1;
    // the same step captured once into a hipGraph (exchange on the joined communication
    // stream, then the launch) and replayed: host cost of hipGraphLaunch per step
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        if (exchange()) return 1;
        hipLaunchKernelGGL(spin, dim3(256), dim3(1024), 0, s, f, 1 << 18);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 50; ++w) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemset(b, 0, 2 * bytes));
        CK(hipMemset(a, 7, 2 * bytes));
        const int n = 2000;
        double host_us = 0;
        CK(hipEventRecord(t0, s));
        for (int i = 0; i < n; ++i) {
            const auto h0 = std::chrono::steady_clock::now();
            CK(hipGraphLaunch(ge, s));
            host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
        }
        CK(hipEventRecord(t1, s));
        CK(hipEventSynchronize(t1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t0, t1));
        static uint8_t hb[2 * 3840 * 7 * 3];
        CK(hipMemcpy(hb, b, 2 * bytes, hipMemcpyDeviceToHost));
        int bad = 0;
        for (size_t i = 0; i < 2 * bytes; ++i) bad += hb[i] != 7;
        std::printf("%-40s host enqueue %.2f us per step, device %.2f us per step, halo bytes wrong: %d\n",
                    "graph replay (exchange + launch)", host_us / n, ms * 1e3 / n, bad);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    ncclCommDestroy(comm);
    return 0;
}
