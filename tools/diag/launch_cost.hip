// Host cost of the HIP calls a frame makes (launches, event records, stream waits), from one thread
// and from T threads at once on one device (each thread its own streams), to see what a device
// group's concurrent enqueue contends on.  Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/lc launch_cost.hip -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

struct Big {
    float v[256];  // 1 KB of kernel arguments (Chunk1Params-sized)
};

__global__ void k_small(int* p) {
    if (p && threadIdx.x == 1023) p[0] = 1;
}
__global__ void k_big(Big b, int* p) {
    if (p && threadIdx.x == 1023) p[0] = (int)b.v[3];
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t err_ = (x);                                                \
        if (err_ != hipSuccess) {                                           \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(err_));    \
            std::exit(1);                                                  \
        }                                                                  \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One "frame" worth of calls: 9 launches, 3 event records, 3 waits, on two streams.
static double frame_calls(hipStream_t a, hipStream_t b, hipEvent_t* ev, int mode, hipFunction_t fsmall) {
    const double t0 = now_us();
    Big big{};
    int* np = nullptr;
    for (int k = 0; k < 9; ++k) {
        if (mode == 0) {
            k_small<<<256, 256, 0, a>>>(np);
        } else if (mode == 1) {
            k_big<<<256, 256, 0, a>>>(big, np);
        } else {
            void* args[] = {&np};
            CK(hipModuleLaunchKernel(fsmall, 256, 1, 1, 256, 1, 1, 0, a, args, nullptr));
        }
        if (k == 6) {
            CK(hipEventRecord(ev[0], a));
            CK(hipStreamWaitEvent(b, ev[0], 0));
        }
    }
    CK(hipEventRecord(ev[1], a));
    CK(hipStreamWaitEvent(b, ev[1], 0));
    CK(hipEventRecord(ev[2], b));
    CK(hipStreamWaitEvent(a, ev[2], 0));
    return now_us() - t0;
}

int main(int argc, char** argv) {
    const int maxT = argc > 1 ? std::atoi(argv[1]) : 8;
    hipFunction_t fsmall;
    CK(hipGetFuncBySymbol(&fsmall, reinterpret_cast<const void*>(&k_small)));
    for (int mode = 0; mode < 3; ++mode) {
        for (int T : {1, 2, 4, maxT}) {
            std::vector<std::thread> th;
            std::vector<double> med(T);
            std::atomic<int> ready{0};
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    CK(hipSetDevice(0));
                    hipStream_t a, b;
                    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
                    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
                    hipEvent_t ev[3];
                    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
                    for (int w = 0; w < 20; ++w) frame_calls(a, b, ev, mode, fsmall);
                    CK(hipStreamSynchronize(a));
                    CK(hipStreamSynchronize(b));
                    ready.fetch_add(1);
                    while (ready.load() < T) {
                    }
                    std::vector<double> v;
                    for (int r = 0; r < 200; ++r) {
                        v.push_back(frame_calls(a, b, ev, mode, fsmall));
                        if (r % 8 == 7) {  // keep the queues short
                            CK(hipStreamSynchronize(a));
                            CK(hipStreamSynchronize(b));
                        }
                    }
                    std::sort(v.begin(), v.end());
                    med[t] = v[v.size() / 2];
                    CK(hipStreamSynchronize(a));
                    CK(hipStreamSynchronize(b));
                    for (auto& e : ev) CK(hipEventDestroy(e));
                    CK(hipStreamDestroy(a));
                    CK(hipStreamDestroy(b));
                });
            for (auto& x : th) x.join();
            double mx = 0, mean = 0;
            for (double m : med) {
                mx = std::max(mx, m);
                mean += m / T;
            }
            std::printf("%s threads %d: per frame (9 launches, 3 records, 3 waits) median %.1f us (max over threads %.1f)\n",
                        mode == 0 ? "<<<>>> 8 B args " : mode == 1 ? "<<<>>> 1 KB args" : "hipModuleLaunch ", T, mean, mx);
            std::fflush(stdout);
        }
    }
    return 0;
}
