// Host cost of enqueuing kernels on one stream (no sync between launches): hipLaunchKernelGGL
// with small and large by-value arguments, and hipModuleLaunchKernel through a function handle
// from hipGetFuncBySymbol.  Empty kernels; the GPU drains at the end.
//   hipcc --offload-arch=gfx950 -O2 -o tools/diag/bin/launch_path tools/diag/launch_path.hip && tools/diag/bin/launch_path
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Small { int a; float* p; };
struct Big { float v[200]; float* p; int n; };  // ~ProjParams-sized (808 B)

__global__ void k_small(Small s) { if (s.a == 12345 && threadIdx.x == 0) s.p[0] = 1.0f; }
__global__ void k_big(Big b) { if (b.n == 12345 && threadIdx.x == 0) b.p[0] = b.v[3]; }

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    hipStream_t st;
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    float* d;
    CHK(hipMalloc(&d, 4));
    Small s{0, d};
    Big b{};
    b.p = d;
    const int N = 20000;
    auto run = [&](const char* name, auto&& f) -> int {
        for (int i = 0; i < 200; ++i) f();
        if (hipStreamSynchronize(st) != hipSuccess) return 1;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) f();
        const auto t1 = std::chrono::steady_clock::now();
        if (hipStreamSynchronize(st) != hipSuccess) return 1;
        const auto t2 = std::chrono::steady_clock::now();
        std::printf("%-34s enqueue %.2f us/launch, drained %.2f us/launch\n", name,
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                    std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
        return 0;
    };
    if (run("hipLaunchKernelGGL small args", [&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st, s); })) return 1;
    if (run("hipLaunchKernelGGL 808-B args", [&] { hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, st, b); })) return 1;
    hipFunction_t fs, fb;
    CHK(hipGetFuncBySymbol(&fs, reinterpret_cast<const void*>(k_small)));
    CHK(hipGetFuncBySymbol(&fb, reinterpret_cast<const void*>(k_big)));
    if (run("hipModuleLaunchKernel small args", [&] {
            size_t sz = sizeof(s);
            void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &s, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
            (void)hipModuleLaunchKernel(fs, 1, 1, 1, 64, 1, 1, 0, st, nullptr, cfg);
        })) return 1;
    if (run("hipModuleLaunchKernel 808-B args", [&] {
            size_t sz = sizeof(b);
            void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &b, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
            (void)hipModuleLaunchKernel(fb, 1, 1, 1, 64, 1, 1, 0, st, nullptr, cfg);
        })) return 1;
    hipEvent_t ev;
    CHK(hipEventCreateWithFlags(&ev, hipEventDisableSystemFence));
    if (run("hipEventRecord", [&] { (void)hipEventRecord(ev, st); })) return 1;
    hipStream_t st2;
    CHK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
    if (run("hipStreamWaitEvent (other stream)", [&] { (void)hipStreamWaitEvent(st2, ev, 0); })) return 1;
    CHK(hipStreamSynchronize(st2));
    CHK(hipFree(d));
    return 0;
}
