// launch_probe.hip -- host enqueue cost of one kernel launch by API form (diagnostic).
//
//   hipcc -O2 --offload-arch=gfx950 tools/csrc/launch_probe.hip -o tools/csrc/launch_probe
//
// Times N back-to-back launches of a trivial kernel on one stream (host time to enqueue, then
// the wall time once the stream has drained), for:
//   chevron     kernel<<<g, b, 0, s>>>(args)              small kernarg (3 pointers)
//   chevron200  the same with a 200-B kernarg (25 pointer/int arguments, like the CG kernels)
//   launch      hipLaunchKernel(fn, g, b, args, 0, s)
//   extlaunch   hipExtLaunchKernel(..., nullptr, nullptr, 0)  (the dispatch-packet event form)
//   module      hipModuleLaunchKernel on the hipFunction_t of the same kernel
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>

struct Big {
    const float* p[20];
    int k[10];
};

__global__ void tiny(float* a, const float* b, int n) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) a[0] = b[0];
}
__global__ void tiny_big(Big a) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && a.k[0] < 0) const_cast<float*>(a.p[0])[0] = 1.f;
}

template <typename F>
static void timeit(const char* name, F fn, hipStream_t s, int n = 2000) {
    for (int i = 0; i < 100; ++i) fn();
    (void)hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) fn();
    auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(s);
    auto t2 = std::chrono::steady_clock::now();
    const double enq = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
    const double wall = std::chrono::duration<double, std::micro>(t2 - t0).count() / n;
    printf("%-12s enqueue %6.2f us/launch   wall %6.2f us/launch\n", name, enq, wall);
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    float* a = nullptr;
    (void)hipMalloc(&a, 1024);
    const float* b = a;
    int n = 1;
    Big big{};
    for (int i = 0; i < 20; ++i) big.p[i] = a;
    timeit("chevron", [&] { tiny<<<256, 256, 0, s>>>(a, b, n); }, s);
    timeit("chevron200", [&] { tiny_big<<<256, 256, 0, s>>>(big); }, s);
    void* args[] = {&a, &b, &n};
    timeit("launch", [&] {
        (void)hipLaunchKernel(reinterpret_cast<const void*>(tiny), dim3(256), dim3(256), args, 0, s);
    }, s);
    timeit("extlaunch", [&] {
        (void)hipExtLaunchKernel(reinterpret_cast<const void*>(tiny), dim3(256), dim3(256), args, 0,
                                 s, nullptr, nullptr, 0);
    }, s);
    hipFunction_t f = nullptr;
    if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(tiny)) == hipSuccess && f) {
        timeit("module", [&] {
            (void)hipModuleLaunchKernel(f, 256, 1, 1, 256, 1, 1, 0, s, args, nullptr);
        }, s);
        struct {
            float* a;
            const float* b;
            int n;
        } kp{a, b, n};
        size_t sz = sizeof(kp);
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &kp, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                       HIP_LAUNCH_PARAM_END};
        timeit("module_buf", [&] {
            (void)hipModuleLaunchKernel(f, 256, 1, 1, 256, 1, 1, 0, s, nullptr, cfg);
        }, s);
    } else {
        printf("hipGetFuncBySymbol unavailable\n");
    }
    // default (null) stream for comparison
    timeit("chevron_null", [&] { tiny<<<256, 256, 0, 0>>>(a, b, n); }, 0);
    (void)hipFree(a);
    return 0;
}
