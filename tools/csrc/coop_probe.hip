// Minimal cooperative-launch probe (diagnostic): does a process that made a
// hipLaunchCooperativeKernel call survive its own exit under rocprofv3?  No libgll, no torch,
// no static event pools -- separates the library from the profiler.
//
//   coop_probe [mode] [launches]      mode 0: ordinary launches, 1: cooperative launches,
//                                     2: cooperative, then hipDeviceReset() before exit
// Each launch: 256 workgroups of 256 threads, each writes its block index (no grid barrier,
// so a refused or partial residency cannot hang it).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void touch(int* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = int(blockIdx.x);
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 1;
    const int launches = argc > 2 ? atoi(argv[2]) : 4;
    int dev = 0, coop = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    int* d = nullptr;
    if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 2;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    for (int i = 0; i < launches; ++i) {
        if (mode == 0) {
            touch<<<256, 256, 0, s>>>(d);
        } else {
            void* args[] = {&d};
            const hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(touch),
                                                            dim3(256), dim3(256), args, 0, s);
            if (e != hipSuccess) {
                printf("cooperative launch failed: %s\n", hipGetErrorString(e));
                return 3;
            }
        }
    }
    (void)hipStreamSynchronize(s);
    int h[256];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += h[i] != i;
    (void)hipStreamDestroy(s);
    (void)hipFree(d);
    if (mode == 2) (void)hipDeviceReset();
    printf("coop_probe mode=%d launches=%d coop_attr=%d bad=%d\n", mode, launches, coop, bad);
    return bad ? 1 : 0;
}
