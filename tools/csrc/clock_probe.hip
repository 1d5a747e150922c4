// Shader clock vs the constant 100 MHz clock on one CU, cold and after a busy phase
// (diagnostic): is the engine clock boosted during short latency-bound kernels?
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned long long* out, int spins) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    float v = threadIdx.x;
    for (int i = 0; i < spins; ++i) v = v * 1.0000001f + 1e-7f;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = v > 1e30f;
    }
}

__global__ void busy(float* p, int spins) {
    float v = threadIdx.x;
    for (int i = 0; i < spins; ++i) v = v * 1.0000001f + 1e-7f;
    p[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

int main() {
    unsigned long long* d;
    float* buf;
    hipMalloc(&d, 64);
    hipMalloc(&buf, 1024 * 256 * 4);
    unsigned long long h[3];
    for (int rep = 0; rep < 3; ++rep) {
        for (int spins : {1000, 100000}) {
            probe<<<1, 64>>>(d, spins);
            hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
            printf("cold   spins=%6d: memtime %8llu ticks, realtime %6llu (x10ns) -> %.3f GHz (if memtime = sclk)\n",
                   spins, h[0], h[1], h[1] ? h[0] / (h[1] * 10.0) : 0.0);
        }
        busy<<<1024, 256>>>(buf, 200000);
        probe<<<1, 64>>>(d, 100000);
        hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
        printf("after busy spins=100000: memtime %8llu, realtime %6llu -> %.3f GHz\n", h[0], h[1],
               h[1] ? h[0] / (h[1] * 10.0) : 0.0);
    }
    return 0;
}
