// Tile-row load rate of the Gram kernel's access pattern (diagnostic).  Each workgroup pulls
// the 2 x 64 rows of one upper-triangle 64-tile of X (n x d fp32, row stride ld floats) the
// way gram_bf3_kernel does -- slot q: rows 8q + (lane >> 3), 16 B piece lane & 7, 32-feature
// chunks split over the waves -- and only sums them.  Sweeps the row stride (channel
// camping at power-of-two strides?), waves per workgroup and chunks in flight per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NW, int INF>
__global__ __launch_bounds__(64 * NW) void tile_load(const float* __restrict__ X, int n, int d,
                                                    int ld, int T, float* __restrict__ out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, pc = lane & 7;
    int bi = 0, rem = blockIdx.x;
    while (rem >= T - bi) { rem -= T - bi; ++bi; }
    const int bj = bi + rem;
    const float* rp[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int R = 8 * q + (lane >> 3);
        const int row = R < 64 ? bi * 64 + R : bj * 64 + R - 64;
        rp[q] = X + size_t(row < n ? row : n - 1) * ld + 4 * pc;
    }
    const int nchunk = d / 32;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = w; c0 < nchunk; c0 += NW * INF) {
        f32x4 v[INF][16];
#pragma unroll
        for (int f = 0; f < INF; ++f) {
            const int c = c0 + NW * f < nchunk ? c0 + NW * f : c0;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[f][q] = *reinterpret_cast<const f32x4*>(rp[q] + 32 * c);
        }
#pragma unroll
        for (int f = 0; f < INF; ++f)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc += v[f][q];
    }
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 12345.678f) out[blockIdx.x] = s;   // keep the loads
}

template <int NW, int INF>
float run(const float* X, int n, int d, int ld, float* out) {
    const int T = (n + 63) / 64, tiles = T * (T + 1) / 2;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) tile_load<NW, INF><<<tiles, 64 * NW>>>(X, n, d, ld, T, out);
    hipEventRecord(a);
    const int reps = 50;
    for (int i = 0; i < reps; ++i) tile_load<NW, INF><<<tiles, 64 * NW>>>(X, n, d, ld, T, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = 1e3 * ms / reps;
    const double bytes = double(tiles) * 128 * d * 4;
    printf("n=%d d=%d ld=%d NW=%d INF=%d: %7.2f us/launch (back-to-back), %6.2f TB/s L2->CU, %5.1f GB/s per busy CU\n",
           n, d, ld, NW, INF, us, bytes / us / 1e6, bytes / us / 1e3 / (tiles < 256 ? tiles : 256));
    return us;
}

int main() {
    float *X, *out;
    const size_t maxe = size_t(8192) * 1056;
    hipMalloc(&X, maxe * 4);
    hipMalloc(&out, 1 << 20);
    std::vector<float> h(maxe, 0.5f);
    hipMemcpy(X, h.data(), maxe * 4, hipMemcpyHostToDevice);
    for (int ld : {512, 516, 544, 520}) {
        run<4, 2>(X, 1000, 512, ld, out);
        run<4, 4>(X, 1000, 512, ld, out);
        run<8, 2>(X, 1000, 512, ld, out);
        run<16, 1>(X, 1000, 512, ld, out);
    }
    for (int ld : {1024, 1028, 1056}) {
        run<4, 2>(X, 8192, 1024, ld, out);
        run<8, 2>(X, 8192, 1024, ld, out);
    }
    return 0;
}
