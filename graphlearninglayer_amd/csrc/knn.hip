// knn.hip -- exact brute-force kNN for the GLL graph (replaces the annoy search of
// graphlearning.weightmatrix.knnsearch, /root/reference/GLL.py:183).
//
//  K1a gram_lds_kernel  D2 = |x_i|^2 + |x_j|^2 - 2 X X^T on fp32 MFMA (v_mfma_f32_32x32x2_f32),
//                       upper-triangle 64x64 tiles only (mirrored writes), split-K over two
//                       wave groups, LDS-staged double-buffered k-chunks, row norms from the
//                       same operands.
//  K1b knn_select_kernel one wave per row:
//                       1. per-lane sorted candidate lists over the D2 row (16-B loads);
//                       2. a 64-lane merge to kc = K-1+margin candidates, one DPP arg-min of
//                          the packed (d2, index) key per round;
//                       3. exact re-ranking with d^2 = sum_k (x_ik - x_jk)^2, eight candidates
//                          at a time (8-lane groups, DPP group sums) -- bitwise symmetric in
//                          (i, j) because both orders run the same lane mapping;
//                       4. the K-1 nearest by (exact d^2, index); self forced to rank 0 with
//                          distance 0 (the stand-in contract of SURVEY.md §8c);
//                       5. every valid pair (i -> j) is pushed onto j's reverse list (or the
//                          overflow list), which is how the symmetric union of GLL.py:197 is
//                          built without an n x n structure or a prefix sum.
#include <limits.h>

#include <type_traits>

#include "gll_internal.h"

namespace gll {

GLL_TRACE_UNIT(knn)

// --------------------------------------------------------------------------------------
// K1a: symmetric Gram tile.  D2 is symmetric, so only tiles bi <= bj are computed and the
// off-diagonal ones are written in both orientations.  Small problems have fewer tiles than
// CUs, so the feature dimension is split over KS workgroups per tile (gram_splits): each
// writes a partial plane  |a_i|^2_s + |b_j|^2_s - 2 <a_i, b_j>_s  over its slice s, and the
// select kernel adds the planes in a fixed order -- no inter-workgroup synchronisation.
//
// 512 threads = 8 waves: wave (kh, qd) owns the 32x32 quadrant qd of the 64x64 tile and the
// k-half kh of every 64-deep chunk (split-K inside the workgroup, halves combined in LDS in a
// fixed order).  Operands stream through a register ring of NCH chunks: chunk c of the next
// super-chunk is loaded into ring slot c right after slot c went to LDS, so a load has
// NCH-1 chunks of MFMA work to hide behind; LDS is double-buffered per chunk.
// --------------------------------------------------------------------------------------
// k per LDS chunk: GK = 64 or 128 (template); rows padded to GK + 4 floats (conflict-free
// ds_read_b128).  128-deep chunks halve the barriers per tile (one LDS turnaround each).
constexpr int kGK = 64;

// 16 MFMAs over 32 k: lane (r, h) holds A[r][8u + 4h + t], B[c=r][8u + 4h + t].  Two
// independent accumulator chains (alternate u) -- with 2 waves per SIMD that keeps four
// chains in flight per SIMD, what the fp32 MFMA needs to issue every 64 cycles.
__device__ __forceinline__ void gram_chunk_mfma(const f32x4 (&a)[4], const f32x4 (&b)[4],
                                                f32x16 (&acc)[2], float& sa, float& sb) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        sa += a[u].x * a[u].x + a[u].y * a[u].y + a[u].z * a[u].z + a[u].w * a[u].w;
        sb += b[u].x * b[u].x + b[u].y * b[u].y + b[u].z * b[u].z + b[u].w * b[u].w;
        f32x16& c = acc[u & 1];
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].x, b[u].x, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].y, b[u].y, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].z, b[u].z, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].w, b[u].w, c, 0, 0, 0);
    }
}

template <bool VEC, int NCH, int GK>
__global__ __launch_bounds__(512) void gram_lds_kernel(const float* __restrict__ X, int n, int d,
                                                       int T, int KS, int kspan,
                                                       float* __restrict__ D2, int ld,
                                                       size_t plane,
                                                       int32_t* __restrict__ status,
                                                       int32_t* __restrict__ rev_cnt,
                                                       size_t xs, size_t wss) {
    GLL_TRACE_SCOPE(0);
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    constexpr int kGL = GK + 4;
    constexpr int CS = GK / 64;   // 64-column segments of a chunk row
    // stage[buf][A|B][64 rows][kGL]; the epilogue reuses the same storage
    __shared__ __attribute__((aligned(16))) float smem[2 * 2 * 64 * kGL];
    __shared__ float s_sq[2][64];
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wave = tid >> 6;
    const int kh = wave >> 2;             // k-half of every chunk
    const int qd = wave & 3;              // 32x32 quadrant of this wave
    const int r = lane & 31, h = lane >> 5;
    const int ks = blockIdx.x % KS;
    int bi = 0, rem = blockIdx.x / KS;
    while (rem >= T - bi) {
        rem -= T - bi;
        ++bi;
    }
    const int bj = bi + rem;
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = blockIdx.x * 512 + tid;
        if (g < GLL_ST_NWORDS) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 512) rev_cnt[q] = 0;
    }
    GLL_TRACE_PT(10);
#ifdef GLL_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0) g_trace[21] = __builtin_amdgcn_s_memtime();
#endif
    const int k_lo = ks * kspan;
    const int k_hi = min(d, k_lo + kspan);
    const int nsup = kspan / (GK * NCH);
    // loader role: thread t moves float4 column 4 (t & 15) of rows (t >> 4) and (t >> 4) + 32
    // of A and of B for every chunk
    const int lrow = tid >> 4, lcol = 4 * (tid & 15);
    const float* ga0 = X + size_t(min(bi * 64 + lrow, n - 1)) * d;
    const float* ga1 = X + size_t(min(bi * 64 + lrow + 32, n - 1)) * d;
    const float* gb0 = X + size_t(min(bj * 64 + lrow, n - 1)) * d;
    const float* gb1 = X + size_t(min(bj * 64 + lrow + 32, n - 1)) * d;
    f32x4 ring[NCH][4 * CS];
    auto gload = [&](int chunk, f32x4 (&v)[4 * CS]) {   // raw: masked when stored to LDS
#pragma unroll
        for (int cs = 0; cs < CS; ++cs) {
            const int k = k_lo + chunk * GK + cs * 64 + lcol;
            v[4 * cs + 0] = load4_raw<VEC>(ga0, k, k_hi);
            v[4 * cs + 1] = load4_raw<VEC>(ga1, k, k_hi);
            v[4 * cs + 2] = load4_raw<VEC>(gb0, k, k_hi);
            v[4 * cs + 3] = load4_raw<VEC>(gb1, k, k_hi);
        }
    };
    auto lstore = [&](int chunk, int buf, const f32x4 (&v)[4 * CS]) {
        float* A = smem + (buf * 2 + 0) * 64 * kGL;
        float* B = smem + (buf * 2 + 1) * 64 * kGL;
#pragma unroll
        for (int cs = 0; cs < CS; ++cs) {
            const int k = k_lo + chunk * GK + cs * 64 + lcol;
            const int col = cs * 64 + lcol;
            *reinterpret_cast<f32x4*>(A + lrow * kGL + col) = mask4<VEC>(v[4 * cs + 0], k, k_hi);
            *reinterpret_cast<f32x4*>(A + (lrow + 32) * kGL + col) = mask4<VEC>(v[4 * cs + 1], k, k_hi);
            *reinterpret_cast<f32x4*>(B + lrow * kGL + col) = mask4<VEC>(v[4 * cs + 2], k, k_hi);
            *reinterpret_cast<f32x4*>(B + (lrow + 32) * kGL + col) = mask4<VEC>(v[4 * cs + 3], k, k_hi);
        }
    };
    f32x16 acc2[2];
#pragma unroll
    for (int g = 0; g < 16; ++g) acc2[0][g] = acc2[1][g] = 0.f;
    float sa = 0.f, sb = 0.f;
    const int arow = (qd >> 1) * 32 + r, brow = (qd & 1) * 32 + r;
#pragma unroll
    for (int c = 0; c < NCH; ++c) gload(c, ring[c]);
    // one super-chunk: chunks straight from the ring.  Several: ring slot c is reloaded with
    // the next super-chunk's chunk c right after it went to LDS -- unconditionally (the last
    // super-chunk re-reads its own, clamped), so the outstanding-load count is the same on
    // every path and the compiler waits for exactly the slot it stores next.
    auto run_super = [&](int sc, auto reload) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int buf = (sc * NCH + c) & 1;
            lstore(sc * NCH + c, buf, ring[c]);
            if constexpr (decltype(reload)::value) gload(min(sc + 1, nsup - 1) * NCH + c, ring[c]);
            __syncthreads();
            if (sc == 0 && c == 0) GLL_TRACE_PT(15);
            // wave half kh takes k [kh GK/2, (kh+1) GK/2) of the chunk, 32 at a time
#pragma unroll
            for (int sub = 0; sub < CS; ++sub) {
                const int ko = kh * (GK / 2) + sub * 32 + 4 * h;
                const float* A = smem + (buf * 2 + 0) * 64 * kGL + arow * kGL + ko;
                const float* B = smem + (buf * 2 + 1) * 64 * kGL + brow * kGL + ko;
                f32x4 a[4], b[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    a[u] = *reinterpret_cast<const f32x4*>(A + 8 * u);
                    b[u] = *reinterpret_cast<const f32x4*>(B + 8 * u);
                }
                gram_chunk_mfma(a, b, acc2, sa, sb);
            }
        }
    };
    if (nsup == 1) {
        run_super(0, std::false_type{});
        GLL_TRACE_PT(11);
    } else {
        for (int sc = 0; sc < nsup; ++sc) run_super(sc, std::true_type{});
    }
    __syncthreads();
    GLL_TRACE_PT(12);
    f32x16 acc = acc2[0] + acc2[1];
    // combine the k-halves in a fixed order (half 0 + half 1) through LDS
    float* part = smem;                    // [4 quadrants][16][64]
    float* nrm = smem + 4 * 16 * 64;       // [2][4][64]
    if (kh == 1) {
#pragma unroll
        for (int g = 0; g < 16; ++g) part[(qd * 16 + g) * 64 + lane] = acc[g];
        nrm[(0 * 4 + qd) * 64 + lane] = sa;
        nrm[(1 * 4 + qd) * 64 + lane] = sb;
    }
    __syncthreads();
    if (kh == 0) {
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] += part[(qd * 16 + g) * 64 + lane];
        sa += nrm[(0 * 4 + qd) * 64 + lane];
        sb += nrm[(1 * 4 + qd) * 64 + lane];
        sa += __shfl_xor(sa, 32);   // the two k quarters of row r
        sb += __shfl_xor(sb, 32);
        if (h == 0) {
            if ((qd & 1) == 0) s_sq[0][(qd >> 1) * 32 + r] = sa;
            if ((qd >> 1) == 0) s_sq[1][(qd & 1) * 32 + r] = sb;
        }
    }
    __syncthreads();
    float* tile = smem + 8 * 16 * 64;      // [64][65], past part/nrm
    if (kh == 0) {
        const int tc = (qd & 1) * 32 + r;
        const float sqc = s_sq[1][tc];
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int tr = (qd >> 1) * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
            tile[tr * 65 + tc] = s_sq[0][tr] + sqc - 2.f * acc[g];
        }
    }
    __syncthreads();
    GLL_TRACE_PT(13);
    float* P = D2 + size_t(ks) * plane;
    const int cr = tid >> 4, cc = (tid & 15) * 4;
    for (int rr = cr; rr < 64; rr += 32) {
        const int i = bi * 64 + rr;
        if (i < n) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (bj * 64 + cc + t < n) P[size_t(i) * ld + bj * 64 + cc + t] = tile[rr * 65 + cc + t];
        }
        const int jr = bj * 64 + rr;
        if (bi != bj && jr < n) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (bi * 64 + cc + t < n) P[size_t(jr) * ld + bi * 64 + cc + t] = tile[(cc + t) * 65 + rr];
        }
    }
    GLL_TRACE_PT(14);
#ifdef GLL_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0) g_trace[22] = __builtin_amdgcn_s_memtime();
#endif
}

// --------------------------------------------------------------------------------------
// K1a'': 48 x 48 tiles for small problems, where 64-tiles leave CUs idle (n = 1000: 136 64-tiles
// vs 231 48-tiles for 256 CUs).  v_mfma_f32_16x16x4f32 (A[l&15][k=l>>4], B[k=l>>4][l&15];
// C col = l&15, row = 4(l>>4) + reg).  12 waves = 4 k-quarters of each 64-deep chunk x 3
// row blocks; a wave owns the 3 blocks of its row (3 independent accumulators).  Lane group
// g = l >> 4 takes k = 16 kq + 4 g + s at step s, so one ds_read_b128 feeds 4 MFMA steps.
// --------------------------------------------------------------------------------------
constexpr int k48L = kGK + 4;   // padded LDS row (floats)

template <bool VEC, int NCH>
__global__ __launch_bounds__(768) void gram48_kernel(const float* __restrict__ X, int n, int d,
                                                     int T, float* __restrict__ D2, int ld,
                                                     int32_t* __restrict__ status,
                                                     int32_t* __restrict__ rev_cnt,
                                                     size_t xs, size_t wss) {
    GLL_TRACE_SCOPE(3);
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    // stage[buf][A|B][48][k48L]; the epilogue reuses it: partials [4][3][3][4][64], norms
    // 2 x [4][3][64], tile [48][49] -- sized for the larger of the two
    constexpr int kStage = 2 * 2 * 48 * k48L;
    constexpr int kEpi = 4 * 3 * 3 * 256 + 2 * 4 * 3 * 64 + 48 * 49;
    __shared__ __attribute__((aligned(16))) float smem[kStage > kEpi ? kStage : kEpi];
    __shared__ float s_sq[2][48];
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wave = tid >> 6;
    const int kq = wave / 3, rb = wave % 3;
    const int lr = lane & 15, lg = lane >> 4;
    int bi = 0, rem = blockIdx.x;
    while (rem >= T - bi) {
        rem -= T - bi;
        ++bi;
    }
    const int bj = bi + rem;
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = blockIdx.x * 768 + tid;
        if (g < GLL_ST_NWORDS) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 768) rev_cnt[q] = 0;
    }
    // loader: thread t moves float4 column 4 (t & 15) of row t >> 4 (< 48) of A and of B
    const int lrow = tid >> 4, lcol = 4 * (tid & 15);
    const float* ga = X + size_t(min(bi * 48 + lrow, n - 1)) * d;
    const float* gb = X + size_t(min(bj * 48 + lrow, n - 1)) * d;
    const int nchunk = (d + kGK - 1) / kGK;
    const int nsup = (nchunk + NCH - 1) / NCH;
    f32x4 ring[NCH][2];
    auto gload = [&](int chunk, f32x4 (&v)[2]) {
        const int k = chunk * kGK + lcol;
        v[0] = load4_raw<VEC>(ga, k, d);
        v[1] = load4_raw<VEC>(gb, k, d);
    };
    auto lstore = [&](int chunk, int buf, const f32x4 (&v)[2]) {
        const int k = chunk * kGK + lcol;
        float* A = smem + (buf * 2 + 0) * 48 * k48L;
        float* B = smem + (buf * 2 + 1) * 48 * k48L;
        *reinterpret_cast<f32x4*>(A + lrow * k48L + lcol) = mask4<VEC>(v[0], k, d);
        *reinterpret_cast<f32x4*>(B + lrow * k48L + lcol) = mask4<VEC>(v[1], k, d);
    };
    f32x4 acc[3];
#pragma unroll
    for (int cb = 0; cb < 3; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    float sa = 0.f, sb[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) gload(min(c, nchunk - 1), ring[c]);
    for (int sc = 0; sc < nsup; ++sc) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int chunk = sc * NCH + c;
            if (chunk >= nchunk) break;   // uniform
            const int buf = chunk & 1;
            lstore(chunk, buf, ring[c]);
            gload(min(chunk + NCH, nchunk - 1), ring[c]);   // unconditional: static counts
            __syncthreads();
            const int ko = 16 * kq + 4 * lg;
            const float* A = smem + (buf * 2 + 0) * 48 * k48L;
            const float* B = smem + (buf * 2 + 1) * 48 * k48L;
            const f32x4 a = *reinterpret_cast<const f32x4*>(A + (16 * rb + lr) * k48L + ko);
            f32x4 b[3];
#pragma unroll
            for (int cb = 0; cb < 3; ++cb)
                b[cb] = *reinterpret_cast<const f32x4*>(B + (16 * cb + lr) * k48L + ko);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
#pragma unroll
                for (int cb = 0; cb < 3; ++cb)
                    acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[cb][t], acc[cb], 0, 0, 0);
            }
            sa += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
#pragma unroll
            for (int cb = 0; cb < 3; ++cb)
                sb[cb] += b[cb].x * b[cb].x + b[cb].y * b[cb].y + b[cb].z * b[cb].z + b[cb].w * b[cb].w;
        }
    }
    __syncthreads();
    // combine the k-quarters in a fixed order through LDS
    float* part = smem;                     // [kq][rb][cb][4][64]
    float* nA = smem + 4 * 3 * 3 * 256;     // [kq][rb][64]
    float* nB = nA + 4 * 3 * 64;            // [kq][cb][64]   (rb == 0 waves)
#pragma unroll
    for (int cb = 0; cb < 3; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) part[(((kq * 3 + rb) * 3 + cb) * 4 + g) * 64 + lane] = acc[cb][g];
    nA[(kq * 3 + rb) * 64 + lane] = sa;
    if (rb == 0) {
#pragma unroll
        for (int cb = 0; cb < 3; ++cb) nB[(kq * 3 + cb) * 64 + lane] = sb[cb];
    }
    __syncthreads();
    if (tid < 96) {   // row norms: 48 A rows, 48 B rows; sum over k-quarters and lane groups
        const int which = tid / 48, row = tid % 48, blk = row >> 4, r16 = row & 15;
        const float* src = which == 0 ? nA : nB;
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int g = 0; g < 4; ++g) s += src[(q * 3 + blk) * 64 + g * 16 + r16];
        s_sq[which][row] = s;
    }
    __syncthreads();
    float* tile = nB + 4 * 3 * 64;          // [48][49]
    if (kq == 0) {
#pragma unroll
        for (int cb = 0; cb < 3; ++cb) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float v = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) v += part[(((q * 3 + rb) * 3 + cb) * 4 + g) * 64 + lane];
                const int tr = 16 * rb + 4 * lg + g, tc = 16 * cb + lr;
                tile[tr * 49 + tc] = s_sq[0][tr] + s_sq[1][tc] - 2.f * v;
            }
        }
    }
    __syncthreads();
    if (tid < 48 * 12) {   // 48 rows x 12 groups of 4 columns, both orientations
        const int rr = tid / 12, cc = (tid % 12) * 4;
        const int i = bi * 48 + rr;
        if (i < n) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (bj * 48 + cc + t < n) D2[size_t(i) * ld + bj * 48 + cc + t] = tile[rr * 49 + cc + t];
        }
        const int jr = bj * 48 + rr;
        if (bi != bj && jr < n) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (bi * 48 + cc + t < n) D2[size_t(jr) * ld + bi * 48 + cc + t] = tile[(cc + t) * 49 + rr];
        }
    }
}

// --------------------------------------------------------------------------------------
// K1a (default): split-bf16 Gram on v_mfma_f32_32x32x16_bf16.  Each fp32 feature is split as
// x = hi + lo with hi = bf16(x), lo = bf16(x - hi), and x.y ~ hi.hi + hi.lo + lo.hi: three
// bf16 MFMAs at 16x the fp32 MFMA rate (5.3x fewer MFMA cycles than v_mfma_f32_32x32x2_f32).
// The dropped terms are <= 2^-16 |x_k y_k| each (~1e-6 on the d^2 of unit rows at d = 512,
// against ~1e-7 for fp32); D2 only nominates the K-1+margin candidates that the select
// kernel re-ranks with exact fp32 difference-form distances, so the kNN result keeps the
// fp32 exactness contract.  Row norms come from the fp32 values.
//
// 64 x 64 tile per workgroup (upper triangle, mirrored writes), 16 waves.  What bounds a
// tile at small n is how fast one CU pulls its 2 x 64 rows (256 KiB at d = 512) out of L2,
// which needs many loads in flight: tools/csrc/load_probe.hip measured 6.9 us for the tile
// loads with 4 waves x 2 chunks in flight and 4.0 us with 16 waves x 1 chunk.  So:
//   - features go in phases of 256; in a phase wave w loads rows 16s + w (s = 0..7) of the
//     128 tile rows (0..63 = rows bi*64.., 64..127 = rows bj*64..), one 1 KiB row segment
//     per wave instruction (whole lines); two phases of loads are in flight per wave;
//   - each phase is split into hi / lo bf16 planes in LDS (2 x 128 x 256, row stride 264
//     bf16: conflict-free ds_read_b128 fragment reads), one barrier, then wave (qd, kq)
//     multiplies quadrant qd of the tile over feature quarter kq of the phase (4 k-steps x 3
//     MFMAs into one 32 x 32 accumulator);
//   - the 4 feature-quarter partials of each quadrant are summed in LDS in a fixed order.
// --------------------------------------------------------------------------------------
// XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs (block b runs on XCD
// b % 8, MI355X_MICROARCH.md), so block b takes tile (b % 8) * ceil-share + b / 8: each XCD
// works through a contiguous run of the row-major upper-triangle tile list -- a band of row
// blocks bi whose rows stay in that XCD's L2 -- instead of every XCD touching every row.
// (Measured neutral at NS, B = 64 and stress, tools/ab_flags.py: the tile loads are bound by
// per-CU issue, not by L2 misses.)
__device__ __forceinline__ int xcd_tile(int b, int nt) {
    const int x = b & 7, q = b >> 3;
    const int per = nt >> 3, extra = nt & 7;   // the first `extra` XCDs take one tile more
    return x * per + (x < extra ? x : extra) + q;
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int kBP = 256;            // features per phase
constexpr int kBS = kBP + 8;        // LDS plane row stride (bf16)

// Epilogue of the 64-tile split-bf16 Gram: row norms (wave sums of the per-slot squares),
// the 4 feature-quarter partials of each quadrant summed in LDS in a fixed order,
// D2 = |a_i|^2 + |b_j|^2 - 2 <a_i, b_j> staged as a [64][65] tile, then the direct and mirrored
// stores (a diagonal tile takes the upper triangle for both halves: D2 bitwise symmetric).
// nrm_of(t) reads norm t (0..63 rows bi, 64..127 rows bj) out of sqp[slot][wave]; Dz, when
// set, receives zeros at the direct positions (the unused plane of a split diagonal tile).
// The full-width stores are non-temporal: D2 is read once, by the select kernel on other XCDs,
// and streaming it out leaves less for the end-of-kernel L2 write-back (NS call 71.4 -> 70.5 us
// over 300 calls, alternating builds, tools/ab_flags.py --lib; on the 128-tile kernel the same
// change measured +0.6% at stress and -1.3% at B = 64, so that one keeps ordinary stores).
template <typename NF>
__device__ __forceinline__ void bf3_epilogue(const f32x16& acc, const float (&sq)[8], float* smem,
                                             float (*sqp)[16], float* nrm, NF nrm_of, int bi,
                                             int bj, int n, float* __restrict__ D2, int ld,
                                             float* __restrict__ Dz) {
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int qd = w & 3, kq = w >> 2;
    // row norms: slot s of wave w is tile row 16 s + w, its features spread over the wave
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const float t = wave_sum_dpp(sq[s]);
        if (lane == 0) sqp[s][w] = t;
    }
    __syncthreads();   // fragment reads done: the planes become partial / tile space
    // partial quadrant -> LDS part[kq][qd][32][33] (C layout: col = lane & 31,
    // row = (e&3) + 8(e>>2) + 4h)
    float* pw = smem + (kq * 4 + qd) * 32 * 33;
#pragma unroll
    for (int e = 0; e < 16; ++e) pw[((e & 3) + 8 * (e >> 2) + 4 * h) * 33 + r] = acc[e];
    if (tid < 128) nrm[tid] = nrm_of(tid);
    __syncthreads();
    // tile element (ti, tj..tj+3): sum of the 4 feature quarters, fixed order
    const int ti = tid >> 4, tj = 4 * (tid & 15);
    float v[4];
    {
        const int q = 2 * (ti >> 5) + (tj >> 5), rr = ti & 31;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int cc = (tj & 31) + e;
            float t = 0.f;
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) t += smem[(k4 * 4 + q) * 32 * 33 + rr * 33 + cc];
            v[e] = t;
        }
    }
    __syncthreads();
    float* tile = smem + 16 * 32 * 33;   // [64][65], past the partials
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[ti * 65 + tj + e] = nrm[ti] + nrm[64 + tj + e] - 2.f * v[e];
    __syncthreads();
    // direct orientation: row bi*64 + ti, columns bj*64 + tj .. +3; a diagonal tile takes the
    // upper triangle for both halves so D2 stays bitwise symmetric
    const int i = bi * 64 + ti;
    if (i < n) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int jj = tj + e;
            o[e] = (bi == bj && jj < ti) ? tile[jj * 65 + ti] : tile[ti * 65 + jj];
        }
        float* dst = D2 + size_t(i) * ld + bj * 64 + tj;
        float* dz = Dz ? Dz + size_t(i) * ld + bj * 64 + tj : nullptr;
        if (bj * 64 + tj + 4 <= n) {
            __builtin_nontemporal_store(f32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4*>(dst));
            if (dz) __builtin_nontemporal_store(f32x4{0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f32x4*>(dz));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (bj * 64 + tj + e < n) {
                    dst[e] = o[e];
                    if (dz) dz[e] = 0.f;
                }
        }
    }
    // mirrored orientation: row bj*64 + ti, columns bi*64 + tj .. +3 from the tile's column ti
    const int jr = bj * 64 + ti;
    if (bi != bj && jr < n) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = tile[(tj + e) * 65 + ti];
        float* dst = D2 + size_t(jr) * ld + bi * 64 + tj;
        if (bi * 64 + tj + 4 <= n) {
            __builtin_nontemporal_store(f32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4*>(dst));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (bi * 64 + tj + e < n) dst[e] = o[e];
        }
    }
}

template <bool VEC>
__global__ __launch_bounds__(1024) void gram_bf3_kernel(const float* __restrict__ X, int n, int d,
                                                        int T, float* __restrict__ D2, int ld,
                                                        int32_t* __restrict__ status,
                                                        int32_t* __restrict__ rev_cnt,
                                                        size_t xs, size_t wss) {
    GLL_TRACE_SCOPE(4);
    GLL_TRACE_PT(10);
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    // hi plane [128][kBS] then lo plane [128][kBS] (bf16); after the k loop the space holds
    // the partial quadrants [kq][qd][32][33] and then the finished tile [64][65] (floats)
    constexpr int kPlane = 128 * kBS;                                   // bf16 per plane
    __shared__ __attribute__((aligned(16))) __bf16 smem_h[2 * kPlane];
    __shared__ float sqp[8][16];                                        // [slot][wave]
    __shared__ float nrm[128];
    float* smem = reinterpret_cast<float*>(smem_h);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar row bases
    const int r = lane & 31, h = lane >> 5;
    int bi = 0, rem = xcd_tile(blockIdx.x, gridDim.x);
    while (rem >= T - bi) {
        rem -= T - bi;
        ++bi;
    }
    const int bj = bi + rem;
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = blockIdx.x * 1024 + tid;
        if (g < GLL_ST_NWORDS) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 1024) rev_cnt[q] = 0;
    }
    const int fo = 4 * lane;   // this lane's 4 features inside a phase
    auto slot_row = [&](int s) {   // row 16 s + w of the 128 tile rows; rows past n clamped
        const int R = 16 * s + w;
        const int row = (R < 64 ? bi * 64 + R : bj * 64 + R - 64);
        return X + size_t(row < n ? row : n - 1) * d;
    };
    const int nph = (d + kBP - 1) / kBP;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    float sq[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) sq[s] = 0.f;
    const int qd = w & 3, kq = w >> 2;              // MFMA role: quadrant, feature quarter
    const int qa = qd >> 1, qb = qd & 1;

    auto gload = [&](int ph, f32x4 (&v)[8]) {
        const int k = ph * kBP + fo;
#pragma unroll
        for (int s = 0; s < 8; ++s) v[s] = load4_raw<VEC>(slot_row(s), k, d);
    };
    auto phase = [&](int ph, const f32x4 (&v)[8]) {
        const int k = ph * kBP + fo;
        __syncthreads();   // the previous phase's fragment reads are done
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const f32x4 f = mask4<VEC>(v[s], k, d);
            sq[s] += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
            bf16x4 hv, lv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const __bf16 hb = static_cast<__bf16>(f[e]);
                hv[e] = hb;
                lv[e] = static_cast<__bf16>(f[e] - static_cast<float>(hb));
            }
            const int o = (16 * s + w) * kBS + fo;
            *reinterpret_cast<bf16x4*>(smem_h + o) = hv;
            *reinterpret_cast<bf16x4*>(smem_h + kPlane + o) = lv;
        }
        __syncthreads();
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int kk = 64 * kq + 16 * st + 8 * h;
            const int oa = (32 * qa + r) * kBS + kk, ob = (64 + 32 * qb + r) * kBS + kk;
            const bf16x8 ha = *reinterpret_cast<const bf16x8*>(smem_h + oa);
            const bf16x8 la = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + oa);
            const bf16x8 hb = *reinterpret_cast<const bf16x8*>(smem_h + ob);
            const bf16x8 lb = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + ob);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(la, hb, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, lb, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, hb, acc, 0, 0, 0);
        }
    };
    {
        f32x4 va[8], vb[8];
        gload(0, va);
        for (int ph = 0; ph < nph; ph += 2) {
            gload(ph + 1 < nph ? ph + 1 : ph, vb);   // unconditional: static vmcnt counts
#ifdef GLL_TRACE
            if (ph == 0) {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                GLL_TRACE_PT(15);
            }
#endif
            phase(ph, va);
            if (ph + 1 >= nph) break;
            gload(ph + 2 < nph ? ph + 2 : ph + 1, va);
            phase(ph + 1, vb);
        }
    }
    GLL_TRACE_PT(12);
    bf3_epilogue(acc, sq, smem, sqp, nrm, [&](int t) { return sqp[t >> 4][t & 15]; }, bi, bj, n,
                 D2, ld, nullptr);
    GLL_TRACE_PT(14);
}

// K1a' (one graph, n <= 1024, 256 < d <= 512): the same tile over HALF the features.  With
// T = ceil(n / 64) <= 16 the T (T + 1) / 2 upper-triangle tiles leave CUs idle (136 of 256 at
// NS) while each tile pulls 256 KiB through one CU, and that pull is what bounds the kernel
// (load_probe above).  Here each off-diagonal tile runs as two workgroups -- feature phase 0
// into plane 0, phase 1 into plane 1 -- and each diagonal tile as one workgroup that loads its
// 64 rows once for both phases (LDS rows 0..63: phase 0, rows 64..127: phase 1).  That is T^2
// workgroups with 128 KiB of loads each; the select kernel adds the two planes in a fixed order
// (NP = 2) and a diagonal tile writes zeros into plane 1.  Partial planes carry partial norms,
// |a|^2_s + |b|^2_s - 2 <a, b>_s, so the plane sum is D2.
template <bool VEC>
__global__ __launch_bounds__(1024) void gram_bf3s_kernel(const float* __restrict__ X, int n,
                                                         int d, int T, float* __restrict__ D2,
                                                         int ld, size_t plane,
                                                         int32_t* __restrict__ status,
                                                         int32_t* __restrict__ rev_cnt,
                                                         size_t xs, size_t wss) {
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    constexpr int kPlane = 128 * kBS;
    __shared__ __attribute__((aligned(16))) __bf16 smem_h[2 * kPlane];
    __shared__ float sqp[8][16];
    __shared__ float nrm[128];
    float* smem = reinterpret_cast<float*>(smem_h);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int b = xcd_tile(blockIdx.x, gridDim.x);
    const bool dg = b < T;   // block-uniform
    int bi = b, bj = b, half = 0;
    if (!dg) {   // strictly-upper tile (b - T) / 2, row-major; half = feature phase = plane
        int rem = (b - T) >> 1;
        half = (b - T) & 1;
        bi = 0;
        while (rem >= T - 1 - bi) {
            rem -= T - 1 - bi;
            ++bi;
        }
        bj = bi + 1 + rem;
    }
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = blockIdx.x * 1024 + tid;
        if (g < GLL_ST_NWORDS) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 1024) rev_cnt[q] = 0;
    }
    const int fo = 4 * lane;
    // slot s -> LDS row 16 s + w.  Off-diagonal: tile row 16 s + w (0..63 rows bi, 64..127
    // rows bj), features of phase `half`.  Diagonal: row bi*64 + 16 (s & 3) + w, phase s >> 2.
    f32x4 v[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int R = dg ? 16 * (s & 3) + w : 16 * s + w;
        const int row = R < 64 ? bi * 64 + R : bj * 64 + R - 64;
        const int k = (dg ? (s >> 2) : half) * kBP + fo;
        v[s] = load4_raw<VEC>(X + size_t(row < n ? row : n - 1) * d, k, d);
    }
    float sq[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int k = (dg ? (s >> 2) : half) * kBP + fo;
        const f32x4 f = mask4<VEC>(v[s], k, d);
        sq[s] = f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
        bf16x4 hv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const __bf16 hb = static_cast<__bf16>(f[e]);
            hv[e] = hb;
            lv[e] = static_cast<__bf16>(f[e] - static_cast<float>(hb));
        }
        const int o = (16 * s + w) * kBS + fo;
        *reinterpret_cast<bf16x4*>(smem_h + o) = hv;
        *reinterpret_cast<bf16x4*>(smem_h + kPlane + o) = lv;
    }
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    const int qd = w & 3, kq = w >> 2;
    const int qa = qd >> 1, qb = qd & 1;
    auto mfma3 = [&](int oa, int ob) {
        const bf16x8 ha = *reinterpret_cast<const bf16x8*>(smem_h + oa);
        const bf16x8 la = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + oa);
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(smem_h + ob);
        const bf16x8 lb = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + ob);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(la, hb, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, lb, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, hb, acc, 0, 0, 0);
    };
#pragma unroll
    for (int st = 0; st < 4; ++st) {
        const int kk = 64 * kq + 16 * st + 8 * h;
        if (dg) {   // both operands from the tile's own rows, phase 0 then phase 1
            mfma3((32 * qa + r) * kBS + kk, (32 * qb + r) * kBS + kk);
            mfma3((64 + 32 * qa + r) * kBS + kk, (64 + 32 * qb + r) * kBS + kk);
        } else {
            mfma3((32 * qa + r) * kBS + kk, (64 + 32 * qb + r) * kBS + kk);
        }
    }
    if (dg)   // norm of row t: its phase-0 slot plus its phase-1 slot, both halves the same rows
        bf3_epilogue(acc, sq, smem, sqp, nrm,
                     [&](int t) {
                         const int u = t & 63;
                         return sqp[u >> 4][u & 15] + sqp[(u >> 4) + 4][u & 15];
                     },
                     bi, bj, n, D2, ld, D2 + plane);
    else
        bf3_epilogue(acc, sq, smem, sqp, nrm, [&](int t) { return sqp[t >> 4][t & 15]; }, bi, bj,
                     n, D2 + size_t(half) * plane, ld, nullptr);
}

// --------------------------------------------------------------------------------------
// K1a (large problems and batches): split-bf16 Gram on 128 x 128 tiles.  With many tiles the
// kernel is bound by the tile rows every CU pulls out of L2 (2 x 64 rows per 64-tile: 4.3 GB
// at stress); a 128-tile halves those bytes per output.  16 waves, wave w owns the 32 x 32
// sub-tile (w >> 2, w & 3) over the WHOLE feature range, so there is no cross-wave reduction.
// Features go in phases of 128: thread t loads 4 features of row 32 s + (t >> 5) of the 256
// tile rows (0..127 = rows bi*128.., 128..255 = rows bj*128..) for slot s = 0..7 -- half a
// wave per 512-B row segment -- and splits them into hi / lo bf16 planes in LDS (row stride
// 136 bf16: conflict-free ds_read_b128); one barrier, then 8 k-steps x 3 MFMAs per wave.
// Off-diagonal tiles store straight from the accumulators in both orientations; diagonal
// tiles go through LDS so D2 stays bitwise symmetric (upper triangle mirrored).
// --------------------------------------------------------------------------------------
constexpr int kWP = 128;            // features per phase
constexpr int kWS = kWP + 8;        // LDS plane row stride (bf16)

template <bool VEC>
__global__ __launch_bounds__(1024) void gram_bf3w_kernel(const float* __restrict__ X, int n,
                                                         int d, int T, float* __restrict__ D2,
                                                         int ld, int32_t* __restrict__ status,
                                                         int32_t* __restrict__ rev_cnt,
                                                         size_t xs, size_t wss) {
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    constexpr int kPlane = 256 * kWS;                                   // bf16 per plane
    __shared__ __attribute__((aligned(16))) __bf16 smem_h[2 * kPlane];  // 136 KiB
    __shared__ float nrm[256];
    float* smem = reinterpret_cast<float*>(smem_h);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    int bi = 0, rem = xcd_tile(blockIdx.x, gridDim.x);
    while (rem >= T - bi) {
        rem -= T - bi;
        ++bi;
    }
    const int bj = bi + rem;
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = blockIdx.x * 1024 + tid;
        if (g < GLL_ST_NWORDS) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 1024) rev_cnt[q] = 0;
    }
    const int fo = 4 * (tid & 31);       // this thread's 4 features inside a phase
    const int rs = tid >> 5;             // its row inside a slot (0..31)
    auto slot_row = [&](int s) {         // tile row 32 s + rs; rows past n clamped
        const int R = 32 * s + rs;
        const int row = (R < 128 ? bi * 128 + R : bj * 128 + R - 128);
        return X + size_t(row < n ? row : n - 1) * d;
    };
    const int nph = (d + kWP - 1) / kWP;
    const int sa = w >> 2, sb = w & 3;   // this wave's 32 x 32 sub-tile
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    // row norms: slot q's half-wave sum is kept by lane q of that half-wave (one register)
    float sq = 0.f;

    auto gload = [&](int ph, f32x4 (&v)[8]) {
        const int k = ph * kWP + fo;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = load4_raw<VEC>(slot_row(q), k, d);
    };
    auto phase = [&](int ph, const f32x4 (&v)[8]) {
        const int k = ph * kWP + fo;
        __syncthreads();   // the previous phase's fragment reads are done
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const f32x4 f = mask4<VEC>(v[q], k, d);
            float t = f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
            t = dpp_add<0xB1, 0xf>(t);    // quad
            t = dpp_add<0x4E, 0xf>(t);
            t = dpp_add<0x141, 0xf>(t);   // half row (8)
            t = dpp_add<0x140, 0xf>(t);   // row (16)
            t += __shfl_xor(t, 16);       // the 32 lanes of the row segment
            sq += (lane & 31) == q ? t : 0.f;
            bf16x4 hv, lv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const __bf16 hb = static_cast<__bf16>(f[e]);
                hv[e] = hb;
                lv[e] = static_cast<__bf16>(f[e] - static_cast<float>(hb));
            }
            const int o = (32 * q + rs) * kWS + fo;
            *reinterpret_cast<bf16x4*>(smem_h + o) = hv;
            *reinterpret_cast<bf16x4*>(smem_h + kPlane + o) = lv;
        }
        __syncthreads();
#pragma unroll
        for (int st = 0; st < kWP / 16; ++st) {
            const int kk = 16 * st + 8 * h;
            const int oa = (32 * sa + r) * kWS + kk, ob = (128 + 32 * sb + r) * kWS + kk;
            const bf16x8 ha = *reinterpret_cast<const bf16x8*>(smem_h + oa);
            const bf16x8 la = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + oa);
            const bf16x8 hb = *reinterpret_cast<const bf16x8*>(smem_h + ob);
            const bf16x8 lb = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + ob);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(la, hb, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, lb, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, hb, acc, 0, 0, 0);
        }
    };
    {
        f32x4 va[8], vb[8];
        gload(0, va);
        for (int ph = 0; ph < nph; ph += 2) {
            gload(ph + 1 < nph ? ph + 1 : ph, vb);   // unconditional: static vmcnt counts
            phase(ph, va);
            if (ph + 1 >= nph) break;
            gload(ph + 2 < nph ? ph + 2 : ph + 1, va);
            phase(ph + 1, vb);
        }
    }
    if ((lane & 31) < 8) nrm[32 * (lane & 31) + rs] = sq;   // tile row 32 q + rs, q = lane
    __syncthreads();   // norms visible; fragment reads done (the planes may be reused)
    // C layout of 32x32: col = lane & 31, row = (e&3) + 8(e>>2) + 4h
    const int i0 = bi * 128 + 32 * sa, j0 = bj * 128 + 32 * sb;
    float dv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * h;
        dv[e] = nrm[32 * sa + rr] + nrm[128 + 32 * sb + r] - 2.f * acc[e];
    }
    if (bi != bj) {
        // direct orientation: element e is (i0 + rr, j0 + r) -- 32 lanes per 128-B row piece
        const int j = j0 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int i = i0 + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (i < n && j < n) D2[size_t(i) * ld + j] = dv[e];
        }
        // mirrored: row j0 + r, columns i0 + 8 g + 4 h .. +3 are registers 4 g .. 4 g + 3
        if (j < n) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int i = i0 + 8 * g + 4 * h;
                float* dst = D2 + size_t(j) * ld + i;
                if (i + 4 <= n) {
                    *reinterpret_cast<f32x4*>(dst) =
                        f32x4{dv[4 * g], dv[4 * g + 1], dv[4 * g + 2], dv[4 * g + 3]};
                } else {
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        if (i + t < n) dst[t] = dv[4 * g + t];
                }
            }
        }
    } else {
        // diagonal tile: stage [128][129] in LDS, store the upper triangle in both orientations
        float* tile = smem;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int rr = 32 * sa + (e & 3) + 8 * (e >> 2) + 4 * h;
            tile[rr * 129 + 32 * sb + r] = dv[e];
        }
        __syncthreads();
        for (int q = tid; q < 128 * 128; q += 1024) {
            const int ti = q >> 7, tj = q & 127;
            const int i = bi * 128 + ti, j = bi * 128 + tj;
            if (i < n && j < n) D2[size_t(i) * ld + j] = tj >= ti ? tile[ti * 129 + tj] : tile[tj * 129 + ti];
        }
    }
}

// --------------------------------------------------------------------------------------
// K1a': wide symmetric Gram tile for large problems (many tiles): 128 x 128 per workgroup, 4
// waves each owning a 64 x 64 sub-tile as 2 x 2 independent 32 x 32 MFMA accumulators (one
// A fragment feeds two MFMAs, four chains keep the MFMA pipe full from one wave per SIMD),
// 32-deep chunks through a register ring of NCH chunks into double-buffered LDS.
// --------------------------------------------------------------------------------------
constexpr int kWK = 32;           // k per chunk
constexpr int kWL = kWK + 4;      // padded LDS row (floats)

template <bool VEC, int NCH>
__global__ __launch_bounds__(256) void gram_wide_kernel(const float* __restrict__ X, int n, int d,
                                                        int T, float* __restrict__ D2, int ld,
                                                        int32_t* __restrict__ status,
                                                        int32_t* __restrict__ rev_cnt,
                                                        size_t xs, size_t wss) {
    GLL_TRACE_SCOPE(2);
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    // stage[buf][A|B][128][kWL]; the epilogue reuses it as tile[128][129]
    __shared__ __attribute__((aligned(16))) float smem[2 * 2 * 128 * kWL];
    __shared__ float s_sq[2][128];
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;   // 64-row / 64-column half of the tile
    const int r = lane & 31, h = lane >> 5;
    int bi = 0, rem = blockIdx.x;
    while (rem >= T - bi) {
        rem -= T - bi;
        ++bi;
    }
    const int bj = bi + rem;
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = blockIdx.x * 256 + tid;
        if (g < GLL_ST_NWORDS) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 256) rev_cnt[q] = 0;
    }
    // loader: thread t moves float4 column 4 (t & 7) of rows (t >> 3) + 32 s, s < 4, of A and B
    const int lrow = tid >> 3, lcol = 4 * (tid & 7);
    const float* ga[4];
    const float* gb[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
        ga[s4] = X + size_t(min(bi * 128 + lrow + 32 * s4, n - 1)) * d;
        gb[s4] = X + size_t(min(bj * 128 + lrow + 32 * s4, n - 1)) * d;
    }
    const int nchunk = (d + kWK - 1) / kWK;
    const int nsup = (nchunk + NCH - 1) / NCH;
    f32x4 ring[NCH][8];
    auto gload = [&](int chunk, f32x4 (&v)[8]) {   // raw: masked when stored to LDS
        const int k = chunk * kWK + lcol;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            v[s4] = load4_raw<VEC>(ga[s4], k, d);
            v[4 + s4] = load4_raw<VEC>(gb[s4], k, d);
        }
    };
    auto lstore = [&](int chunk, int buf, const f32x4 (&v)[8]) {
        const int k = chunk * kWK + lcol;
        float* A = smem + (buf * 2 + 0) * 128 * kWL;
        float* B = smem + (buf * 2 + 1) * 128 * kWL;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            *reinterpret_cast<f32x4*>(A + (lrow + 32 * s4) * kWL + lcol) = mask4<VEC>(v[s4], k, d);
            *reinterpret_cast<f32x4*>(B + (lrow + 32 * s4) * kWL + lcol) = mask4<VEC>(v[4 + s4], k, d);
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[i][j][g] = 0.f;
    float sa[2] = {0.f, 0.f}, sb[2] = {0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) gload(min(c, nchunk - 1), ring[c]);
    for (int sc = 0; sc < nsup; ++sc) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int chunk = sc * NCH + c;
            if (chunk >= nchunk) break;   // uniform
            const int buf = chunk & 1;
            lstore(chunk, buf, ring[c]);
            gload(min(chunk + NCH, nchunk - 1), ring[c]);   // unconditional: static counts
            __syncthreads();
            const float* A = smem + (buf * 2 + 0) * 128 * kWL;
            const float* B = smem + (buf * 2 + 1) * 128 * kWL;
            f32x4 a[2][4], b[2][4];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    a[i][u] = *reinterpret_cast<const f32x4*>(A + (64 * wr + 32 * i + r) * kWL + 4 * h + 8 * u);
                    b[i][u] = *reinterpret_cast<const f32x4*>(B + (64 * wc + 32 * i + r) * kWL + 4 * h + 8 * u);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][u][t], b[j][u][t],
                                                                           acc[i][j], 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    sa[i] += a[i][u].x * a[i][u].x + a[i][u].y * a[i][u].y +
                             a[i][u].z * a[i][u].z + a[i][u].w * a[i][u].w;
                    sb[i] += b[i][u].x * b[i][u].x + b[i][u].y * b[i][u].y +
                             b[i][u].z * b[i][u].z + b[i][u].w * b[i][u].w;
                }
            }
        }
    }
    __syncthreads();   // (one barrier per chunk suffices: buffer `buf` is rewritten only after
                       //  every wave has passed the next chunk's barrier)
    // row norms: the two k-quarters of a lane pair (xor 32), A rows from wc == 0 waves, B rows
    // (columns) from wr == 0 waves
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        sa[i] += __shfl_xor(sa[i], 32);
        sb[i] += __shfl_xor(sb[i], 32);
        if (h == 0 && wc == 0) s_sq[0][64 * wr + 32 * i + r] = sa[i];
        if (h == 0 && wr == 0) s_sq[1][64 * wc + 32 * i + r] = sb[i];
    }
    __syncthreads();
    float* tile = smem;   // [128][129]
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int tc = 64 * wc + 32 * j + r;
            const float sqc = s_sq[1][tc];
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int tr = 64 * wr + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
                tile[tr * 129 + tc] = s_sq[0][tr] + sqc - 2.f * acc[i][j][g];
            }
        }
    }
    __syncthreads();
    const int cr = tid >> 5, cc = (tid & 31) * 4;
    for (int rr = cr; rr < 128; rr += 8) {
        const int i = bi * 128 + rr;
        if (i < n) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (bj * 128 + cc + t < n) D2[size_t(i) * ld + bj * 128 + cc + t] = tile[rr * 129 + cc + t];
        }
        const int jr = bj * 128 + rr;
        if (bi != bj && jr < n) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (bi * 128 + cc + t < n) D2[size_t(jr) * ld + bi * 128 + cc + t] = tile[(cc + t) * 129 + rr];
        }
    }
}

// --------------------------------------------------------------------------------------
// K1b: per-row selection + exact re-rank + reverse scatter
// --------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t pack_key(float d2, int j) {
    // d2 >= 0 after the clamp, so its IEEE bits order like the value; index breaks ties
    return (uint64_t(__float_as_uint(d2 > 0.f ? d2 : 0.f)) << 32) | uint32_t(j);
}

template <int KC>
__device__ __forceinline__ void list_insert(uint64_t (&key)[KC], uint64_t v) {
    // precondition: v < key[KC-1]; ascending order kept (keys are unique)
#pragma unroll
    for (int t = KC - 1; t > 0; --t) {
        const uint64_t prev = key[t - 1];
        key[t] = prev > v ? prev : (key[t] > v ? v : key[t]);
    }
    key[0] = key[0] > v ? v : key[0];
}

template <int KC>
__device__ __forceinline__ void list_pop(uint64_t (&key)[KC], bool pop) {
#pragma unroll
    for (int t = 0; t < KC - 1; ++t) key[t] = pop ? key[t + 1] : key[t];
    key[KC - 1] = pop ? ~0ull : key[KC - 1];
}

// Per-lane scan of row i of D2 (the sum of NP partial planes, added in plane order) into a
// sorted list of the lane's KC smallest keys; returns how many valid columns the lane saw.
// NB float4 per lane and plane are loaded before any is consumed (one memory latency per
// 256*NB columns); addresses past the row are clamped, not branched around.
template <int KC, int NP>
__device__ __forceinline__ int scan_row(const float* __restrict__ row, size_t plane, int n,
                                        int ld, int i, uint64_t (&key)[KC]) {
    constexpr int NB = 4;
    const int lane = lane_id();
#pragma unroll
    for (int t = 0; t < KC; ++t) key[t] = ~0ull;
    int seen = 0;
    for (int jb = 0; jb < n; jb += 4 * kWave * NB) {
        f32x4 v[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int j0 = jb + 4 * (b * kWave + lane);
            const int jc = j0 < ld ? j0 : 0;
            v[b] = *reinterpret_cast<const f32x4*>(row + jc);
#pragma unroll
            for (int p = 1; p < NP; ++p) v[b] += *reinterpret_cast<const f32x4*>(row + p * plane + jc);
        }
#ifdef GLL_TRACE
        if (jb == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (blockIdx.x == 0 && threadIdx.x == 0) g_trace[23] = __builtin_amdgcn_s_memrealtime();
        }
#endif
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int j0 = jb + 4 * (b * kWave + lane);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = j0 + t;
                if (j < n && j != i && v[b][t] == v[b][t]) {   // NaN rows never enter
                    ++seen;
                    const uint64_t kv = pack_key(v[b][t], j);
                    if (kv < key[KC - 1]) list_insert<KC>(key, kv);
                }
            }
        }
    }
    return seen;
}

// Wave64 minimum of a 32-bit unsigned key through DPP (broadcast result).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_min_u32(uint32_t v) {
    const uint32_t o = __builtin_amdgcn_update_dpp(0xFFFFFFFFu, v, CTRL, ROW_MASK, 0xf, false);
    return o < v ? o : v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = dpp_min_u32<0xB1, 0xf>(v);
    v = dpp_min_u32<0x4E, 0xf>(v);
    v = dpp_min_u32<0x141, 0xf>(v);
    v = dpp_min_u32<0x140, 0xf>(v);
    v = dpp_min_u32<0x142, 0xa>(v);
    v = dpp_min_u32<0x143, 0xc>(v);
    return __builtin_amdgcn_readlane(v, 63);
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_max_u32(uint32_t v) {
    const uint32_t o = __builtin_amdgcn_update_dpp(0u, v, CTRL, ROW_MASK, 0xf, false);
    return o > v ? o : v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = dpp_max_u32<0xB1, 0xf>(v);
    v = dpp_max_u32<0x4E, 0xf>(v);
    v = dpp_max_u32<0x141, 0xf>(v);
    v = dpp_max_u32<0x140, 0xf>(v);
    v = dpp_max_u32<0x142, 0xa>(v);
    v = dpp_max_u32<0x143, 0xc>(v);
    return __builtin_amdgcn_readlane(v, 63);
}

// Exact merge (fallback): round t hands the t-th smallest (d2, index) key to lane t.
template <int KC>
__device__ __forceinline__ int merge_exact(uint64_t (&key)[KC], int kc) {
    const int lane = lane_id();
    uint64_t mine = ~0ull;
    for (int t = 0; t < kc; ++t) {
        const uint64_t best = wave_min_u64(key[0]);
        if (lane == t) mine = best;
        list_pop<KC>(key, best != ~0ull && key[0] == best);
    }
    return mine == ~0ull ? -1 : int(uint32_t(mine));
}

// Fast merge: 32-bit DPP arg-min on (value bits with the lane id in the 6 low bits).  The
// candidate SET can differ from the exact one only between values within 64 ulp of each
// other, which the exact re-rank margin absorbs.  Returns true when some lane emptied its
// list while holding more columns (the set may then miss one): the caller re-runs exactly.
template <int KS>
__device__ __forceinline__ bool merge_fast(uint64_t (&key)[KS], int kc, int seen, int& ci) {
    const int lane = lane_id();
    int popped = 0;
    ci = -1;
    for (int t = 0; t < kc; ++t) {
        const uint32_t hi = uint32_t(key[0] >> 32);
        const uint32_t packed = key[0] == ~0ull ? 0xFFFFFFFFu : ((hi & ~63u) | uint32_t(lane));
        const uint32_t m = wave_min_u32(packed);
        if (m == 0xFFFFFFFFu) break;
        const int wl = int(m & 63u);
        const int idx = __builtin_amdgcn_readlane(int(uint32_t(key[0])), wl);
        if (lane == t) ci = idx;
        const bool pop = lane == wl;
        list_pop<KS>(key, pop);
        popped += pop ? 1 : 0;
    }
    return __ballot(popped == KS && seen > KS) != 0;
}

// Threshold merge: T = the kc-th smallest 32-bit key head (the D2 bits) over all lanes' lists,
// by bisection -- each step is KS ballots and scalar popcounts, no DPP chain (~0.4 us against
// ~2 us for kc arg-min rounds at NS).  Every list entry <= T is a candidate, ties at T
// included, so the set is exact on the D2 values (at most 64).  Returns true when it may be
// incomplete: some lane's whole list is <= T while that lane saw more columns, or more than 64
// candidates tie in; the caller then re-runs the exact merge.
template <int KS>
__device__ __forceinline__ bool merge_threshold(const uint64_t (&key)[KS], int kc, int seen,
                                                int* __restrict__ cand, int& ci, int& kce) {
    const int lane = lane_id();
    uint32_t hv[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) hv[s] = uint32_t(key[s] >> 32);   // empty slots: 0xFFFFFFFF
    auto count_le = [&](uint32_t t) {
        int c = 0;
#pragma unroll
        for (int s = 0; s < KS; ++s) c += __popcll(__ballot(hv[s] <= t));
        return c;
    };
    // T lies between the smallest list head and, when at least kc entries are that small, the
    // largest head: a bracket of ~2^24 instead of 2^32 (8 fewer steps at NS)
    uint32_t lo = wave_min_u32(hv[0]), up = 0xFFFFFFFEu;
    const uint32_t hmax = wave_max_u32(hv[0] == 0xFFFFFFFFu ? 0u : hv[0]);
    if (lo > up) lo = up;   // every list empty
    if (hmax >= lo && count_le(hmax) >= kc) up = hmax;
    if (count_le(up) >= kc) {
        while (lo < up) {   // smallest T with count_le(T) >= kc (wave-uniform, <= 32 steps)
            const uint32_t mid = lo + ((up - lo) >> 1);
            if (count_le(mid) >= kc) up = mid;
            else lo = mid + 1u;
        }
    }
    const uint32_t T = up;   // fewer than kc valid entries: all of them
    const uint64_t below = (1ull << lane) - 1ull;
    int mine = 0, before = 0, total = 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const uint64_t mk = __ballot(hv[s] <= T);
        mine += hv[s] <= T ? 1 : 0;
        before += __popcll(mk & below);
        total += __popcll(mk);
    }
    const bool redo = (__ballot(mine == KS && seen > KS) != 0) || total > kWave;
    if (!redo) {   // a lane's entries <= T are a prefix of its sorted list
#pragma unroll
        for (int s = 0; s < KS; ++s)
            if (hv[s] <= T) cand[before + s] = int(uint32_t(key[s]));
    }
    __builtin_amdgcn_wave_barrier();   // a wave's LDS ops run in order: the reads see the stores
    asm volatile("" ::: "memory");
    kce = total;
    ci = (!redo && lane < total) ? cand[lane] : -1;
    return redo;
}

template <int KC, bool VEC, int NP, int PG>
__global__ __launch_bounds__(256) void knn_select_kernel(
    const float* __restrict__ D2, int ld, size_t plane, const float* __restrict__ X, int n, int d, int K,
    int kc, float eps_fixed, int auto_eps, int RCAP, int32_t* __restrict__ knn_idx,
    float* __restrict__ knn_d2, float* __restrict__ eps, int32_t* __restrict__ rev_cnt,
    int32_t* __restrict__ rev_idx, float* __restrict__ rev_d2, int32_t* __restrict__ ovf,
    int32_t* __restrict__ status, int32_t* __restrict__ status_pub, size_t xs, size_t wss,
    size_t sts) {
    GLL_TRACE_SCOPE(1);
    GLL_TRACE_PT(20);
    D2 = gshift(D2, wss);
    X = gshift(X, xs);
    knn_idx = gshift(knn_idx, wss);
    knn_d2 = gshift(knn_d2, wss);
    eps = gshift(eps, wss);
    rev_cnt = gshift(rev_cnt, wss);
    rev_idx = gshift(rev_idx, wss);
    rev_d2 = gshift(rev_d2, wss);
    ovf = gshift(ovf, wss);
    status = gshift(status, wss);
    status_pub = gshift(status_pub, sts);
    __shared__ int s_cand[4][kWave];
    const int lane = lane_id();
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;  // whole wave

    // 1-2) candidates: short per-lane lists + threshold merge, exact re-run when inexact
    const float* row = D2 + size_t(i) * ld;
    constexpr int KS = KC <= 16 ? 4 : 8;
    int ci, kce;
    {
        uint64_t key[KS];
        const int seen = scan_row<KS, NP>(row, plane, n, ld, i, key);
        GLL_TRACE_PT(16);
        const bool redo = merge_threshold<KS>(key, kc, seen, s_cand[threadIdx.x >> 6], ci, kce);
        GLL_TRACE_PT(17);
        if (redo) {
            uint64_t full[KC];
            scan_row<KC, NP>(row, plane, n, ld, i, full);
            ci = merge_exact<KC>(full, kc);
            kce = kc;
        }
    }
    // 3) exact squared distances, 8 candidates per pass (8 lanes each, across d).  PG passes
    //    per sweep with every load in flight at once: PG = 2 for single-graph launches (one
    //    wave per SIMD anyway); batches keep PG = 1 (191 VGPRs at PG = 2 cost them 20-45%
    //    occupancy).  Per-candidate arithmetic is the same either way.
    const int grp = lane >> 3, sub = lane & 7;
    const float* xi = X + size_t(i) * d;
    float ce = __builtin_inff();
    for (int p0 = 0; p0 < kce; p0 += 8 * PG) {
        const float* xj[PG];
#pragma unroll
        for (int g2 = 0; g2 < PG; ++g2) {
            const int idx = p0 + 8 * g2 + grp;
            const int j = __shfl(ci, idx < kce ? idx : 0);
            const bool live = idx < kce && j >= 0;
            xj[g2] = X + size_t(live ? j : i) * d;
        }
        float part[PG];
#pragma unroll
        for (int g2 = 0; g2 < PG; ++g2) part[g2] = 0.f;
        for (int kb = 0; kb < d; kb += 512) {   // 16 steps of 32 features: all loads in flight
            f32x4 va[16], vb[PG][16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {   // straight-line: every load issued before use
                const int k = kb + 32 * u + 4 * sub;
                va[u] = load4_raw<VEC>(xi, k, d);
#pragma unroll
                for (int g2 = 0; g2 < PG; ++g2) vb[g2][u] = load4_raw<VEC>(xj[g2], k, d);
            }
#pragma unroll
            for (int g2 = 0; g2 < PG; ++g2) {
#pragma unroll
                for (int u = 0; u < 16; ++u) {   // same order from either end: symmetric in (i, j)
                    const int k = kb + 32 * u + 4 * sub;
                    const f32x4 df = mask4<VEC>(va[u] - vb[g2][u], k, d);
                    part[g2] += df.x * df.x;
                    part[g2] += df.y * df.y;
                    part[g2] += df.z * df.z;
                    part[g2] += df.w * df.w;
                }
            }
        }
#pragma unroll
        for (int g2 = 0; g2 < PG; ++g2) {
            const float tot = group8_sum(part[g2]);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const float v = readlane_f(tot, 8 * g);
                if (lane == p0 + 8 * g2 + g) ce = v;
            }
        }
    }
    GLL_TRACE_PT(18);
    if (ci < 0) ce = __builtin_inff();
    // 4) rank the candidates by (exact d^2, index); keep the K-1 nearest
    const uint64_t myk = ci < 0 ? ~0ull : pack_key(ce, ci);
    int rank = 0;
    for (int u = 0; u < kce; ++u) {
        const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(myk), u);
        const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(myk >> 32), u);
        const uint64_t ku = (uint64_t(hi) << 32) | lo;
        rank += ku < myk ? 1 : 0;
    }
    const bool keep = lane < kce && ci >= 0 && rank < K - 1;
    int32_t* oi = knn_idx + size_t(i) * K;
    float* od = knn_d2 + size_t(i) * K;
    if (lane == 0) {
        oi[0] = i;
        od[0] = 0.f;
    }
    if (keep) {
        oi[1 + rank] = ci;
        od[1 + rank] = ce;
    }
    // rows with fewer valid candidates (non-finite input) fall back to self at distance 0,
    // i.e. dropped edges (sparse.find drops zeros, GLL.py:198)
    const int nkeep = __popcll(__ballot(keep));
    if (lane >= nkeep && lane < K - 1) {
        oi[1 + lane] = i;
        od[1 + lane] = 0.f;
    }
    GLL_TRACE_PT(19);
    float ei = eps_fixed;
    if (auto_eps) {
        // eps_i = d(i, knn_ind[i, K-1])  (GLL.py:205)
        const float e = (keep && rank == K - 2) ? sqrtf(ce) : 0.f;
        ei = wave_sum_dpp(e);
    }
    if (lane == 0) {
        eps[i] = ei;
        if (!(ei >= 1e-10f)) atomicOr(&status_pub[GLL_ST_TINY_EPS], 1);  // GLL.py:240-241
    }
    // 5) reverse entry (ci, i) for every valid pair; zero distances never enter the graph
    if (keep && ce > 0.f) {
        const int pos = atomicAdd(&rev_cnt[ci], 1);
        if (pos < RCAP) {
            rev_idx[size_t(ci) * RCAP + pos] = i;
            rev_d2[size_t(ci) * RCAP + pos] = ce;
        } else {
            const int q = atomicAdd(&status[kStOvfCount], 1);
            ovf[3 * q + 0] = ci;
            ovf[3 * q + 1] = i;
            ovf[3 * q + 2] = __float_as_int(ce);
        }
    }
}

// Wide 128-tiles when there are enough of them to fill the chip twice over (large graphs and
// batches); the 64-tile kernel otherwise (a single NS graph has only 36 wide tiles).
static bool use_wide_gram(const Layout& L, const Batch& bt) {
    if (gram_planes(L, bt.B) != 1 || (L.flags & GLL_FLAG_GRAM_NARROW)) return false;
    const int64_t T = (L.n + 127) / 128;
    return int64_t(bt.B) * T * (T + 1) / 2 >= 512;
}

// 48-tiles when 64-tiles would leave a quarter of the CUs idle and 48-tiles fit in one round.
static bool use_gram48(const Layout& L, const Batch& bt) {
    if (gram_planes(L, bt.B) != 1 || (L.flags & GLL_FLAG_GRAM_NARROW)) return false;
    const int64_t T64 = (L.n + 63) / 64, T48 = (L.n + 47) / 48;
    return int64_t(bt.B) * T64 * (T64 + 1) / 2 < 192 && int64_t(bt.B) * T48 * (T48 + 1) / 2 <= 256;
}

hipError_t launch_gram(const Layout& L, const Batch& bt, void* ws, const float* X, bool vec,
                       hipStream_t s) {
    const int planes = gram_planes(L, bt.B);
    if (planes == 2) {
        const int T = (L.n + 63) / 64;
        const dim3 grid(T * T, bt.B);
        float* D2 = L.at<float>(ws, L.D2);
        const size_t plane = size_t(L.n) * L.ldD;
        int32_t* st = L.at<int32_t>(ws, L.status);
        int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
        prof_begin(GLL_K_GRAM, s);
        if (vec)
            launch_k(gram_bf3s_kernel<true>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, plane, st, rc, bt.x, bt.ws);
        else
            launch_k(gram_bf3s_kernel<false>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, plane, st, rc, bt.x, bt.ws);
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(bf3s)");
    }
    if (!(L.flags & GLL_FLAG_GRAM_F32) && !(L.flags & GLL_FLAG_GRAM_NARROW)) {
        const int T = (L.n + 127) / 128;
        if (int64_t(bt.B) * T * (T + 1) / 2 >= 512) {   // enough 128-tiles to fill the chip twice
            const dim3 grid(T * (T + 1) / 2, bt.B);
            float* D2 = L.at<float>(ws, L.D2);
            int32_t* st = L.at<int32_t>(ws, L.status);
            int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
            prof_begin(GLL_K_GRAM, s);
            if (vec)
                launch_k(gram_bf3w_kernel<true>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws);
            else
                launch_k(gram_bf3w_kernel<false>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws);
            prof_end(GLL_K_GRAM, s);
            return launch_status("knn.hip:launch_gram(bf3w)");
        }
    }
    if (!(L.flags & GLL_FLAG_GRAM_F32)) {
        const int T = (L.n + 63) / 64;
        const dim3 grid(T * (T + 1) / 2, bt.B);
        float* D2 = L.at<float>(ws, L.D2);
        int32_t* st = L.at<int32_t>(ws, L.status);
        int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
        prof_begin(GLL_K_GRAM, s);
        if (vec)
            launch_k(gram_bf3_kernel<true>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws);
        else
            launch_k(gram_bf3_kernel<false>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws);
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(bf3)");
    }
    if (use_gram48(L, bt)) {
        const int T = (L.n + 47) / 48;
        const dim3 grid(T * (T + 1) / 2, bt.B);
        float* D2 = L.at<float>(ws, L.D2);
        int32_t* st = L.at<int32_t>(ws, L.status);
        int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
        const int nchunk = (L.d + kGK - 1) / kGK;
        prof_begin(GLL_K_GRAM, s);
#define GLL_G48(V, N) \
    launch_k(gram48_kernel<V, N>, grid, 768, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws)
        if (vec) { if (nchunk >= 4) GLL_G48(true, 4); else if (nchunk >= 2) GLL_G48(true, 2); else GLL_G48(true, 1); }
        else { if (nchunk >= 4) GLL_G48(false, 4); else if (nchunk >= 2) GLL_G48(false, 2); else GLL_G48(false, 1); }
#undef GLL_G48
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(48)");
    }
    if (use_wide_gram(L, bt)) {
        const int T = (L.n + 127) / 128;
        const dim3 grid(T * (T + 1) / 2, bt.B);
        float* D2 = L.at<float>(ws, L.D2);
        int32_t* st = L.at<int32_t>(ws, L.status);
        int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
        const int nchunk = (L.d + kWK - 1) / kWK;
        prof_begin(GLL_K_GRAM, s);
#define GLL_WIDE(V, N) \
    launch_k(gram_wide_kernel<V, N>, grid, 256, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws)
        if (vec) { if (nchunk >= 2) GLL_WIDE(true, 2); else GLL_WIDE(true, 1); }
        else { if (nchunk >= 2) GLL_WIDE(false, 2); else GLL_WIDE(false, 1); }
#undef GLL_WIDE
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(wide)");
    }
    const int T = (L.n + 63) / 64;
    const int tiles = T * (T + 1) / 2;
    const int KS = planes;
    // slice of the features per split in whole 64-deep chunks, grouped NCH per super-chunk.
    // (128-deep chunks -- half the barriers -- measured no faster at NS, B = 64 or stress:
    // profiles/r01_gram_chunk_depth.txt; the template keeps the depth a parameter.)
    constexpr int GK = kGK;
    const int dsl = (L.d + KS - 1) / KS;
    int kspan = (dsl + GK - 1) / GK * GK;
    const int NCH = kspan >= 2 * GK ? 2 : 1;   // (4 spills beside two accumulator chains)
    kspan = (kspan + NCH * GK - 1) / (NCH * GK) * (NCH * GK);
    float* D2 = L.at<float>(ws, L.D2);
    const size_t plane = size_t(L.n) * L.ldD;
    int32_t* st = L.at<int32_t>(ws, L.status);
    int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
    const dim3 grid(tiles * KS, bt.B);
    prof_begin(GLL_K_GRAM, s);
#define GLL_GRAM(V, N, G)                                                                         \
    launch_k(gram_lds_kernel<V, N, G>, grid, 512, 0, s, X, L.n, L.d, T, KS, kspan, D2, L.ldD, plane, st, \
                                                   rc, bt.x, bt.ws)
    if (vec) {
        if (NCH == 2) GLL_GRAM(true, 2, GK); else GLL_GRAM(true, 1, GK);
    } else {
        if (NCH == 2) GLL_GRAM(false, 2, GK); else GLL_GRAM(false, 1, GK);
    }
#undef GLL_GRAM
    prof_end(GLL_K_GRAM, s);
    return launch_status("knn.hip:launch_gram");
}

hipError_t launch_select(const Layout& L, const Batch& bt, void* ws, const float* X,
                         float eps_fixed, bool auto_eps, bool vec, int32_t* status_pub,
                         hipStream_t s) {
    const int n = L.n, K = L.K;
    // candidate list capacity: smallest of {16, 32, 64} leaving a re-rank margin >= 4
    const int need = K - 1 + 4;
    const int KC = need <= 16 ? 16 : (need <= 32 ? 32 : 64);
    if (K - 1 > 64) return hipErrorInvalidValue;
    int margin = KC - (K - 1);
    if (margin > 8) margin = 8;
    int kc = K - 1 + margin;
    if (kc > n - 1) kc = n - 1;
    dim3 grid((n + 3) / 4, bt.B);
    prof_begin(GLL_K_SELECT, s);
    const size_t plane = size_t(n) * L.ldD;
    const int planes = gram_planes(L, bt.B);
#define GLL_SEL3(KCV, V, NPV)                                                                  \
    launch_k((bt.B == 1 ? knn_select_kernel<KCV, V, NPV, 2> : knn_select_kernel<KCV, V, NPV, 1>), grid, 256, 0, s,  \
        L.at<float>(ws, L.D2), L.ldD, plane, X, n, L.d, K, kc, eps_fixed, auto_eps ? 1 : 0,     \
        L.RCAP,                                                                                \
        L.at<int32_t>(ws, L.knn_idx), L.at<float>(ws, L.knn_d2), L.at<float>(ws, L.eps),       \
        L.at<int32_t>(ws, L.rev_cnt), L.at<int32_t>(ws, L.rev_idx), L.at<float>(ws, L.rev_d2), \
        L.at<int32_t>(ws, L.ovf), L.at<int32_t>(ws, L.status), status_pub, bt.x, bt.ws, bt.st)
#define GLL_SEL(KCV, V)                                                                        \
    do {                                                                                       \
        if (planes == 2) GLL_SEL3(KCV, V, 2);                                                  \
        else GLL_SEL3(KCV, V, 1);                                                              \
    } while (0)
    if (KC == 16) { if (vec) GLL_SEL(16, true); else GLL_SEL(16, false); }
    else if (KC == 32) { if (vec) GLL_SEL(32, true); else GLL_SEL(32, false); }
    else { if (vec) GLL_SEL(64, true); else GLL_SEL(64, false); }
#undef GLL_SEL
#undef GLL_SEL3
    prof_end(GLL_K_SELECT, s);
    return launch_status("knn.hip:launch_select");
}

}  // namespace gll
