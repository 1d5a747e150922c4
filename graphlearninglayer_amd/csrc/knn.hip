// knn.hip -- exact brute-force kNN for the GLL graph (replaces the annoy search of
// graphlearning.weightmatrix.knnsearch, /root/reference/GLL.py:183).
//
//  K1a gram_bf3*_kernel D2 = |a_i|^2 + |a_j|^2 - 2 <a_i, a_j> on split-bf16 MFMA over the
//                       rows centred on row 0 (a = x - x_0: distance-invariant, and it keeps
//                       the product error proportional to the spread of the rows, not to
//                       their offset), upper-triangle tiles only (mirrored writes).  D2 only
//                       NOMINATES candidates.
//  K1b knn_select_kernel one wave per row:
//                       1. per-lane sorted candidate lists over the D2 row (16-B loads);
//                       2. a threshold merge to kc = K-1+margin candidates (exact 64-bit
//                          merge when a lane's list overflowed);
//                       3. exact re-ranking with d^2 = sum_k (x_ik - x_jk)^2 in float64,
//                          eight candidates at a time (8-lane groups, DPP group sums) --
//                          bitwise symmetric in (i, j) because both orders run the same lane
//                          mapping;
//                       4. the K-1 nearest by (exact d^2, index); self forced to rank 0 with
//                          distance 0 (the stand-in contract of SURVEY.md §8c);
//                       5. a certificate that no column left out of the candidates can beat
//                          the (K-1)-th exact distance given the Gram's error bound, else an
//                          exact re-rank of every column under the bound (rare; counted in
//                          GLL_ST_KNN_RESCAN) -- the result is the exact kNN for any input;
//                       6. every valid pair (i -> j) is pushed onto j's reverse list (or the
//                          overflow list), which is how the symmetric union of GLL.py:197 is
//                          built without an n x n structure or a prefix sum.
#include <limits.h>

#include <type_traits>


#include "gll_internal.h"

namespace gll {

GLL_TRACE_UNIT(knn)

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
// b % 8), so block b takes tile (b % 8) * ceil-share + b / 8: each XCD
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
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));

// D2 storage of the pre-split path (round 3): fp16 of D2 x s, s = 2^e per graph with every
// D2 <= 4 max|a|^2 mapped below 2^14 (d2_scale), or fp32 (H = false).  D2 only nominates
// candidates; the select decodes x 1/s (exact) and widens its error bounds by the fp16 rounding.
template <bool H>
__device__ __forceinline__ void dput(float* D2, size_t o, float v, float s) {
    if constexpr (H) reinterpret_cast<_Float16*>(D2)[o] = static_cast<_Float16>(v * s);
    else D2[o] = v;
}
template <bool H>
__device__ __forceinline__ void dput4(float* D2, size_t o, f32x4 v, float s) {
    if constexpr (H) {
        const h16x4 hv = {static_cast<_Float16>(v.x * s), static_cast<_Float16>(v.y * s),
                          static_cast<_Float16>(v.z * s), static_cast<_Float16>(v.w * s)};
        *reinterpret_cast<h16x4*>(reinterpret_cast<_Float16*>(D2) + o) = hv;
    } else {
        *reinterpret_cast<f32x4*>(D2 + o) = v;
    }
}
constexpr int kBP = 256;            // features per phase
constexpr int kMaxCen = 4096;       // LDS copy of the centre row: d <= 4096 (gll.h limit)
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
// NT = 512 is the half tile (gram_bf3h_kernel): 2 feature halves instead of 4 quarters, and
// 8 tile elements per thread; slot s of wave w holds rows 16 s + 2 w (lanes 0..31) and
// 16 s + 2 w + 1 (lanes 32..63), reduced per half wave.
template <int NT = 1024, typename NF>
__device__ __forceinline__ void bf3_epilogue(const f32x16& acc, const float (&sq)[8], float* smem,
                                             float (*sqp)[16], float* nrm, NF nrm_of, int bi,
                                             int bj, int n, float* __restrict__ D2, int ld,
                                             float* __restrict__ Dz) {
    static_assert(NT == 1024 || NT == 512, "bf3_epilogue: 1024- or 512-thread tiles");
    constexpr int KQ = NT / 256;     // feature groups per quadrant
    constexpr int EP = 4096 / NT;    // tile elements per thread
    constexpr int CPR = 64 / EP;     // threads per tile row
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int qd = w & 3, kq = w >> 2;
    if constexpr (NT == 1024) {
        // row norms: slot s of wave w is tile row 16 s + w, its features spread over the wave
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const float t = wave_sum_dpp(sq[s]);
            if (lane == 0) sqp[s][w] = t;
        }
    } else {
        // half-wave sums: row sums of 16 lanes, then row_bcast15 carries row 0 into row 1 and
        // row 2 into row 3 (lane 31: lanes 0..31, lane 63: lanes 32..63)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            float t = dpp_add<0xB1, 0xf>(sq[s]);
            t = dpp_add<0x4E, 0xf>(t);
            t = dpp_add<0x141, 0xf>(t);
            t = dpp_add<0x140, 0xf>(t);
            t = dpp_add<0x142, 0xa>(t);
            if ((lane & 31) == 31) sqp[s][2 * w + h] = t;
        }
    }
    __syncthreads();   // fragment reads done: the planes become partial / tile space
    // partial quadrant -> LDS part[kq][qd][32][33] (C layout: col = lane & 31,
    // row = (e&3) + 8(e>>2) + 4h)
    float* pw = smem + (kq * 4 + qd) * 32 * 33;
#pragma unroll
    for (int e = 0; e < 16; ++e) pw[((e & 3) + 8 * (e >> 2) + 4 * h) * 33 + r] = acc[e];
    if (tid < 128) nrm[tid] = nrm_of(tid);
    __syncthreads();
    // tile element (ti, tj..tj+EP-1): sum of the KQ feature groups, fixed order
    const int ti = tid / CPR, tj = EP * (tid % CPR);
    float v[EP];
    {
        const int q = 2 * (ti >> 5) + (tj >> 5), rr = ti & 31;
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            const int cc = (tj & 31) + e;
            float t = 0.f;
#pragma unroll
            for (int k4 = 0; k4 < KQ; ++k4) t += smem[(k4 * 4 + q) * 32 * 33 + rr * 33 + cc];
            v[e] = t;
        }
    }
    __syncthreads();
    float* tile = smem + KQ * 4 * 32 * 33;   // [64][65], past the partials
#pragma unroll
    for (int e = 0; e < EP; ++e) tile[ti * 65 + tj + e] = nrm[ti] + nrm[64 + tj + e] - 2.f * v[e];
    __syncthreads();
    // direct orientation: row bi*64 + ti, columns bj*64 + tj .. +EP-1; a diagonal tile takes
    // the upper triangle for both halves so D2 stays bitwise symmetric
    const int i = bi * 64 + ti;
    if (i < n) {
#pragma unroll
        for (int c = 0; c < EP; c += 4) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int jj = tj + c + e;
                o[e] = (bi == bj && jj < ti) ? tile[jj * 65 + ti] : tile[ti * 65 + jj];
            }
            const int j0 = bj * 64 + tj + c;
            float* dst = D2 + size_t(i) * ld + j0;
            float* dz = Dz ? Dz + size_t(i) * ld + j0 : nullptr;
            if (j0 + 4 <= n) {
                __builtin_nontemporal_store(f32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4*>(dst));
                if (dz) __builtin_nontemporal_store(f32x4{0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f32x4*>(dz));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (j0 + e < n) {
                        dst[e] = o[e];
                        if (dz) dz[e] = 0.f;
                    }
            }
        }
    }
    // mirrored orientation: row bj*64 + ti, columns bi*64 + tj .. from the tile's column ti
    const int jr = bj * 64 + ti;
    if (bi != bj && jr < n) {
#pragma unroll
        for (int c = 0; c < EP; c += 4) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = tile[(tj + c + e) * 65 + ti];
            const int j0 = bi * 64 + tj + c;
            float* dst = D2 + size_t(jr) * ld + j0;
            if (j0 + 4 <= n) {
                __builtin_nontemporal_store(f32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4*>(dst));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (j0 + e < n) dst[e] = o[e];
            }
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
    __shared__ __attribute__((aligned(16))) float cen[kMaxCen];          // centre row x_0
    float* smem = reinterpret_cast<float*>(smem_h);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar row bases
    const int r = lane & 31, h = lane >> 5;
    int bi = 0, rem = xcd_tile(bx(), gridDim.x);
    while (rem >= T - bi) {
        rem -= T - bi;
        ++bi;
    }
    const int bj = bi + rem;
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = bx() * 1024 + tid;
        if (g < kStWords) status[g] = 0;
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
        __syncthreads();   // the previous phase's fragment reads are done (and cen is staged)
        const f32x4 c = *reinterpret_cast<const f32x4*>(cen + ph * kBP + fo);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const f32x4 f = mask4<VEC>(v[s] - c, k, d);
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
        // the centre row (row 0 of the graph) into LDS: issued first, so staging it waits for
        // that load only (loads return in order) while the first phase's rows stay in flight
        const f32x4 cv = load4_raw<VEC>(X, 4 * tid, d);
        f32x4 va[8], vb[8];
        gload(0, va);
        if (4 * tid < nph * kBP) *reinterpret_cast<f32x4*>(cen + 4 * tid) = mask4<VEC>(cv, 4 * tid, d);
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

// K1a'' (d <= 128, fewer than 512 64-tiles): the same tile at half the workgroup.  The
// 1024-thread tile stages kBP = 256 features per phase, so at d <= 128 half its loads and half
// its MFMAs run on zero features, and its 151 KiB of LDS holds one workgroup per CU: FullySup's
// 300 tiles (n = 1500) ran as two rounds over 256 CUs.  Here 8 waves (4 quadrants x 2 feature
// halves) stage 128 rows x 128 features in 70 KiB: two workgroups per CU, one round.  Lanes
// 0..31 and 32..63 of a wave hold two rows (512 contiguous bytes each), so the loads stay
// coalesced; the epilogue is bf3_epilogue<512>.
constexpr int kHP = 128;          // features of the half tile
constexpr int kHS = kHP + 8;      // its LDS plane row stride (bf16)
template <bool VEC>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void gram_bf3h_kernel(const float* __restrict__ X, int n, int d, int T, float* __restrict__ D2,
                      int ld, int32_t* __restrict__ status, int32_t* __restrict__ rev_cnt,
                      size_t xs, size_t wss) {
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    constexpr int kPlane = 128 * kHS;
    static_assert(2 * kPlane * 2 >= (8 * 32 * 33 + 64 * 65) * 4, "half tile: epilogue space");
    __shared__ __attribute__((aligned(16))) __bf16 smem_h[2 * kPlane];
    __shared__ float sqp[8][16];
    __shared__ float nrm[128];
    float* smem = reinterpret_cast<float*>(smem_h);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    int bi = 0, rem = xcd_tile(bx(), gridDim.x);
    while (rem >= T - bi) {
        rem -= T - bi;
        ++bi;
    }
    const int bj = bi + rem;
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = bx() * 512 + tid;
        if (g < kStWords) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 512) rev_cnt[q] = 0;
    }
    const int fo = 4 * r;   // this lane's 4 features
    // slot s -> LDS row 16 s + 2 w + h (0..63 rows bi, 64..127 rows bj; rows past n clamped);
    // the centre row's load is issued first
    const f32x4 c = load4_raw<VEC>(X, fo, d);
    f32x4 v[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int R = 16 * s + 2 * w + h;
        const int row = R < 64 ? bi * 64 + R : bj * 64 + R - 64;
        v[s] = load4_raw<VEC>(X + size_t(row < n ? row : n - 1) * d, fo, d);
    }
    float sq[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const f32x4 f = mask4<VEC>(v[s] - c, fo, d);
        sq[s] = f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
        bf16x4 hv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const __bf16 hb = static_cast<__bf16>(f[e]);
            hv[e] = hb;
            lv[e] = static_cast<__bf16>(f[e] - static_cast<float>(hb));
        }
        const int o = (16 * s + 2 * w + h) * kHS + fo;
        *reinterpret_cast<bf16x4*>(smem_h + o) = hv;
        *reinterpret_cast<bf16x4*>(smem_h + kPlane + o) = lv;
    }
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    const int qd = w & 3, kq = w >> 2;   // quadrant, feature half
    const int qa = qd >> 1, qb = qd & 1;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
        const int kk = 64 * kq + 16 * st + 8 * h;
        const int oa = (32 * qa + r) * kHS + kk, ob = (64 + 32 * qb + r) * kHS + kk;
        const bf16x8 ha = *reinterpret_cast<const bf16x8*>(smem_h + oa);
        const bf16x8 la = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + oa);
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(smem_h + ob);
        const bf16x8 lb = *reinterpret_cast<const bf16x8*>(smem_h + kPlane + ob);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(la, hb, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, lb, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha, hb, acc, 0, 0, 0);
    }
    bf3_epilogue<512>(acc, sq, smem, sqp, nrm, [&](int t) { return sqp[t >> 4][t & 15]; }, bi, bj,
                      n, D2, ld, nullptr);
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
    const int b = xcd_tile(bx(), gridDim.x);
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
        const int g = bx() * 1024 + tid;
        if (g < kStWords) status[g] = 0;
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
    // centre row (row 0 of the graph) over the phase(s) this workgroup multiplies
    const f32x4 cen0 = load4_raw<VEC>(X, (dg ? 0 : half) * kBP + fo, d);
    const f32x4 cen1 = load4_raw<VEC>(X, (dg ? 1 : half) * kBP + fo, d);
    float sq[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int k = (dg ? (s >> 2) : half) * kBP + fo;
        const f32x4 f = mask4<VEC>(v[s] - (s >= 4 ? cen1 : cen0), k, d);
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
                                                         size_t xs, size_t wss, int r0,
                                                         int pt) {
    // pt > 0 (a row panel, build_graph): rectangular tiles of rows r0 .. r0 + 128 pt against
    // every column block, stored in the direct orientation only into the panel's rows of D2
    X = gshift_br(X, xs);
    D2 = gshift_br(D2, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    constexpr int kPlane = 256 * kWS;                                   // bf16 per plane
    __shared__ __attribute__((aligned(16))) __bf16 smem_h[2 * kPlane];  // 136 KiB
    __shared__ float nrm[256];
    __shared__ __attribute__((aligned(16))) float cen[kMaxCen];          // centre row x_0
    float* smem = reinterpret_cast<float*>(smem_h);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    int bi = 0, rem = xcd_tile(bx(), gridDim.x), bj;
    if (pt > 0) {
        bi = (r0 >> 7) + rem / T;
        bj = rem % T;
    } else {
        while (rem >= T - bi) {
            rem -= T - bi;
            ++bi;
        }
        bj = bi + rem;
    }
    if (r0 == 0) {   // per-call reset of the counters the select kernel accumulates into
        const int g = bx() * 1024 + tid;
        if (g < kStWords) status[g] = 0;
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
        __syncthreads();   // the previous phase's fragment reads are done (and cen is staged)
        const f32x4 c = *reinterpret_cast<const f32x4*>(cen + ph * kWP + fo);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const f32x4 f = mask4<VEC>(v[q] - c, k, d);
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
        const f32x4 cv = load4_raw<VEC>(X, 4 * tid, d);   // centre row x_0 -> LDS (see gram_bf3)
        f32x4 va[8], vb[8];
        gload(0, va);
        if (4 * tid < nph * kWP) *reinterpret_cast<f32x4*>(cen + 4 * tid) = mask4<VEC>(cv, 4 * tid, d);
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
    if (pt > 0) {   // panel: every tile in the direct orientation, rows relative to r0
        const int j = j0 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int i = i0 + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (i < n && j < n) D2[size_t(i - r0) * ld + j] = dv[e];
        }
    } else if (bi != bj) {
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
// K1a (large problems and batches, round 2): the split done once per row, then a bf16 GEMM.
//
// gram_split_kernel: a_i = x_i - x_0 (centred on row 0 as above), hi = bf16(a), lo = bf16(a -
// hi) into two [n][dp] bf16 planes (dp = d rounded up to 64, zero-padded) and |a_i|^2 (fp32)
// into nrm[n]: one pass over X.  gram_bf3w_kernel redid this split for every tile a row takes
// part in (T times), on the VALU between two barriers per 128-feature phase.
//
// gram_pk_kernel: 128 x 128 upper-triangle tiles (same tile list and XCD order as bf3w), 4
// waves of 64 x 64 (2 x 2 accumulators of 32 x 32), k-stages of 64 features: the four tile
// planes (A hi, A lo, B hi, B lo; 64 KiB) go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no VGPR staging, no conversion), double-buffered so stage k+1's
// loads are in flight while stage k's 48 MFMAs per wave run.  Rows are 128 B in LDS with the
// 16-B segments XOR-swizzled by (row >> 1) & 7 -- on the SOURCE address, the DMA writes
// lane-linearly -- so the ds_read_b128 fragment reads of 16 consecutive rows hit 16 distinct
// bank groups.  One raw s_barrier per stage; the next stage's DMAs are issued between the
// current stage's MFMA groups.
// --------------------------------------------------------------------------------------
constexpr int kPK = 64;                  // features per k-stage
typedef __attribute__((address_space(3))) void lds_void;

// fp16 D2 scale of a graph with M = max |a_i|^2: s = 2^(14 - e) with 4M < 2^e, so every
// stored D2 x s stays below 2^14 (fp16 max 65504); 1 for an all-zero or non-finite graph.
__device__ __forceinline__ float d2_scale(float M) {
    const float t = 4.f * M;
    if (!(t > 1e-30f) || !(t < 1e38f)) return 1.f;
    int e;
    (void)frexpf(t, &e);   // t = f 2^e, f in [0.5, 1)
    int k = 14 - e;
    k = k < -120 ? -120 : (k > 120 ? 120 : k);
    return ldexpf(1.f, k);
}

// Block-wide max of nrm[0 .. n) (the graph's |a_i|^2 from gram_split) -> the fp16 scale; every
// tile of the GEMM computes the same value from the same array, and each stores it to the
// graph's scale word for the select: identical plain stores, no atomics, nothing to reset.
template <int NT>
__device__ __forceinline__ float tile_d2_scale(const float* __restrict__ nrm, int n, float* red) {
    float mx = 0.f;
    for (int q = threadIdx.x; q < n; q += NT) mx = fmaxf(mx, nrm[q]);   // NaN: dropped
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    mx = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) mx = fmaxf(mx, red[w]);
    return d2_scale(mx);
}

template <bool VEC>
__global__ __launch_bounds__(256) void gram_split_kernel(const float* __restrict__ X, int n, int d,
                                                         int dp, __bf16* __restrict__ Ph,
                                                         __bf16* __restrict__ Pl,
                                                         float* __restrict__ nrm,
                                                         int32_t* __restrict__ status,
                                                         int32_t* __restrict__ rev_cnt,
                                                         size_t xs, size_t wss) {
    X = gshift_br(X, xs);
    Ph = gshift_br(Ph, wss);
    Pl = gshift_br(Pl, wss);
    nrm = gshift_br(nrm, wss);
    status = gshift_br(status, wss);
    rev_cnt = gshift_br(rev_cnt, wss);
    {   // per-call reset of the counters the select kernel accumulates into
        const int g = bx() * 256 + threadIdx.x;
        if (g < kStWords) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * 256) rev_cnt[q] = 0;
    }
    const int lane = lane_id();
    const int i = bx() * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const float* xi = X + size_t(i) * d;
    float sq = 0.f;
    for (int k = 4 * lane; k < dp; k += 4 * kWave) {
        const f32x4 c = load4<VEC>(X, k, d);
        const f32x4 f = load4<VEC>(xi, k, d) - c;   // zeros past d
        sq += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
        bf16x4 hv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const __bf16 hb = static_cast<__bf16>(f[e]);
            hv[e] = hb;
            lv[e] = static_cast<__bf16>(f[e] - static_cast<float>(hb));
        }
        *reinterpret_cast<bf16x4*>(Ph + size_t(i) * dp + k) = hv;
        *reinterpret_cast<bf16x4*>(Pl + size_t(i) * dp + k) = lv;
    }
    sq = wave_sum_dpp(sq);
    if (lane == 0) nrm[i] = sq;
}

// Tile t of the upper triangle of T x T blocks in supertile order: supertiles of kSR x kSC
// blocks, row-major, each walked row-major.  With the XCD-contiguous deal of xcd_tile, the ~32
// tiles an XCD runs at once come from one or two supertiles, whose kSR + kSC row blocks
// (512 KB each at d = 1024) mostly stay in that XCD's 4 MB L2, instead of a row-major run whose
// 32 column blocks are streamed from the MALL once per tile.
constexpr int kSR = 4, kSC = 8;
__device__ __forceinline__ void supertile_tile(int t, int T, int& bi, int& bj) {
    for (int I = 0; I * kSR < T; ++I) {
        for (int J = (I * kSR) / kSC; J * kSC < T; ++J) {
            int cnt = 0;
#pragma unroll
            for (int a = 0; a < kSR; ++a) {
                const int r = I * kSR + a;
                const int lo = max(r, J * kSC), hi = min(T, J * kSC + kSC);
                cnt += r < T && hi > lo ? hi - lo : 0;
            }
            if (t < cnt) {
                for (int a = 0; a < kSR; ++a) {
                    const int r = I * kSR + a;
                    const int lo = max(r, J * kSC), hi = min(T, J * kSC + kSC);
                    const int c = r < T && hi > lo ? hi - lo : 0;
                    if (t < c) {
                        bi = r;
                        bj = lo + t;
                        return;
                    }
                    t -= c;
                }
            }
            t -= cnt;
        }
    }
    bi = bj = 0;   // not reached for t < T (T + 1) / 2
}

// One-dimensional grid over B graphs x T (T + 1) / 2 tiles: xcd_tile deals each XCD a
// contiguous run of the graph-major sequence, so a batch's graphs are XCD-local too.
// t0 >= 0 (the tail of a 256-tile launch, launch_gram): with Q = 256 / TS, block Q^2 j + s
// computes TS-subtile s of 256-tile t0 + j in gram_pk2_kernel's sequence (T2 = ceil(T / Q)
// blocks a side, T counted in TS-tiles); subtiles below a diagonal 256-tile's diagonal or past
// n return at once.  TS = 64 (round 6): the tail's 16 256-tiles at stress become 256 workgroups,
// one per CU, instead of 64 128-subtiles on a quarter of the chip; each wave then holds one
// 32 x 32 accumulator.  Every element still sums the same MFMA sequence over k: D2 is bitwise
// the same for any TS.
template <bool H, int TS>
__global__ __launch_bounds__(256) void gram_pk_kernel(const __bf16* __restrict__ Ph,
                                                      const __bf16* __restrict__ Pl,
                                                      const float* __restrict__ nrm, int n,
                                                      int dp, int T, float* __restrict__ D2,
                                                      int ld, size_t wss,
                                                      float* __restrict__ d2s, int t0) {
    const int nks = dp / kPK;
    int g, bi, bj;
    if (t0 < 0) {
        const int NT = T * (T + 1) / 2;
        const int idx = xcd_tile(blockIdx.x, gridDim.x);
        g = idx / NT;
        supertile_tile(idx - g * NT, T, bi, bj);
    } else {
        constexpr int Q = 256 / TS;
        const int T2 = (T + Q - 1) / Q, NT2 = T2 * (T2 + 1) / 2;
        const int idx2 = t0 + int(blockIdx.x) / (Q * Q), sub = int(blockIdx.x) % (Q * Q);
        int b2i, b2j;
        g = idx2 / NT2;
        supertile_tile(idx2 - g * NT2, T2, b2i, b2j);
        bi = Q * b2i + sub / Q;
        bj = Q * b2j + sub % Q;
        if (bi > bj || bj >= T) return;   // whole workgroup, before any barrier
    }
    {
        const size_t off = size_t(g) * wss;   // graph g's workspace block
        Ph = reinterpret_cast<const __bf16*>(reinterpret_cast<const char*>(Ph) + off);
        Pl = reinterpret_cast<const __bf16*>(reinterpret_cast<const char*>(Pl) + off);
        nrm = reinterpret_cast<const float*>(reinterpret_cast<const char*>(nrm) + off);
        D2 = reinterpret_cast<float*>(reinterpret_cast<char*>(D2) + off);
        d2s = reinterpret_cast<float*>(reinterpret_cast<char*>(d2s) + off);
    }
    static_assert(TS == 128 || TS == 64, "128- or 64-row tiles");
    constexpr int MA = TS / 64;                // 32 x 32 accumulators a side per wave
    constexpr int RG = TS / 32;                // 32-row DMA groups per plane
    constexpr int NQ = 4 * RG;                 // DMA pieces per stage (4 planes)
    constexpr int kTP = TS * kPK;                                   // bf16 per tile plane
    __shared__ __attribute__((aligned(16))) __bf16 sm[2 * 4 * kTP];  // TS KiB: [buf][plane]
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int wr = w >> 1, wc = w & 1;
    // this lane's DMA sources: NQ per stage = plane q / RG, rows 8 c .. 8 c + 7 (c = (q % RG) 4
    // + w) as 1 KiB pieces; lane -> row 8 c + lane / 8, LDS segment lane % 8 <- source segment
    // (lane % 8) ^ ((row >> 1) & 7)
    const __bf16* src[16];   // NQ used (a dependent bound here drops the host-side kernel stub)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int pl = q / RG, c = (q % RG) * 4 + w;
        const int row = 8 * c + (lane >> 3);
        const int seg = (lane & 7) ^ ((row >> 1) & 7);
        int grow = (pl < 2 ? bi : bj) * TS + row;
        grow = grow < n ? grow : n - 1;
        src[q] = ((pl & 1) ? Pl : Ph) + size_t(grow) * dp + 8 * seg;
    }
    // DMAs of stage ks into buffer buf, pieces [q0, q0 + NQ / 4)
    auto issue4 = [&](int ks, int buf, int q0) {
#pragma unroll
        for (int q = q0; q < q0 + NQ / 4; ++q) {
            const int pl = q / RG, c = (q % RG) * 4 + w;
            __bf16* dst = sm + (buf * 4 + pl) * kTP + c * 8 * kPK;
            __builtin_amdgcn_global_load_lds(src[q] + ks * kPK, (lds_void*)dst, 16, 0, 0);
        }
    };
    f32x16 acc[MA][MA];
#pragma unroll
    for (int a = 0; a < MA; ++a)
#pragma unroll
        for (int b = 0; b < MA; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    auto frag = [&](int buf, int pl, int row, int kk) {
        const int pos = (2 * kk + h) ^ ((row >> 1) & 7);
        return *reinterpret_cast<const bf16x8*>(sm + (buf * 4 + pl) * kTP + row * kPK + 8 * pos);
    };
    // One wave per SIMD: the next stage's 16 DMAs are issued in four groups between this
    // stage's MFMA groups, so their issue overlaps the MFMA pipe.  One barrier per stage: it
    // orders stage ks's DMAs (each wave drained its own with vmcnt(0) first) before any
    // fragment read, and every wave's reads of the buffer the next DMAs overwrite (stage ks-1's)
    // before those DMAs are issued.
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += NQ / 4) issue4(0, 0, q0);
    float dsc = 1.f;   // fp16 D2 scale (H), computed under the first stage's DMAs
    if constexpr (H) {
        __shared__ float red[4];
        dsc = tile_d2_scale<256>(nrm, n, red);
        if (threadIdx.x == 0) *d2s = dsc;
    }
    for (int ks = 0; ks < nks; ++ks) {
        const int buf = ks & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's stage-ks DMAs
        __builtin_amdgcn_s_barrier();                          // every wave's
        const bool more = ks + 1 < nks;
#pragma unroll
        for (int kk = 0; kk < kPK / 16; ++kk) {
            if (more) issue4(ks + 1, buf ^ 1, (NQ / 4) * kk);
            bf16x8 ah[MA], al[MA], bh[MA], bl[MA];
#pragma unroll
            for (int m = 0; m < MA; ++m) {
                ah[m] = frag(buf, 0, wr * (TS / 2) + m * 32 + r, kk);
                al[m] = frag(buf, 1, wr * (TS / 2) + m * 32 + r, kk);
                bh[m] = frag(buf, 2, wc * (TS / 2) + m * 32 + r, kk);
                bl[m] = frag(buf, 3, wc * (TS / 2) + m * 32 + r, kk);
            }
#pragma unroll
            for (int a = 0; a < MA; ++a)
#pragma unroll
                for (int b = 0; b < MA; ++b) {
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
                }
        }
    }
    __syncthreads();   // the last stage's reads are done before the diagonal epilogue reuses sm
    // epilogue: D2 = |a_i|^2 + |a_j|^2 - 2 <a_i, a_j>; C layout of 32x32: col = lane & 31,
    // row = (e & 3) + 8 (e >> 2) + 4 h
    float nj[MA];
#pragma unroll
    for (int b = 0; b < MA; ++b) {
        const int j = bj * TS + wc * (TS / 2) + b * 32 + r;
        nj[b] = nrm[j < n ? j : n - 1];
    }
    if (bi != bj) {
#pragma unroll
        for (int a = 0; a < MA; ++a) {
            const int i0 = bi * TS + wr * (TS / 2) + a * 32;
            float ni[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int i = i0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                ni[e] = nrm[i < n ? i : n - 1];
            }
#pragma unroll
            for (int b = 0; b < MA; ++b) {
                const int j = bj * TS + wc * (TS / 2) + b * 32 + r;
                float dv[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) dv[e] = ni[e] + nj[b] - 2.f * acc[a][b][e];
#pragma unroll
                for (int e = 0; e < 16; ++e) {   // direct: 32 lanes per 128-B row piece
                    const int i = i0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (i < n && j < n) dput<H>(D2, size_t(i) * ld + j, dv[e], dsc);
                }
                if (j < n) {   // mirrored: row j, columns i0 + 8 g + 4 h .. +3
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int i = i0 + 8 * g + 4 * h;
                        const size_t o = size_t(j) * ld + i;
                        if (i + 4 <= n) {
                            dput4<H>(D2, o, f32x4{dv[4 * g], dv[4 * g + 1], dv[4 * g + 2], dv[4 * g + 3]}, dsc);
                        } else {
#pragma unroll
                            for (int t = 0; t < 4; ++t)
                                if (i + t < n) dput<H>(D2, o + t, dv[4 * g + t], dsc);
                        }
                    }
                }
            }
        }
    } else {
        // diagonal tile: stage [TS][TS + 1] in LDS, store the upper triangle in both orientations
        float* tile = reinterpret_cast<float*>(sm);
        constexpr int LT = TS + 1;
#pragma unroll
        for (int a = 0; a < MA; ++a)
#pragma unroll
            for (int b = 0; b < MA; ++b)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int ti = wr * (TS / 2) + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    const int tj = wc * (TS / 2) + b * 32 + r;
                    const int i = bi * TS + ti;
                    tile[ti * LT + tj] = nrm[i < n ? i : n - 1] + nj[b] - 2.f * acc[a][b][e];
                }
        __syncthreads();
        for (int q = threadIdx.x; q < TS * TS; q += 256) {
            const int ti = q / TS, tj = q % TS;
            const int i = bi * TS + ti, j = bi * TS + tj;
            if (i < n && j < n) dput<H>(D2, size_t(i) * ld + j, tj >= ti ? tile[ti * LT + tj] : tile[tj * LT + ti], dsc);
        }
    }
}

// --------------------------------------------------------------------------------------
// K1b: per-row selection + exact re-rank + reverse scatter
// --------------------------------------------------------------------------------------
// A row of D2 as the select reads it: fp32, or fp16 x s decoded x 1/s (H, the pre-split route;
// 1/s is a power of two, so decoding adds no rounding).  Element offsets, 4-aligned for ld4.
template <bool H>
struct D2Row {
    const char* base;
    float inv;
    __device__ __forceinline__ f32x4 ld4(size_t e) const {
        if constexpr (H) {
            const h16x4 v = *reinterpret_cast<const h16x4*>(base + 2 * e);
            return f32x4{float(v.x) * inv, float(v.y) * inv, float(v.z) * inv, float(v.w) * inv};
        } else {   // streamed once per select: nontemporal (stress select 171 -> 153 us,
                   // profiles/r04s_ab_nt.txt)
            return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(base + 4 * e));
        }
    }
    __device__ __forceinline__ float ld1(size_t e) const {
        if constexpr (H) return float(*reinterpret_cast<const _Float16*>(base + 2 * e)) * inv;
        else return *reinterpret_cast<const float*>(base + 4 * e);
    }
};

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

// Threshold scan: each lane keeps only its TOP smallest D2 bits (min/max network, ~2 VALU per
// slot, against the ~35 of the sorted 64-bit list insert it replaced -- that select was VALU-issue
// bound), T = the kc-th smallest of the 64 x TOP lane entries by bisection -- at least kc distinct
// columns are <= T, so the kc-th smallest D2 is too -- and every column with D2 bits <= T is
// compacted into the wave's LDS slots.  Simulated at kc = 13 / n = 1,000 (TOP = 2) the set
// averages 13.2 columns, at kc = 32 / n = 1,500 (TOP = 3) 32.4; kc = 37 / n = 8,192 (stress,
// TOP = 5) holds ~0.6 of the kc nearest per lane -- five slots, not four, leave fewer rows
// with a full lane list and so a second read (stress select 151 -> 145 us,
// profiles/r04f8_ab_top5.txt).  CH > 0: the row (n <= 1024 CH) stays in
// registers between the two passes; CH = 0 re-reads it (L2 / MALL-hot).  Returns true when more
// than 64 columns tie in (the caller runs select_fallback, tb = T on return).  tb: D2 bits every
// left-out column is >= to (+inf when every valid column is a candidate).
constexpr int kSelNB = 4;   // float4 per lane per 1024-column chunk of a D2 row

// Loads of CH 1024-column chunks of D2 row `row` (sum of NP planes), clamped past ld.
template <int NP, int CH, bool H = false>
__device__ __forceinline__ void load_d2_row(const D2Row<H>& row, size_t plane, int ld,
                                            f32x4 (&v)[CH * kSelNB]) {
    const int lane = lane_id();
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int b = 0; b < kSelNB; ++b) {
            const int j0 = c * 4 * kWave * kSelNB + 4 * (b * kWave + lane);
            const int jc = j0 < ld ? j0 : 0;
            v[c * kSelNB + b] = row.ld4(jc);
#pragma unroll
            for (int p = 1; p < NP; ++p)
                v[c * kSelNB + b] += row.ld4(p * plane + jc);
        }
}

template <int TOP, int NP, int CH, bool H = false>
__device__ __forceinline__ bool select_threshold(const D2Row<H>& row, size_t plane,
                                                 int n, int ld, int i, int kc,
                                                 int* __restrict__ cand,
                                                 uint32_t* __restrict__ cgd, int& ci, int& kce,
                                                 uint32_t& tb, uint32_t& gbits,
                                                 const f32x4 (&vin)[CH > 0 ? CH * kSelNB : 1]) {
    constexpr int NB = kSelNB;
    constexpr int HV = CH > 0 ? CH * NB * 4 : 1;
    const int lane = lane_id();
    uint32_t m[TOP];
    int mj[CH > 0 ? 1 : TOP];   // CH = 0: the columns of the lane's TOP smallest
#pragma unroll
    for (int t = 0; t < TOP; ++t) m[t] = 0xFFFFFFFFu;
#pragma unroll
    for (int t = 0; t < (CH > 0 ? 1 : TOP); ++t) mj[t] = -1;
    uint32_t hv[HV];
    auto load_chunk = [&](int jb, f32x4 (&v)[NB]) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int j0 = jb + 4 * (b * kWave + lane);
            const int jc = j0 < ld ? j0 : 0;
            v[b] = row.ld4(jc);
#pragma unroll
            for (int p = 1; p < NP; ++p) v[b] += row.ld4(p * plane + jc);
        }
    };
    auto bits_of = [&](float x, int j) -> uint32_t {   // invalid: 0xFFFFFFFF (> any T)
        return (j < n && j != i && x == x) ? __float_as_uint(x > 0.f ? x : 0.f) : 0xFFFFFFFFu;
    };
    int nvalid = 0;
    // pass 1: per-lane TOP smallest
    auto absorb = [&](uint32_t u) {
        nvalid += u != 0xFFFFFFFFu ? 1 : 0;
#pragma unroll
        for (int t = 0; t < TOP; ++t) {
            const uint32_t lo = m[t] < u ? m[t] : u;
            u = m[t] < u ? u : m[t];
            m[t] = lo;
        }
    };
    auto absorb_j = [&](uint32_t u, int j) {   // the same network carrying the column
        nvalid += u != 0xFFFFFFFFu ? 1 : 0;
#pragma unroll
        for (int t = 0; t < (CH > 0 ? 1 : TOP); ++t) {
            const bool sw = u < m[t];
            const uint32_t mt = m[t];
            const int jt = mj[t];
            m[t] = sw ? u : mt;
            mj[t] = sw ? j : jt;
            u = sw ? mt : u;
            j = sw ? jt : j;
        }
    };
    if constexpr (CH > 0) {   // the row was loaded by the caller (prefetched under the last row)
#pragma unroll
        for (int c = 0; c < CH; ++c) {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t u = bits_of(vin[c * NB + b][t], c * 4 * kWave * NB + 4 * (b * kWave + lane) + t);
                    hv[(c * NB + b) * 4 + t] = u;
                    absorb(u);
                }
        }
    } else {
        for (int jb = 0; jb < n; jb += 4 * kWave * NB) {
            f32x4 v[NB];
            load_chunk(jb, v);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int j = jb + 4 * (b * kWave + lane) + t;
                    absorb_j(bits_of(v[b][t], j), j);
                }
        }
    }
    GLL_TRACE_PT(16);
    auto count_le = [&](uint32_t t) {
        int c = 0;
#pragma unroll
        for (int s = 0; s < TOP; ++s) c += __popcll(__ballot(m[s] <= t));
        return c;
    };
    uint32_t T = 0xFFFFFFFEu;   // fewer than kc valid entries: every valid column
    if (count_le(T) >= kc) {
        // between the smallest entry and the largest valid one
        uint32_t top = 0;
#pragma unroll
        for (int s = 0; s < TOP; ++s) top = m[s] != 0xFFFFFFFFu ? m[s] : top;
        uint32_t lo = wave_min_u32(m[0]), up = wave_max_u32(top);
        // a T with count_le(T) >= kc (wave-uniform, <= 32 steps); one holding exactly kc list
        // entries ends the search early -- any such T leaves the same list entries in the set
        // (left-out columns stay covered by tb = T + 1, and the kNN is exact either way)
        while (lo < up) {
            const uint32_t mid = lo + ((up - lo) >> 1);
            const int c = count_le(mid);
            if (c == kc) {
                up = mid;
                break;
            }
            if (c > kc) up = mid;
            else lo = mid + 1u;
        }
        T = up;
    }
    // pass 2: compact every column <= T.  CH = 0 (rows re-read from memory): when no lane may
    // hold more columns <= T than its TOP list (a lane whose whole list is <= T while it saw
    // more columns), the lists ARE that set and the row is not read again -- stress: the second
    // read was 22 of a wave's 81 us (profiles/r04p_trace_stress.txt)
    int base = 0, mine = 0;
    auto emit = [&](uint32_t u, int j) {
        const bool p = u <= T;
        const uint64_t mk = __ballot(p);
        const int pos = base + lanes_below(mk);
        if (p && pos < kWave) {
            cand[pos] = j;
            cgd[pos] = u;
        }
        mine += p ? 1 : 0;
        base += __popcll(mk);
    };
    if constexpr (CH > 0) {
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    emit(hv[(c * NB + b) * 4 + t], c * 4 * kWave * NB + 4 * (b * kWave + lane) + t);
    } else if (__ballot(m[TOP - 1] <= T && nvalid > TOP) == 0ull) {
#pragma unroll
        for (int t = 0; t < (CH > 0 ? 1 : TOP); ++t) emit(m[t], mj[t]);
    } else {
        for (int jb = 0; jb < n; jb += 4 * kWave * NB) {
            f32x4 v[NB];
            load_chunk(jb, v);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int j = jb + 4 * (b * kWave + lane) + t;
                    emit(bits_of(v[b][t], j), j);
                }
        }
    }
    const bool redo = base > kWave;
    tb = redo ? T : (__ballot(mine != nvalid) == 0 ? 0x7F800000u : T + 1u);
    __builtin_amdgcn_wave_barrier();   // a wave's LDS ops run in order: the reads see the stores
    asm volatile("" ::: "memory");
    kce = base;
    ci = (!redo && lane < base) ? cand[lane] : -1;
    gbits = (!redo && lane < base) ? cgd[lane] : 0xFFFFFFFFu;
    return redo;
}

// Fallback of the threshold scan when more than 64 columns have D2 bits <= T (ties: duplicate
// points): T' = the kc-th smallest D2 bits of the whole row, by bisection on full-row counts in
// [0, T] (the scan's T already has >= kc columns at or below it; <= 31 passes over the hot row,
// rare), then every column below T' -- fewer than kc -- and columns at T' in index order up to
// 64 slots.  Every column left out is >= T' (tb).  Registers: the scan's, no per-lane key lists
// (the 64-key exact merge it replaces held 128 VGPRs and set the select's occupancy).
template <int NP, bool H = false>
__device__ __forceinline__ void select_fallback(const D2Row<H>& row, size_t plane, int n, int ld,
                                                int i, int kc, int* __restrict__ cand,
                                                uint32_t* __restrict__ cgd, int& ci, int& kce,
                                                uint32_t& tb, uint32_t& gbits) {
    constexpr int NB = kSelNB;
    const int lane = lane_id();
    auto bits_of = [&](float x, int j) -> uint32_t {
        return (j < n && j != i && x == x) ? __float_as_uint(x > 0.f ? x : 0.f) : 0xFFFFFFFFu;
    };
    auto wave_count_le = [&](uint32_t thr) {   // wave-uniform
        int c = 0;
        for (int jb = 0; jb < n; jb += 4 * kWave * NB) {
            f32x4 v[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int j0 = jb + 4 * (b * kWave + lane);
                const int jc = j0 < ld ? j0 : 0;
                v[b] = row.ld4(jc);
#pragma unroll
                for (int p = 1; p < NP; ++p) v[b] += row.ld4(p * plane + jc);
            }
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    c += __popcll(__ballot(bits_of(v[b][t], jb + 4 * (b * kWave + lane) + t) <= thr));
        }
        return c;
    };
    uint32_t lo = 0u, up = tb;   // count_le(tb) >= kc (select_threshold's T)
    while (lo < up) {   // smallest T' with count_le(T') >= kc (wave-uniform)
        const uint32_t mid = lo + ((up - lo) >> 1);
        if (wave_count_le(mid) >= kc) up = mid;
        else lo = mid + 1u;
    }
    const uint32_t T = up;
    // columns below T' (any order), then ties at T' in index order: lane-contiguous columns
    int base = 0;
    auto emit = [&](bool p, uint32_t u, int j) {
        const uint64_t mk = __ballot(p);
        const int pos = base + lanes_below(mk);
        if (p && pos < kWave) {
            cand[pos] = j;
            cgd[pos] = u;
        }
        base += __popcll(mk);
    };
    for (int j0 = 0; j0 < n; j0 += kWave) {
        const int j = j0 + lane;
        float x = 0.f;
        if (j < n) {
            x = row.ld1(j);
#pragma unroll
            for (int p = 1; p < NP; ++p) x += row.ld1(p * plane + j);
        }
        const uint32_t u = bits_of(x, j);
        emit(u < T, u, j);
    }
    for (int j0 = 0; j0 < n && base < kWave; j0 += kWave) {
        const int j = j0 + lane;
        float x = 0.f;
        if (j < n) {
            x = row.ld1(j);
#pragma unroll
            for (int p = 1; p < NP; ++p) x += row.ld1(p * plane + j);
        }
        const uint32_t u = bits_of(x, j);
        emit(u == T, u, j);
    }
    tb = T;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    kce = base < kWave ? base : kWave;
    ci = lane < kce ? cand[lane] : -1;
    gbits = lane < kce ? cgd[lane] : 0xFFFFFFFFu;
}

// 64-bit DPP add of the 8-lane group butterfly (two 32-bit moves per stage).
template <int CTRL>
__device__ __forceinline__ double dpp_add_d(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_update_dpp(0, uint32_t(b), CTRL, 0xf, 0xf, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0, uint32_t(b >> 32), CTRL, 0xf, 0xf, false);
    return v + __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}
__device__ __forceinline__ double group8_sum_d(double v) {
    v = dpp_add_d<0xB1>(v);
    v = dpp_add_d<0x4E>(v);
    v = dpp_add_d<0x141>(v);
    return v;
}
__device__ __forceinline__ double shfl_d(double v, int src) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = uint32_t(__shfl(int(uint32_t(b)), src));
    const uint32_t hi = uint32_t(__shfl(int(uint32_t(b >> 32)), src));
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(b), l);
    const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(b >> 32), l);
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}

// Exact squared distances d(i, c_L)^2 = sum_k (x_ik - x_jk)^2 for the candidates c_L held by
// lanes L in [lo, hi) (ci = -1: no candidate), 8 lanes per candidate across d, PG groups of 8
// candidates per sweep with every load in flight.  ACC = float: fp32 differences and sums
// (the fast path); ACC = double: float64 differences and sums -- the reference's stand-in
// ranks in float64 -- used where fp32 cannot separate two candidates.  Either
// way the (i, j) and (j, i) sums run the same lane mapping on negated differences: bitwise
// symmetric for the same ACC.  Lanes outside [lo, hi) keep `ce`.
// FULL: d is a multiple of 32 NU, so every feature step is in range -- no clamped addresses and
// no masks (the masked form adds exact zeros there: the same sums bit for bit).  Single-graph
// selects: NS 12.4 -> 11.7-12.1 us, FullySup 22.0 -> 21.3-21.5 us, stress unchanged
// (profiles/r05zx_ab_select_unmasked_gated.txt).
template <bool VEC, int PG, typename ACC, int NU, bool XL, bool FULL, bool SPLIT = false>
__device__ __forceinline__ ACC exact_d2_body(const float* __restrict__ X,
                                             const float* __restrict__ xi, int i, int d, int ci,
                                             int lo, int hi, ACC ce, const float* xs) {
    constexpr bool F64 = std::is_same<ACC, double>::value;
    const int lane = lane_id();
    const int grp = lane >> 3, sub = lane & 7;
    for (int p0 = lo; p0 < hi; p0 += 8 * PG) {
        const float* xj[PG];
#pragma unroll
        for (int g2 = 0; g2 < PG; ++g2) {
            const int idx = p0 + 8 * g2 + grp;
            const int j = __shfl(ci, idx < hi ? idx : lo);
            const bool live = idx < hi && j >= 0;
            xj[g2] = X + size_t(live ? j : i) * d;
        }
        ACC part[PG];
#pragma unroll
        for (int g2 = 0; g2 < PG; ++g2) part[g2] = ACC(0);
        // one step of NU x 32 features, every load in flight; F: no masks (in range)
        auto step = [&](const int kb, auto full) {
            constexpr bool F = decltype(full)::value;
            f32x4 va[NU], vb[PG][NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) {   // straight-line: every load issued before use
                const int k = kb + 32 * u + 4 * sub;
                if constexpr (F) {
                    if constexpr (!XL) va[u] = *reinterpret_cast<const f32x4*>(xi + k);
#pragma unroll
                    for (int g2 = 0; g2 < PG; ++g2)
                        vb[g2][u] = *reinterpret_cast<const f32x4*>(xj[g2] + k);
                } else {
                    if constexpr (!XL) va[u] = load4_raw<VEC>(xi, k, d);
#pragma unroll
                    for (int g2 = 0; g2 < PG; ++g2) vb[g2][u] = load4_raw<VEC>(xj[g2], k, d);
                }

            }
#pragma unroll
            for (int g2 = 0; g2 < PG; ++g2) {
#pragma unroll
                for (int u = 0; u < NU; ++u) {   // same order from either end: symmetric
                    const int k = kb + 32 * u + 4 * sub;
                    if constexpr (XL)   // x_i from the wave's LDS copy, read at use
                        va[u] = *reinterpret_cast<const f32x4*>(xs + k);
                    if constexpr (F64) {
                        const f32x4 a = F ? va[u] : mask4<VEC>(va[u], k, d);
                        const f32x4 b = F ? vb[g2][u] : mask4<VEC>(vb[g2][u], k, d);
                        const double d0 = double(a.x) - double(b.x), d1 = double(a.y) - double(b.y);
                        const double d2 = double(a.z) - double(b.z), d3 = double(a.w) - double(b.w);
                        part[g2] = __builtin_fma(d0, d0, part[g2]);
                        part[g2] = __builtin_fma(d1, d1, part[g2]);
                        part[g2] = __builtin_fma(d2, d2, part[g2]);
                        part[g2] = __builtin_fma(d3, d3, part[g2]);
                    } else {
                        // explicit fma chain: contraction left to the compiler differed
                        // between instantiations (packed multiplies, then adds), and with it
                        // the last bit of d^2 between the select's two forms
                        const f32x4 df = F ? va[u] - vb[g2][u] : mask4<VEC>(va[u] - vb[g2][u], k, d);
                        part[g2] = __builtin_fmaf(df.x, df.x, part[g2]);
                        part[g2] = __builtin_fmaf(df.y, df.y, part[g2]);
                        part[g2] = __builtin_fmaf(df.z, df.z, part[g2]);
                        part[g2] = __builtin_fmaf(df.w, df.w, part[g2]);
                    }
                }
            }
        };
        if constexpr (FULL) {
            for (int kb = 0; kb < d; kb += 32 * NU) step(kb, std::true_type{});
        } else if constexpr (SPLIT) {
            // the whole steps unmasked, then at most one masked step
            const int df = d - d % (32 * NU);
            int kb = 0;
            for (; kb < df; kb += 32 * NU) step(kb, std::true_type{});
            if (kb < d) step(kb, std::false_type{});
        } else {
            for (int kb = 0; kb < d; kb += 32 * NU) step(kb, std::false_type{});
        }
#pragma unroll
        for (int g2 = 0; g2 < PG; ++g2) {
            ACC tot;
            if constexpr (F64) tot = group8_sum_d(part[g2]);
            else tot = group8_sum(part[g2]);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                ACC v;
                if constexpr (F64) v = readlane_d(tot, 8 * g);
                else v = readlane_f(tot, 8 * g);
                if (lane == p0 + 8 * g2 + g) ce = v;
            }
        }
    }
    return ce;
}

template <bool VEC, int PG, typename ACC, int NU = 16, bool XL = false>
__device__ __forceinline__ ACC exact_d2(const float* __restrict__ X, const float* __restrict__ xi,
                                        int i, int d, int ci, int lo, int hi, ACC ce,
                                        const float* xs = nullptr) {
    // only the single-graph sweep (NU = 16): in the occupancy forms (x_i in LDS, <= 64 / 80
    // VGPRs, NU = 4) a second body -- theirs or the rescan's / refinement's -- spilled (B = 64 NS
    // select 159 -> 186 us, profiles/r05zw_ab_select_unmasked.txt).  Those take SPLIT instead:
    // one body, whole steps unmasked and at most one masked step (B = 64 NS select 161 -> 148 us,
    // FullySup 332 -> 315 us, profiles/r05zy_ab_select_split_b64.txt)
    if constexpr (VEC && !XL && NU >= 16)
        if (d % (32 * NU) == 0)
            return exact_d2_body<VEC, PG, ACC, NU, XL, true>(X, xi, i, d, ci, lo, hi, ce, xs);
    return exact_d2_body<VEC, PG, ACC, NU, XL, false, VEC && XL>(X, xi, i, d, ci, lo, hi, ce, xs);
}

// Rank of this lane's (exact d^2, index) key among lanes [0, cnt); lanes without a candidate
// (ci < 0) sort last.
__device__ __forceinline__ int key_rank(double ce, int ci, int cnt) {
    const int me = ci < 0 ? INT_MAX : ci;
    int rank = 0;
    for (int u = 0; u < cnt; ++u) {
        const double du = readlane_d(ce, u);
        const int iu0 = __builtin_amdgcn_readlane(ci, u);
        const int iu = iu0 < 0 ? INT_MAX : iu0;
        rank += (du < ce || (du == ce && iu < me)) ? 1 : 0;
    }
    return rank;
}

// Conservative bound on |D2_gram(i, j) - d(i, j)^2| for the split-bf16 Gram over centred rows
// a = x - x_0: the dropped lo*lo terms and the bf16 rounding of lo (<= 3 * 2^-18 |a_k b_k|,
// doubled by the -2<a, b> term: 2^-15.4 |a||b|), plus fp32 accumulation at the kernels'
// depth (<= 3d/16 MFMA steps: 2^-24 * 3d/16 * 2 |a||b|, 1.1e-5 |a||b| at d = 1024) and the
// rounding of the centring and of the norms -- all below 2^-13 (|a| + |b|)^2 >= 2^-11 |a||b|
// for d <= 8192 (gll.h caps d at 4096).
constexpr double kGramErr = 1.0 / 8192.0;

// Float64 re-rank of the candidate list (rare: fp32 cannot separate the boundary pair); a
// shallow load pipeline (4 steps in flight) keeps its registers under the common path's.
template <bool VEC>
__device__ __forceinline__ double refine_d2(const float* __restrict__ X, const float* __restrict__ xi,
                                            int i, int d, int ci, int kce) {
    return exact_d2<VEC, 1, double, 4>(X, xi, i, d, ci, 0, kce, __builtin_inf());
}

struct KnnPick {
    double d;   // exact d^2 (float64)
    int j;      // column, -1: none
};

// Exact rescan of every column with D2_gram <= thr (the certificate failed): candidates in
// chunks of up to 64 - (K-1) lanes, float64 distances, the K-1 best (by d^2, index) carried
// in lanes 0..K-2 across chunks (rare path, shallow load pipeline).
template <bool VEC, int NP, bool H = false>
__device__ __forceinline__ KnnPick knn_rescan(const D2Row<H>& row, size_t plane, int n,
                                           int i, const float* __restrict__ X,
                                           const float* __restrict__ xi, int d, int K,
                                           double thr, int* s_cand) {
    const int lane = lane_id();
    const int F = kWave - (K - 1);          // free lanes per chunk (launch: K-1 <= 56)
    int bi = -1;                             // running best: lanes 0..K-2
    double bd = __builtin_inf();
    for (int jb = 0; jb < n; jb += kWave) {
        const int j = jb + lane;
        float v = 0.f;
        if (j < n) {
            v = row.ld1(j);
#pragma unroll
            for (int p = 1; p < NP; ++p) v += row.ld1(p * plane + j);
        }
        bool take = j < n && j != i && v == v && double(v) <= thr;
        uint64_t mask = __ballot(take);
        while (mask) {
            const int pos = lanes_below(mask);
            const bool sel = take && pos < F;
            if (sel) s_cand[pos] = j;
            const int cnt = __popcll(__ballot(sel));
            mask &= ~__ballot(sel);
            take = take && !sel;
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const int off = lane - (K - 1);
            const int cc = lane < K - 1 ? bi : (off < cnt ? s_cand[off] : -1);
            double cd = lane < K - 1 ? bd : __builtin_inf();
            cd = exact_d2<VEC, 1, double, 4>(X, xi, i, d, cc, K - 1, K - 1 + cnt, cd);
            if (cc < 0) cd = __builtin_inf();
            const int rk = key_rank(cd, cc, K - 1 + cnt);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            // keep the K-1 best in rank order: the lane holding rank L goes to LDS slot L
            const uint64_t live = __ballot(lane < K - 1 + cnt && rk < K - 1 && cc >= 0);
            if (((live >> lane) & 1ull) != 0) s_cand[rk] = lane;
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const int nl = __popcll(live);
            const int src = lane < nl ? s_cand[lane] : lane;
            const int nbi = __shfl(cc, src);
            const double nbd = shfl_d(cd, src);
            bi = lane < nl ? nbi : -1;
            bd = lane < nl ? nbd : __builtin_inf();
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
    }
    return KnnPick{bd, bi};
}

// XQ > 0: x_i staged in LDS, d <= 256 XQ.  CH > 0 (KC <= 32): n <= 1024 CH, the D2 row held in
// registers by the threshold scan.
template <int KC, bool VEC, int NP, int PG, int NU, int XQ = 0, bool R = false, int CH = 0,
          bool H = false>
// Occupancy forms (x_i in LDS): NU = 8 load steps at 6 waves per SIMD (<= 80 VGPRs), NU = 4 at
// 8 waves per SIMD (<= 64 VGPRs).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(XQ > 0 ? (NU <= 4 ? 8 : (NU <= 8 ? 6 : 1)) : 1)))
void knn_select_kernel(
    const float* __restrict__ D2, int ld, size_t plane, const float* __restrict__ X, int n, int d, int K,
    int kc, float eps_fixed, int auto_eps, int RCAP, int32_t* __restrict__ knn_idx,
    float* __restrict__ knn_d2, float* __restrict__ eps, int32_t* __restrict__ rev_cnt,
    int32_t* __restrict__ rev_idx, float* __restrict__ rev_d2, int32_t* __restrict__ ovf,
    int32_t* __restrict__ status, int32_t* __restrict__ status_pub, size_t xs, size_t wss,
    size_t sts, int r0, int r1, const float* __restrict__ d2s, const int32_t* __restrict__ perm) {
    GLL_TRACE_SCOPE(1);
    GLL_TRACE_PT(20);
    const int2 gxy = batch_xy<R>();   // once (per pointer it re-reads gridDim and divides)
    D2 = gshift_at(D2, wss, gxy.y);
    X = gshift_at(X, xs, gxy.y);
    knn_idx = gshift_at(knn_idx, wss, gxy.y);
    knn_d2 = gshift_at(knn_d2, wss, gxy.y);
    eps = gshift_at(eps, wss, gxy.y);
    rev_cnt = gshift_at(rev_cnt, wss, gxy.y);
    rev_idx = gshift_at(rev_idx, wss, gxy.y);
    rev_d2 = gshift_at(rev_d2, wss, gxy.y);
    ovf = gshift_at(ovf, wss, gxy.y);
    status = gshift_at(status, wss, gxy.y);
    status_pub = gshift_at(status_pub, sts, gxy.y);
    d2s = gshift_at(d2s, wss, gxy.y);
    __shared__ int s_cand[4][kWave];
    __shared__ uint32_t s_cgd[4][kWave];
    constexpr bool XL = XQ > 0;
    __shared__ float s_xi[XL ? 4 : 1][XL ? 256 * XQ : 1];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    // rows r0 .. r1 - 1: all, or a panel (D2 row i - r0); with a locality order (one large graph,
    // no panels) block b takes positions of the order dealt XCD-contiguously (xcd_tile): each
    // XCD works through a run of rows whose neighbours mostly lie in that same run
    int i;
    if (perm) {
        const int sl = xcd_tile(int(blockIdx.x), int(gridDim.x)) * 4 + wv;
        if (sl >= r1) return;  // whole wave
        i = perm[sl];
    } else {
        i = r0 + gxy.x * 4 + wv;
        if (i >= r1) return;  // whole wave
    }
    // XL: x_i is staged once in LDS by LDS-DMA (global_load_lds: no registers held across the
    // D2 scan -- round 3 staged it through 4 XQ VGPRs that stayed live until the scan ended), so
    // the exact distances hold only the candidates' rows in registers (occupancy) and do not
    // re-load x_i per sweep.  Lanes past d re-read the row's first 16 B (in bounds; the features
    // past d are masked at use).
    if constexpr (XL) {
        const float* xg = X + size_t(i) * d;
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            const int k = 4 * lane + 256 * q;
            __builtin_amdgcn_global_load_lds(xg + (k < d ? k : 0), (lds_void*)&s_xi[wv][256 * q],
                                             16, 0, 0);
        }
    }

    // 1-2) candidates: short per-lane lists + threshold merge, exact re-run when inexact.
    //      tb: D2 bits every non-candidate column is >= to (+inf: all valid columns taken)
    // fp16 storage (H): decoded x 1/s; its rounding widens every Gram error bound below by
    // rho (relative, half an fp16 ulp) plus sub (absolute, half the smallest subnormal step)
    const float dsc = H ? *d2s : 1.f;   // written by every tile of the GEMM (the same value)
    const D2Row<H> row{reinterpret_cast<const char*>(D2) + size_t(i - r0) * ld * (H ? 2 : 4),
                       1.f / dsc};
    const double rho = H ? 1.0 / 2048.0 : 0.0;
    const double sub = H ? 0x1p-25 / double(dsc) : 0.0;
    // bounds between a true Gram value v and its stored decoding t: |t - v| <= rho |v| + sub
    auto up = [&](double t) { return H ? t + 2.0 * rho * fabs(t) + sub : t; };   // >= v
    auto lo = [&](double t) { return H ? t - 2.0 * rho * fabs(t) - sub : t; };   // <= v
    int ci, kce;
    uint32_t tb, gb;   // gb: this lane's candidate's Gram D2 bits
    {
        f32x4 vrow[CH > 0 ? CH * kSelNB : 1];
        if constexpr (CH > 0) load_d2_row<NP, CH, H>(row, plane, ld, vrow);
        constexpr int TOP = KC == 16 ? 2 : (KC == 32 ? 3 : 5);
        const bool redo = select_threshold<TOP, NP, CH, H>(row, plane, n, ld, i, kc, s_cand[wv],
                                                           s_cgd[wv], ci, kce, tb, gb, vrow);
        GLL_TRACE_PT(17);
        if (redo) {
            if (lane == 0) atomicAdd(&status_pub[GLL_ST_KNN_MERGE], 1);
            select_fallback<NP, H>(row, plane, n, ld, i, kc, s_cand[wv], s_cgd[wv], ci, kce, tb, gb);
        }
    }
    // 2b) drop the candidates the Gram's error bound already rules out, before their exact
    //     distances are computed (each is a d-float row gather): with G = the (K-1)-th smallest
    //     Gram D2 among the candidates and B its error bound (kGramErr, below), the exact
    //     (K-1)-th distance is <= G + B, and a column whose exact d^2 is below that has Gram
    //     D2 < G + 2B; candidates above G + 2B join the left-out columns (tb) that the
    //     certificate of step 5 covers.  NS: 16 candidates -> ~9-10 re-ranked.
    if (K >= 2 && kce > K - 1) {
        const float g = ci >= 0 && lane < kce ? __uint_as_float(gb) : __builtin_inff();
        int grk = 0;   // rank of (g, index) among the candidates
        for (int u = 0; u < kce; ++u) {
            const float gu = readlane_f(g, u);
            const int cu = __builtin_amdgcn_readlane(ci, u);
            grk += (gu < g || (gu == g && cu < ci)) ? 1 : 0;
        }
        const uint64_t kb = __ballot(lane < kce && ci >= 0 && grk == K - 2);
        if (kb) {
            const double G = up(double(readlane_f(g, int(__builtin_ctzll(kb)))));
            float a2 = row.ld1(0);
#pragma unroll
            for (int p = 1; p < NP; ++p) a2 += row.ld1(p * plane);
            const double ai = sqrt(up(double(a2 > 0.f ? a2 : 0.f)));
            const double gp = G > 0.0 ? G : 0.0;
            const double b0 = kGramErr * (2.0 * ai + sqrt(gp)) * (2.0 * ai + sqrt(gp));
            const double r1 = 2.0 * ai + sqrt(gp + b0);
            const double thr = up(G + 2.0 * kGramErr * r1 * r1);   // in stored units
            const bool need = lane < kce && ci >= 0 && (grk < K - 1 || double(g) <= thr);
            const bool drop = lane < kce && ci >= 0 && !need;
            // the smallest dropped Gram D2 joins the left-out bound
            const uint32_t dmin = wave_min_u32(drop ? gb : 0xFFFFFFFFu);
            if (dmin < tb) tb = dmin;
            const uint64_t nm = __ballot(need);
            if (need) s_cand[wv][lanes_below(nm)] = ci;
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            kce = __popcll(nm);
            ci = lane < kce ? s_cand[wv][lane] : -1;
        }
    }
    // 3) exact squared distances of the candidates, fp32.  PG passes per sweep for single
    //    graphs (one wave per SIMD anyway); batches keep PG = 1 (register pressure).
    const float* xi = X + size_t(i) * d;
    // the LDS-DMA copy of x_i (issued at entry) has landed: DMA writes count in vmcnt, which
    // the compiler does not track for them
    if constexpr (XL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double ce = double(exact_d2<VEC, PG, float, NU, XL>(X, xi, i, d, ci, 0, kce,
                                                        __builtin_inff(), &s_xi[wv][0]));
    GLL_TRACE_PT(18);
    if (ci < 0) ce = __builtin_inf();
    // 4) rank the candidates by (exact d^2, index); keep the K-1 nearest
    int rank = key_rank(ce, ci, kce);
    //    fp32 sums of d terms carry <= (d/8 + 3) 2^-24 relative error: where the pair at the
    //    set boundary (ranks K-2 | K-1) -- or, for auto eps, the pair that decides the kth
    //    neighbour (K-3 | K-2) -- is closer than 4x that, rank again in float64
    {
        const double tol = double(d / 8 + 16) * (1.0 / 4194304.0);
        auto at_rank = [&](int r) -> double {
            const uint64_t b = __ballot(lane < kce && ci >= 0 && rank == r);
            return b ? readlane_d(ce, int(__builtin_ctzll(b))) : __builtin_inf();
        };
        bool tie = false;
        if (K >= 2 && kce > K - 1) {
            const double a = at_rank(K - 2), b = at_rank(K - 1);
            tie |= b - a <= tol * b;
        }
        if (auto_eps && K >= 3) {
            const double a = at_rank(K - 3), b = at_rank(K - 2);
            tie |= b - a <= tol * b;
        }
        if (tie) {
            ce = refine_d2<VEC>(X, xi, i, d, ci, kce);
            if (ci < 0) ce = __builtin_inf();
            rank = key_rank(ce, ci, kce);
        }
    }
    bool keep = lane < kce && ci >= 0 && rank < K - 1;
    int nkeep = __popcll(__ballot(keep));

    // 5) certificate: every column left out has D2_gram >= tb; a left-out j that belongs in
    //    the K-1 nearest has d_ij^2 <= dK (the (K-1)-th exact distance found) and so
    //    |a_j| <= |a_i| + sqrt(dK), D2_gram <= dK + B with B = kGramErr (2|a_i| + sqrt(dK))^2.
    //    tb > dK + B rules that out.  |a_i|^2 = D2[i][0] (row 0 is the Gram's centre, a_0 = 0).
    //    Otherwise (rare: features far from row 0 relative to the neighbour gaps) every
    //    column with D2_gram <= dK + B is re-ranked exactly (knn_rescan).
    if (K >= 2 && nkeep == K - 1 && tb < 0x7F800000u) {
        const uint64_t kb = __ballot(keep && rank == K - 2);
        const double dK = readlane_d(ce, int(__builtin_ctzll(kb)));
        float a2 = row.ld1(0);
#pragma unroll
        for (int p = 1; p < NP; ++p) a2 += row.ld1(p * plane);
        const double ai = sqrt(up(double(a2 > 0.f ? a2 : 0.f)));
        const double r = 2.0 * ai + sqrt(dK);
        const double thr = dK + kGramErr * r * r;
        if (!(lo(double(__uint_as_float(tb))) > thr)) {
            if (lane == 0) atomicAdd(&status_pub[GLL_ST_KNN_RESCAN], 1);
            const KnnPick pk = knn_rescan<VEC, NP, H>(row, plane, n, i, X, xi, d, K, up(thr),
                                                      s_cand[wv]);
            ci = pk.j;
            ce = pk.d;
            kce = K - 1;
            rank = key_rank(ce, ci, kce);
            keep = lane < kce && ci >= 0 && rank < K - 1;
            nkeep = __popcll(__ballot(keep));
        }
    }
    int32_t* oi = knn_idx + size_t(i) * K;
    float* od = knn_d2 + size_t(i) * K;
    const float cef = float(ce);   // correctly rounded exact d^2
    if (lane == 0) {
        oi[0] = i;
        od[0] = 0.f;
    }
    if (keep) {
        oi[1 + rank] = ci;
        od[1 + rank] = cef;
    }
    // rows with fewer valid candidates (non-finite input) fall back to self at distance 0,
    // i.e. dropped edges (sparse.find drops zeros, GLL.py:198)
    if (lane >= nkeep && lane < K - 1) {
        oi[1 + lane] = i;
        od[1 + lane] = 0.f;
    }
    GLL_TRACE_PT(19);
    float ei = eps_fixed;
    if (auto_eps) {
        // eps_i = d(i, knn_ind[i, K-1])  (GLL.py:205)
        const float e = (keep && rank == K - 2) ? sqrtf(cef) : 0.f;
        ei = wave_sum_dpp(e);
    }
    if (lane == 0) {
        eps[i] = ei;
        if (!(ei >= 1e-10f)) atomicOr(&status_pub[GLL_ST_TINY_EPS], 1);  // GLL.py:240-241
    }
    // 5) reverse entry (ci, i) for every valid pair; zero distances never enter the graph
    if (keep && cef > 0.f) {
        const int pos = atomicAdd(&rev_cnt[ci], 1);
        if (pos < RCAP) {
            rev_idx[size_t(ci) * RCAP + pos] = i;
            rev_d2[size_t(ci) * RCAP + pos] = cef;
        } else {
            const int q = atomicAdd(&status[kStOvfCount], 1);
            ovf[3 * q + 0] = ci;
            ovf[3 * q + 1] = i;
            ovf[3 * q + 2] = __float_as_int(cef);
        }
    }
}

// --------------------------------------------------------------------------------------
// Wide kNN select (kMaxKm1 < K - 1 <= kMaxKm1Huge: k up to 257 incl. self, e.g. utils.laplace
// with knn_num = 64, 100 or 200, utils.py:574).  knn_select_kernel holds one candidate per lane, so
// its list (K - 1 plus a re-rank margin) and the rescan's lanes cap K - 1 at 56.  Here a wave
// keeps its row's candidates in LDS (kWideCap slots) and its running K - 1 nearest as a sorted
// list in LDS, and ranks in float64 throughout:
//   1. the same threshold scan (per-lane TOP = 4 smallest Gram D2 bits, bisection for T with at
//      least kc = K - 1 + 8 list entries <= T, then every column <= T compacted into LDS; more
//      than kWideCap ties: T' = the kc-th smallest of the whole row by bisection on full-row
//      counts, ties at T' in index order);
//   2. trimming by the Gram error bound (knn_select_kernel step 2b): G = the (K-1)-th smallest
//      candidate Gram D2, candidates above G + 2B join the left-out bound tb;
//   3. exact float64 difference-form distances of the kept candidates, 64 per chunk, merged into
//      the sorted list by (d^2, index) -- the reference's stand-in ranks in float64;
//   4. the certificate of knn_select_kernel step 5; if it fails, every column with Gram D2 under
//      the bound is streamed through the same merge (GLL_ST_KNN_RESCAN).
// Exact for any input like the narrow kernel; distances are the float64 sums rounded once.
// --------------------------------------------------------------------------------------
// Two tiers share the kernel: K - 1 <= 128 (kMaxKm1Wide) with 256 candidate slots and per-lane
// lists of 4, and K - 1 <= 256 (kMaxKm1Huge, round 6) with 512 slots and lists of 5 (64 x 5 >=
// kc = K - 1 + 8); the LDS lists of a wave are 5.5 / 10.5 KiB.
template <int CAP, int KMX>
struct WideListsT {
    int cj[CAP];               // candidates: column
    uint32_t cg[CAP];          // candidates: Gram D2 bits
    double cd[kWave];          // a chunk's float64 distances
    int bj[2][KMX];            // sorted K - 1 nearest (double-buffered merge)
    double bd[2][KMX];
};

template <bool VEC, typename WL>
__device__ __forceinline__ int wide_absorb(const float* __restrict__ X, const float* __restrict__ xi,
                                           int i, int d, int Km1, int cj, int cnt, WL& w,
                                           int& cur, int nb) {
    const int lane = lane_id();
    double dv = exact_d2<VEC, 1, double, 4>(X, xi, i, d, lane < cnt ? cj : -1, 0, cnt,
                                            __builtin_inf());
    if (!(dv == dv) || lane >= cnt || cj < 0) dv = __builtin_inf();   // NaN rows rank last
    const int jj = lane < cnt ? cj : INT_MAX;
    w.cd[lane] = dv;
    w.cj[lane] = jj;   // the chunk's candidates were read out of cj[] before this call
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const int nxt = cur ^ 1;
    auto less = [](double da, int ja, double db, int jb) {
        return da < db || (da == db && ja < jb);
    };
    // chunk entry `lane`: its rank among the chunk and among the list
    int rk = 0;
    for (int u = 0; u < cnt; ++u) rk += less(w.cd[u], w.cj[u], dv, jj) ? 1 : 0;
    for (int e = 0; e < nb; ++e) rk += less(w.bd[cur][e], w.bj[cur][e], dv, jj) ? 1 : 0;
    // list entries: rank = own position + chunk entries before it
    for (int e0 = 0; e0 < nb; e0 += kWave) {
        const int e = e0 + lane;
        if (e < nb) {
            const double de = w.bd[cur][e];
            const int je = w.bj[cur][e];
            int r = e;
            for (int u = 0; u < cnt; ++u) r += less(w.cd[u], w.cj[u], de, je) ? 1 : 0;
            if (r < Km1) {
                w.bd[nxt][r] = de;
                w.bj[nxt][r] = je;
            }
        }
    }
    if (lane < cnt && rk < Km1 && dv < __builtin_inf()) {
        w.bd[nxt][rk] = dv;
        w.bj[nxt][rk] = jj;
    }
    int valid = __popcll(__ballot(lane < cnt && dv < __builtin_inf()));
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    cur = nxt;
    return min(nb + valid, Km1);
}

template <bool VEC, int NP, int CAP, int KMX, int TOP>
__global__ __launch_bounds__(256) void knn_select_wide_kernel(
    const float* __restrict__ D2, int ld, size_t plane, const float* __restrict__ X, int n, int d,
    int K, int kc, float eps_fixed, int auto_eps, int RCAP, int32_t* __restrict__ knn_idx,
    float* __restrict__ knn_d2, float* __restrict__ eps, int32_t* __restrict__ rev_cnt,
    int32_t* __restrict__ rev_idx, float* __restrict__ rev_d2, int32_t* __restrict__ ovf,
    int32_t* __restrict__ status, int32_t* __restrict__ status_pub, size_t xs, size_t wss,
    size_t sts, int r0, int r1, const int32_t* __restrict__ perm) {
    const int2 gxy = batch_xy<false>();
    D2 = gshift_at(D2, wss, gxy.y);
    X = gshift_at(X, xs, gxy.y);
    knn_idx = gshift_at(knn_idx, wss, gxy.y);
    knn_d2 = gshift_at(knn_d2, wss, gxy.y);
    eps = gshift_at(eps, wss, gxy.y);
    rev_cnt = gshift_at(rev_cnt, wss, gxy.y);
    rev_idx = gshift_at(rev_idx, wss, gxy.y);
    rev_d2 = gshift_at(rev_d2, wss, gxy.y);
    ovf = gshift_at(ovf, wss, gxy.y);
    status = gshift_at(status, wss, gxy.y);
    status_pub = gshift_at(status_pub, sts, gxy.y);
    constexpr int kWideCap = CAP;
    constexpr int kWideTop = TOP;
    __shared__ WideListsT<CAP, KMX> s_w[4];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    int i;
    if (perm) {
        const int sl = xcd_tile(int(blockIdx.x), int(gridDim.x)) * 4 + wv;
        if (sl >= r1) return;   // whole wave
        i = perm[sl];
    } else {
        i = r0 + gxy.x * 4 + wv;
        if (i >= r1) return;    // whole wave
    }
    WideListsT<CAP, KMX>& w = s_w[wv];
    const int Km1 = K - 1;
    const D2Row<false> row{reinterpret_cast<const char*>(D2) + size_t(i - r0) * ld * 4, 1.f};
    auto bits_of = [&](float x, int j) -> uint32_t {   // invalid: 0xFFFFFFFF (> any T)
        return (j < n && j != i && x == x) ? __float_as_uint(x > 0.f ? x : 0.f) : 0xFFFFFFFFu;
    };
    auto load4 = [&](int jb) {   // columns jb + 4 lane .. + 3 (sum of NP planes), clamped
        const int j0 = jb + 4 * lane;
        const int jc = j0 < ld ? j0 : 0;
        f32x4 v = row.ld4(jc);
#pragma unroll
        for (int p = 1; p < NP; ++p) v += row.ld4(p * plane + jc);
        return v;
    };
    auto ld1 = [&](int j) {
        float x = row.ld1(j);
#pragma unroll
        for (int p = 1; p < NP; ++p) x += row.ld1(p * plane + j);
        return x;
    };
    // ---- 1. threshold scan: per-lane TOP smallest bits
    uint32_t m[kWideTop];
#pragma unroll
    for (int t = 0; t < kWideTop; ++t) m[t] = 0xFFFFFFFFu;
    int nvalid = 0;
    for (int jb = 0; jb < n; jb += 4 * kWave) {
        const f32x4 v = load4(jb);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            uint32_t u = bits_of(v[t], jb + 4 * lane + t);
            nvalid += u != 0xFFFFFFFFu ? 1 : 0;
#pragma unroll
            for (int s = 0; s < kWideTop; ++s) {
                const uint32_t lo = m[s] < u ? m[s] : u;
                u = m[s] < u ? u : m[s];
                m[s] = lo;
            }
        }
    }
    auto count_le = [&](uint32_t t) {
        int c = 0;
#pragma unroll
        for (int s = 0; s < kWideTop; ++s) c += __popcll(__ballot(m[s] <= t));
        return c;
    };
    uint32_t T = 0xFFFFFFFEu;   // fewer than kc valid entries: every valid column
    if (count_le(T) >= kc) {
        uint32_t lo = wave_min_u32(m[0]), up = 0;
        uint32_t top = 0;
#pragma unroll
        for (int s = 0; s < kWideTop; ++s) top = m[s] != 0xFFFFFFFFu ? m[s] : top;
        up = wave_max_u32(top);
        while (lo < up) {
            const uint32_t mid = lo + ((up - lo) >> 1);
            const int c = count_le(mid);
            if (c == kc) {
                up = mid;
                break;
            }
            if (c > kc) up = mid;
            else lo = mid + 1u;
        }
        T = up;
    }
    // compaction of every column <= T
    int base = 0, mine = 0;
    for (int jb = 0; jb < n; jb += 4 * kWave) {
        const f32x4 v = load4(jb);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = jb + 4 * lane + t;
            const uint32_t u = bits_of(v[t], j);
            const bool p = u <= T;
            const uint64_t mk = __ballot(p);
            const int pos = base + lanes_below(mk);
            if (p && pos < kWideCap) {
                w.cj[pos] = j;
                w.cg[pos] = u;
            }
            mine += p ? 1 : 0;
            base += __popcll(mk);
        }
    }
    uint32_t tb;   // Gram D2 bits every left-out column is >= to
    int N;
    if (base > kWideCap) {   // ties: T' = the kc-th smallest of the row, ties in index order
        if (lane == 0) atomicAdd(&status_pub[GLL_ST_KNN_MERGE], 1);
        auto count_full = [&](uint32_t thr) {
            int c = 0;
            for (int jb = 0; jb < n; jb += 4 * kWave) {
                const f32x4 v = load4(jb);
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    c += __popcll(__ballot(bits_of(v[t], jb + 4 * lane + t) <= thr));
            }
            return c;
        };
        uint32_t lo = 0u, up = T;
        while (lo < up) {
            const uint32_t mid = lo + ((up - lo) >> 1);
            if (count_full(mid) >= kc) up = mid;
            else lo = mid + 1u;
        }
        const uint32_t T2 = up;
        base = 0;
        for (int pass = 0; pass < 2; ++pass) {   // below T2 (< kc of them), then ties in order
            for (int j0 = 0; j0 < n && base < kWideCap; j0 += kWave) {
                const int j = j0 + lane;
                const uint32_t u = bits_of(j < n ? ld1(j) : 0.f, j);
                const bool p = pass == 0 ? u < T2 : u == T2;
                const uint64_t mk = __ballot(p);
                const int pos = base + lanes_below(mk);
                if (p && pos < kWideCap) {
                    w.cj[pos] = j;
                    w.cg[pos] = u;
                }
                base += __popcll(mk);
            }
        }
        N = min(base, kWideCap);
        tb = T2;
    } else {
        N = base;
        tb = __ballot(mine != nvalid) == 0 ? 0x7F800000u : T + 1u;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const float* xi = X + size_t(i) * d;
    float a2 = ld1(0);   // |a_i|^2: column 0 is the Gram's centre row (a_0 = 0)
    const double ai = sqrt(double(a2 > 0.f ? a2 : 0.f));
    // ---- 2. trimming: G = the (K-1)-th smallest candidate Gram D2
    if (N > Km1) {
        uint32_t g[kWideCap / kWave];
#pragma unroll
        for (int t = 0; t < kWideCap / kWave; ++t) {
            const int e = t * kWave + lane;
            g[t] = e < N ? w.cg[e] : 0xFFFFFFFFu;
        }
        auto cnt_le = [&](uint32_t thr) {
            int c = 0;
#pragma unroll
            for (int t = 0; t < kWideCap / kWave; ++t) c += __popcll(__ballot(g[t] <= thr));
            return c;
        };
        uint32_t lo = 0u, up = 0xFFFFFFFEu;
        while (lo < up) {
            const uint32_t mid = lo + ((up - lo) >> 1);
            if (cnt_le(mid) >= Km1) up = mid;
            else lo = mid + 1u;
        }
        const double G = double(__uint_as_float(up));
        const double b0 = kGramErr * (2.0 * ai + sqrt(G)) * (2.0 * ai + sqrt(G));
        const double rr = 2.0 * ai + sqrt(G + b0);
        const double thr = G + 2.0 * kGramErr * rr * rr;
        int keep = 0;
        uint32_t dmin = 0xFFFFFFFFu;
#pragma unroll
        for (int t = 0; t < kWideCap / kWave; ++t) {   // in place: chunk t is read before written
            const int e = t * kWave + lane;
            const int j = e < N ? w.cj[e] : -1;
            const bool live = e < N;
            const bool need = live && double(__uint_as_float(g[t])) <= thr;
            if (live && !need) dmin = dmin < g[t] ? dmin : g[t];
            const uint64_t mk = __ballot(need);
            if (need) {
                w.cj[keep + lanes_below(mk)] = j;
                w.cg[keep + lanes_below(mk)] = g[t];
            }
            keep += __popcll(mk);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
        dmin = wave_min_u32(dmin);
        if (dmin < tb) tb = dmin;
        N = keep;
    }
    // ---- 3. float64 distances, merged into the sorted list
    int cur = 0, nb = 0;
    for (int c0 = 0; c0 < N; c0 += kWave) {
        const int cnt = min(kWave, N - c0);
        const int cj = lane < cnt ? w.cj[c0 + lane] : -1;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        nb = wide_absorb<VEC>(X, xi, i, d, Km1, cj, cnt, w, cur, nb);
    }
    // ---- 4. certificate (knn_select_kernel step 5), else a rescan under the bound
    if (Km1 >= 1 && nb == Km1 && tb < 0x7F800000u) {
        const double dK = w.bd[cur][Km1 - 1];
        const double r = 2.0 * ai + sqrt(dK);
        const double thr = dK + kGramErr * r * r;
        if (!(double(__uint_as_float(tb)) > thr)) {
            if (lane == 0) atomicAdd(&status_pub[GLL_ST_KNN_RESCAN], 1);
            nb = 0;
            for (int j0 = 0; j0 < n; j0 += kWave) {
                const int j = j0 + lane;
                const float v = j < n ? ld1(j) : 0.f;
                const bool take = j < n && j != i && v == v && double(v) <= thr;
                const uint64_t mk = __ballot(take);
                if (mk == 0ull) continue;
                if (take) w.cj[lanes_below(mk)] = j;
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                const int cnt = __popcll(mk);
                const int cj = lane < cnt ? w.cj[lane] : -1;
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                nb = wide_absorb<VEC>(X, xi, i, d, Km1, cj, cnt, w, cur, nb);
            }
        }
    }
    // ---- outputs (knn_select_kernel's)
    int32_t* oi = knn_idx + size_t(i) * K;
    float* od = knn_d2 + size_t(i) * K;
    if (lane == 0) {
        oi[0] = i;
        od[0] = 0.f;
    }
    for (int r = lane; r < Km1; r += kWave) {
        const bool live = r < nb;
        oi[1 + r] = live ? w.bj[cur][r] : i;   // fewer valid: self at 0 (dropped edges)
        od[1 + r] = live ? float(w.bd[cur][r]) : 0.f;
    }
    float ei = eps_fixed;
    if (auto_eps) ei = nb == Km1 ? sqrtf(float(w.bd[cur][Km1 - 1])) : 0.f;   // GLL.py:205
    if (lane == 0) {
        eps[i] = ei;
        if (!(ei >= 1e-10f)) atomicOr(&status_pub[GLL_ST_TINY_EPS], 1);   // GLL.py:240-241
    }
    for (int r = lane; r < nb; r += kWave) {   // reverse entries (ci, i); zero distances dropped
        const int ci = w.bj[cur][r];
        const float cef = float(w.bd[cur][r]);
        if (cef > 0.f) {
            const int pos = atomicAdd(&rev_cnt[ci], 1);
            if (pos < RCAP) {
                rev_idx[size_t(ci) * RCAP + pos] = i;
                rev_d2[size_t(ci) * RCAP + pos] = cef;
            } else {
                const int q = atomicAdd(&status[kStOvfCount], 1);
                ovf[3 * q + 0] = ci;
                ovf[3 * q + 1] = i;
                ovf[3 * q + 2] = __float_as_int(cef);
            }
        }
    }
}

// --------------------------------------------------------------------------------------
// gram_pk2_kernel (round 3): the pre-split bf16 GEMM on 256 x 256 upper-triangle tiles with 8
// waves -- two per SIMD -- of 64 x 128 (2 x 4 accumulators of 32 x 32), k-stages of 32 features.
// gram_pk_kernel's 128-tile moves 64 KiB into the CU per 48 MFMAs per wave at one wave per
// SIMD (~96 flops per staged byte; MFMA busy 25-28%, profiles/r02f_mfma_*.json): the CU's
// L2 -> LDS rate, not the matrix pipe, set its pace.  Here a stage is the same 64 KiB (A hi /
// lo and B hi / lo, 256 rows x 64 B each, by LDS-DMA, double-buffered: 128 KiB) for 48 MFMAs
// on EACH of 8 waves -- twice the flops per byte -- and the second wave per SIMD covers the
// other's waits.  Rows are 64 B in LDS, the four 16-B segments XOR-swizzled by (row >> 2) & 3 on
// the source address, which keeps every ds_read_b128 lane group of a fragment read on 16
// distinct bank groups.  Same k order per element as gram_pk_kernel (16-feature chunks in
// ascending order, lo*hi, hi*lo, hi*hi), same epilogue formula, same upper-triangle values
// stored in both orientations: D2 is bitwise gram_pk_kernel's.
// --------------------------------------------------------------------------------------
constexpr int kPK2 = 32;   // features per k-stage of the 256-tile kernel

template <bool H>
__global__ __launch_bounds__(512) void gram_pk2_kernel(const __bf16* __restrict__ Ph,
                                                       const __bf16* __restrict__ Pl,
                                                       const float* __restrict__ nrm, int n,
                                                       int dp, int T, float* __restrict__ D2,
                                                       int ld, size_t wss,
                                                       float* __restrict__ d2s) {
    const int NT = T * (T + 1) / 2;
    const int idx = xcd_tile(blockIdx.x, gridDim.x);
    const int g = idx / NT;
    {
        const size_t off = size_t(g) * wss;   // graph g's workspace block
        Ph = reinterpret_cast<const __bf16*>(reinterpret_cast<const char*>(Ph) + off);
        Pl = reinterpret_cast<const __bf16*>(reinterpret_cast<const char*>(Pl) + off);
        nrm = reinterpret_cast<const float*>(reinterpret_cast<const char*>(nrm) + off);
        D2 = reinterpret_cast<float*>(reinterpret_cast<char*>(D2) + off);
        d2s = reinterpret_cast<float*>(reinterpret_cast<char*>(d2s) + off);
    }
    constexpr int kTP = 256 * kPK2;                                 // bf16 per tile plane
    constexpr int kSS = 260;   // epilogue staging: 128 rows x 256 columns, row stride 260 floats
    constexpr int kSM = 2 * 4 * kTP > 2 * 128 * kSS ? 2 * 4 * kTP : 2 * 128 * kSS;
    __shared__ __attribute__((aligned(16))) __bf16 sm[kSM];   // 130 KiB: [buf][plane] k-stages
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    int bi, bj;
    supertile_tile(idx - g * NT, T, bi, bj);
    const int wr = w >> 1, wc = w & 1;   // rows wr * 64 .., columns wc * 128 ..
    // DMA pieces of a stage: 4 planes x 16 chunks of 16 rows (1 KiB each); wave w issues pieces
    // q = 0..7: plane q >> 1, chunk (q & 1) * 8 + w; lane -> row 16 c + lane / 4, LDS segment
    // lane % 4 <- source segment (lane % 4) ^ ((row >> 2) & 3)
    const __bf16* src[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int pl = q >> 1, c = (q & 1) * 8 + w;
        const int row = 16 * c + (lane >> 2);
        const int seg = (lane & 3) ^ ((row >> 2) & 3);
        int grow = (pl < 2 ? bi : bj) * 256 + row;
        grow = grow < n ? grow : n - 1;
        src[q] = ((pl & 1) ? Pl : Ph) + size_t(grow) * dp + 8 * seg;
    }
    auto issue4 = [&](int ks, int buf, int q0) {
#pragma unroll
        for (int q = q0; q < q0 + 4; ++q) {
            const int pl = q >> 1, c = (q & 1) * 8 + w;
            __bf16* dst = sm + (buf * 4 + pl) * kTP + c * 16 * kPK2;
            __builtin_amdgcn_global_load_lds(src[q] + ks * kPK2, (lds_void*)dst, 16, 0, 0);
        }
    };
    f32x16 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    auto frag = [&](int buf, int pl, int row, int kk) {
        const int pos = (2 * kk + h) ^ ((row >> 2) & 3);
        return *reinterpret_cast<const bf16x8*>(sm + (buf * 4 + pl) * kTP + row * kPK2 + 8 * pos);
    };
    const int nks = dp / kPK2;
    issue4(0, 0, 0);
    issue4(0, 0, 4);
    float dsc = 1.f;   // fp16 D2 scale (H), computed under the first stage's DMAs
    if constexpr (H) {
        __shared__ float red[8];
        dsc = tile_d2_scale<512>(nrm, n, red);
        if (threadIdx.x == 0) *d2s = dsc;
    }
    // (Measured and removed in round 4: requesting both k-steps' fragments of a stage at once,
    // two register sets, 250 VGPRs: B = 64 NS Gram 200 -> 205 us, stress 277 -> 285;
    // profiles/r03y_d2_fp16_ab.txt.)
    {
        for (int ks = 0; ks < nks; ++ks) {
            const int buf = ks & 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's stage-ks DMAs
            __builtin_amdgcn_s_barrier();                          // every wave's
            const bool more = ks + 1 < nks;
#pragma unroll
            for (int kk = 0; kk < kPK2 / 16; ++kk) {
                if (more) issue4(ks + 1, buf ^ 1, 4 * kk);
                bf16x8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    ah[m] = frag(buf, 0, wr * 64 + m * 32 + r, kk);
                    al[m] = frag(buf, 1, wr * 64 + m * 32 + r, kk);
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    bh[m] = frag(buf, 2, wc * 128 + m * 32 + r, kk);
                    bl[m] = frag(buf, 3, wc * 128 + m * 32 + r, kk);
                }
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
                    }
            }
        }
    }
    // epilogue: D2 = |a_i|^2 + |a_j|^2 - 2 <a_i, a_j>; C layout of 32x32: col = lane & 31,
    // row = (e & 3) + 8 (e >> 2) + 4 h.  Diagonal tiles keep the upper triangle (tj >= ti, the
    // value gram_pk_kernel stores there) and write it in both orientations.
    const bool diag = bi == bj;
    if (!diag) {
        // Off-diagonal tiles (round 3): the mirrored orientation leaves the registers as one
        // 16-B store per lane (a lane holds 4 consecutive rows of its column), while the direct
        // one -- 128 four-byte stores per wave, 256 B each -- goes through LDS: each half of the
        // tile (128 rows) is staged row-major and leaves as 1-KiB row stores (16 per wave).
        // Same values, same positions: D2 is bitwise the per-element epilogue's.
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int i0 = bi * 256 + wr * 64 + a * 32;
            float ni[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int i = i0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                ni[e] = nrm[i < n ? i : n - 1];
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = bj * 256 + wc * 128 + b * 32 + r;
                const float nj = nrm[j < n ? j : n - 1];
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[a][b][e] = ni[e] + nj - 2.f * acc[a][b][e];
                if (j < n) {   // mirrored: row j, columns i0 + 8 g + 4 h .. +3
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int i = i0 + 8 * gq + 4 * h;
                        const size_t o = size_t(j) * ld + i;
                        if (i + 4 <= n) {
                            dput4<H>(D2, o, f32x4{acc[a][b][4 * gq], acc[a][b][4 * gq + 1],
                                                  acc[a][b][4 * gq + 2], acc[a][b][4 * gq + 3]}, dsc);
                        } else {
#pragma unroll
                            for (int t = 0; t < 4; ++t)
                                if (i + t < n) dput<H>(D2, o + t, acc[a][b][4 * gq + t], dsc);
                        }
                    }
                }
            }
        }
        float* stg = reinterpret_cast<float*>(sm);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            __syncthreads();   // the k-stage buffers (then the previous half) are no longer read
            if ((wr >> 1) == hh) {
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
#pragma unroll
                        for (int e = 0; e < 16; ++e) {
                            const int row = (wr & 1) * 64 + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                            stg[row * kSS + wc * 128 + b * 32 + r] = acc[a][b][e];
                        }
            }
            __syncthreads();
            const int j = bj * 256 + 4 * lane;
#pragma unroll 4
            for (int q = 0; q < 16; ++q) {
                const int row = w * 16 + q;
                const int i = bi * 256 + hh * 128 + row;
                const f32x4 v = *reinterpret_cast<const f32x4*>(stg + row * kSS + 4 * lane);
                if (i < n) {
                    const size_t o = size_t(i) * ld + j;
                    if (j + 4 <= n) {
                        dput4<H>(D2, o, v, dsc);
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (j + t < n) dput<H>(D2, o + t, v[t], dsc);
                    }
                }
            }
        }
        return;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const int ti0 = wr * 64 + a * 32;
        const int i0 = bi * 256 + ti0;
        float ni[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int i = i0 + (e & 3) + 8 * (e >> 2) + 4 * h;
            ni[e] = nrm[i < n ? i : n - 1];
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int tj = wc * 128 + b * 32 + r;
            const int j = bj * 256 + tj;
            if (diag && wc * 128 + b * 32 + 31 < ti0) continue;   // sub-tile wholly below
            const float nj = nrm[j < n ? j : n - 1];
            float dv[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) dv[e] = ni[e] + nj - 2.f * acc[a][b][e];
#pragma unroll
            for (int e = 0; e < 16; ++e) {   // direct: 32 lanes per 128-B row piece
                const int ti = ti0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                const int i = bi * 256 + ti;
                if (i < n && j < n && (!diag || tj >= ti)) dput<H>(D2, size_t(i) * ld + j, dv[e], dsc);
            }
            if (j < n) {   // mirrored: row j, columns i0 + 8 g + 4 h .. +3
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int ti = ti0 + 8 * gq + 4 * h;
                    const int i = bi * 256 + ti;
                    const size_t o = size_t(j) * ld + i;
                    if (i + 4 <= n && (!diag || tj >= ti + 3)) {
                        dput4<H>(D2, o, f32x4{dv[4 * gq], dv[4 * gq + 1], dv[4 * gq + 2], dv[4 * gq + 3]}, dsc);
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (i + t < n && (!diag || tj >= ti + t)) dput<H>(D2, o + t, dv[4 * gq + t], dsc);
                    }
                }
            }
        }
    }
}

// 256-tiles (gram_pk2_kernel) or 128-tiles (gram_pk_kernel) for the pre-split GEMM: the one
// with fewer waves of one-workgroup-per-CU rounds x k-stage bytes (a round of 256-tiles moves
// the same 64 KiB per stage as one of 128-tiles but does 4x the work, in twice the stages).
// The knob GLL_KNOB_GRAM_TILE = 128 / 256 forces one (tests).
static bool gram_tile256(const Layout& L, const Batch& bt, int T, int T2) {
    if (knob(GLL_KNOB_GRAM_TILE) > 0) return knob(GLL_KNOB_GRAM_TILE) == 256 && L.dp % kPK2 == 0;
    // (d <= 128: a tile is 4 k-stages; the FullySup shape measured 225 -> 230 us at B = 64)
    if (L.dp % kPK2 || L.dp <= 128) return false;
    const int cus = device_cus();
    const int64_t t1 = int64_t(bt.B) * T * (T + 1) / 2, t2 = int64_t(bt.B) * T2 * (T2 + 1) / 2;
    const int64_t r1 = (t1 + cus - 1) / cus, r2 = (t2 + cus - 1) / cus;
    return r2 * 2 * (L.dp / kPK2) * kPK2 < r1 * (L.dp / kPK) * kPK;   // stage bytes equal
}

// The pre-split route (gram_split + gram_pk / gram_pk2): batches, and single graphs with d > 128
// and n <= 12,288 (see launch_gram).  Its D2 is stored fp16 (dput) unless GLL_D2_F32 = 1 (A/B).
static bool presplit_route(const Layout& L, const Batch& bt) {
    const int T = (L.n + 127) / 128;
    return int64_t(bt.B) * T * (T + 1) / 2 >= 256 &&
           !(L.flags & GLL_FLAG_GRAM_INLINE) && (bt.B > 1 || (L.d > 128 && L.n <= 12288)) &&
           gram_planes(L, bt.B) == 1 && L.PR == L.n;
}
// Batches only (single graphs measured slower with it: at stress the wider candidate margin
// cost the select 274 -> 299 us; DESIGN.md §3.1, profiles/r03x_d2_fp16_ab.txt).
// (Not for the wide select, K - 1 > kMaxKm1: it reads fp32 rows.)
static bool d2_half(const Layout& L, const Batch& bt) {
    return !(L.flags & GLL_FLAG_D2_F32) && bt.B > 1 && presplit_route(L, bt) &&
           L.K - 1 <= kMaxKm1;
}

// --------------------------------------------------------------------------------------
// Locality order of the rows of one large graph (gll_internal.h locality_order).  Pivot j is
// row (j * 2654435761 + 12345) mod n -- a hash, so periodic row layouts (labels i % 10 in the
// callers' minibatches) do not alias -- and row i joins the pivot nearest to it under the Gram
// D2, read as the pivots' D2 rows (D2 is symmetric; coalesced across i).  Ties go to the lower
// pivot; a NaN distance never wins.  Speed only: no row's result depends on the order.
// --------------------------------------------------------------------------------------
__device__ __forceinline__ int pivot_row(int j, int n) {
    return int((uint32_t(j) * 2654435761u + 12345u) % uint32_t(n));
}

// 64 rows per workgroup, the pivots split over its 4 waves (16 each: every load of a lane
// issued together), the 4 partial minima combined in LDS in pivot order.  Wave 0 then ranks its
// rows within their pivot (lane order: pid = pivot | rank << 8) and writes the block's rows per
// pivot as one plain 64-int histogram row.  (The first version counted with one global atomic
// per row on 64 counters: 8,192 same-address atomics made this a 13.9 us kernel at stress,
// profiles/r04b_stress_kernel_stats.csv; order_perm then scattered through LDS cursor atomics.)
template <int NP>
__global__ __launch_bounds__(256) void order_pid_kernel(const float* __restrict__ D2, int ld,
                                                        size_t plane, int n,
                                                        int32_t* __restrict__ pid,
                                                        int32_t* __restrict__ hist) {
    constexpr int PPW = kPiv / 4;   // pivots per wave
    static_assert(kPiv == kWave, "one histogram bin per lane");
    __shared__ float s_best[4][kWave];
    __shared__ int s_arg[4][kWave];
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    const int i = int(blockIdx.x) * kWave + lane;
    const int ic = i < n ? i : n - 1;
    float v[PPW];
#pragma unroll
    for (int j = 0; j < PPW; ++j) {   // every load issued before any is compared
        const size_t o = size_t(pivot_row(wv * PPW + j, n)) * ld + ic;
        v[j] = D2[o];
#pragma unroll
        for (int p = 1; p < NP; ++p) v[j] += D2[p * plane + o];
    }
    float best = __builtin_inff();
    int bp = wv * PPW;
#pragma unroll
    for (int j = 0; j < PPW; ++j)
        if (v[j] < best) {   // ties: the lower pivot; a NaN never wins
            best = v[j];
            bp = wv * PPW + j;
        }
    s_best[wv][lane] = best;
    s_arg[wv][lane] = bp;
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int w = 1; w < 4; ++w)
        if (s_best[w][lane] < best) {
            best = s_best[w][lane];
            bp = s_arg[w][lane];
        }
    const bool valid = i < n;
    int rank = 0, cnt = 0;   // cnt: rows of this block at pivot `lane`
    uint64_t todo = __ballot(valid);
    while (todo) {   // one round per distinct pivot of the block (wave-uniform)
        const int v0 = __builtin_amdgcn_readlane(bp, int(__builtin_ctzll(todo)));
        const uint64_t mk = __ballot(valid && bp == v0);
        if (valid && bp == v0) rank = lanes_below(mk);
        if (lane == v0) cnt = __popcll(mk);
        todo &= ~mk;
    }
    if (valid) pid[i] = bp | (rank << 8);
    hist[size_t(blockIdx.x) * kPiv + lane] = cnt;
}

// One workgroup, no atomics: per pivot, the blocks' counts become exclusive offsets (16 block
// groups per pivot, group totals scanned in LDS, pivots scanned by one wave), written back over
// the histogram; then row i goes to offset[block i / 64][pivot] + its rank in the block.
__global__ __launch_bounds__(1024) void order_perm_kernel(int n, const int32_t* __restrict__ pid,
                                                          int32_t* __restrict__ hist,
                                                          int32_t* __restrict__ perm,
                                                          int32_t* __restrict__ status) {
    static_assert(kPiv == kWave, "one wave scans the pivot counts");
    constexpr int NGRP = 1024 / kPiv;   // block groups per pivot
    __shared__ int part[NGRP][kPiv];
    __shared__ int goff[NGRP][kPiv];
    const int tid = threadIdx.x;
    const int nb = (n + kWave - 1) / kWave;
    const int per = (nb + NGRP - 1) / NGRP;
    const int pv = tid & (kPiv - 1), grp = tid / kPiv;
    const int b0 = grp * per, b1 = min(nb, b0 + per);
    int run = 0;
#pragma unroll 8
    for (int b = b0; b < b1; ++b) run += hist[size_t(b) * kPiv + pv];
    part[grp][pv] = run;
    __syncthreads();
    if (tid < kWave) {
        int c = 0;
#pragma unroll
        for (int g = 0; g < NGRP; ++g) c += part[g][tid];
        int incl = c;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int t = __shfl_up(incl, off);
            if (tid >= off) incl += t;
        }
        int o = incl - c;
#pragma unroll
        for (int g = 0; g < NGRP; ++g) {
            goff[g][tid] = o;
            o += part[g][tid];
        }
    }
    __syncthreads();
    int o = goff[grp][pv];
#pragma unroll 8
    for (int b = b0; b < b1; ++b) {
        const size_t q = size_t(b) * kPiv + pv;
        const int h = hist[q];
        hist[q] = o;
        o += h;
    }
    __syncthreads();   // the offsets are visible to the whole workgroup
    constexpr int U = 8;   // rows per thread per batch: every load of a batch in flight together
    for (int i0 = 0; i0 < n; i0 += 1024 * U) {
        int v[U], h[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * 1024 + tid;
            v[u] = i < n ? pid[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * 1024 + tid;
            h[u] = i < n ? hist[size_t(i >> 6) * kPiv + (v[u] & 0xFF)] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * 1024 + tid;
            if (i < n) perm[h[u] + (v[u] >> 8)] = i;
        }
    }
    if (tid == 0) status[kStPermValid] = 1;   // read by the backward (grad.hip launch_backward_grad)
}

hipError_t launch_order(const Layout& L, void* ws, hipStream_t s) {
    const float* D2 = L.at<float>(ws, L.D2);
    int32_t* hist = L.at<int32_t>(ws, L.ohist);
    int32_t* pid = L.at<int32_t>(ws, L.pid);
    const size_t plane = size_t(L.n) * L.ldD;
    const dim3 grid(unsigned((L.n + kWave - 1) / kWave));
    if (gram_planes(L, 1) == 2)
        launch_k(order_pid_kernel<2>, grid, 256, 0, s, D2, L.ldD, plane, L.n, pid, hist);
    else
        launch_k(order_pid_kernel<1>, grid, 256, 0, s, D2, L.ldD, plane, L.n, pid, hist);
    launch_k(order_perm_kernel, dim3(1), 1024, 0, s, L.n, static_cast<const int32_t*>(pid), hist,
             L.at<int32_t>(ws, L.perm), L.at<int32_t>(ws, L.status));
    return launch_status("knn.hip:launch_order");
}

hipError_t launch_gram(const Layout& L, const Batch& bt, void* ws, const float* X, bool vec,
                       hipStream_t s) {
    float* D2 = L.at<float>(ws, L.D2);
    int32_t* st = L.at<int32_t>(ws, L.status);
    int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
    if (gram_planes(L, bt.B) == 2) {
        const int T = (L.n + 63) / 64;
        const dim3 grid(T * T, bt.B);
        const size_t plane = size_t(L.n) * L.ldD;
        prof_begin(GLL_K_GRAM, s);
        if (vec)
            launch_k(gram_bf3s_kernel<true>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, plane, st, rc, bt.x, bt.ws);
        else
            launch_k(gram_bf3s_kernel<false>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, plane, st, rc, bt.x, bt.ws);
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(bf3s)");
    }
    // 128-tiles when there are enough of them to fill the chip twice (large graphs and batches;
    // a single NS graph has only 36); 64-tiles otherwise
    const int T = (L.n + 127) / 128;
    // pre-split GEMM from 256 tiles (NS B = 8, 288 tiles: 58 -> 45 us; a single FullySup graph,
    // 78 tiles, stays on the 64-tile kernel: 17.5 against 21.6 us).  Not for single graphs with
    // d <= 128 (utils.laplace's 250 + 60,000 points: one K stage, nothing for the DMA pipeline to
    // hide, and the whole graph build took 166 ms with it against 19 ms with the inline 128-tile
    // kernel; 20,250 points 3.9 -> 2.1 ms; profiles/r02i_gram_inline_ab.txt).  Batches
    // and d = 1024 keep it (NS B = 64 322 -> 237 us, FullySup B = 64 272 -> 228, stress 485 -> 319).
    // Nor for single graphs past ~12k rows at any d: forward 5.2 vs 3.8 ms at 20,250 x 256, 16.3 vs
    // 8.7 ms at 30,250 x 512, 17.5 vs 11.4 ms at 30,250 x 1024 (tools/gram_route_probe.py,
    // profiles/r02j_gram_route.txt); the stress shape (8,192 x 1024) is the largest measured where
    // it wins, and the 12,288 cut between the two is not measured.
    if (presplit_route(L, bt)) {
        // split once (one pass over X), then the LDS-DMA bf16 GEMM over 128-tiles
        __bf16* Ph = L.at<__bf16>(ws, L.xhi);
        __bf16* Pl = L.at<__bf16>(ws, L.xlo);
        float* nrm = L.at<float>(ws, L.xnrm);
        const bool H = d2_half(L, bt);
        const int T2 = (L.n + 255) / 256;
        const bool t256 = gram_tile256(L, bt, T, T2);
        // one 256-tile per CU at a time: a last round short of a full one (stress: 528 tiles, 16
        // in the third round, profiles/r04b_stress_kernel_stats.csv) runs as subtiles of those
        // tiles instead (gram_pk_kernel's D2 is bitwise the 256-tile kernel's), where they fit
        // one round.  Round 6: 64-row subtiles (16 per tile, two workgroups per CU at 64 KiB of
        // LDS) where they fit: stress 256 of them, one per CU, 18.8 us where 64 128-subtiles on a
        // quarter of the chip took 31.4 (profiles/r06i_ab_gram_tail.txt); otherwise 128-subtiles
        // (4 per tile).  More than one round of subtiles loses to a last round of 256-tiles: B =
        // 64 NS, 128 tail tiles, 2,048 64-subtiles 58 us against ~35 for the round, and two rounds
        // of 128-subtiles 224 -> 235 us (round 5).  GLL_KNOB_GRAM_TAIL: 1 no tail, 2 128-subtiles.
        const int64_t nt2 = int64_t(bt.B) * T2 * (T2 + 1) / 2;
        const int cus = device_cus();
        const int tk = knob(GLL_KNOB_GRAM_TAIL);
        int64_t tail = t256 && nt2 > cus ? nt2 % cus : 0;
        const int sub = (tk != 2 && tail * 16 <= 2 * int64_t(cus)) ? 16 : 4;   // subtiles per tile
        if ((sub == 4 && tail * 4 > cus) || tk == 1) tail = 0;
        // (Measured and dropped: the subtiles split further over 4 k-slices summed by a reduce
        // kernel, 256 workgroups instead of 64: 250 -> 260 us, profiles/r04u_ab_tail.txt.)
        prof_begin(GLL_K_GRAM, s);
        prof_span(tail > 0 ? 3 : 2);
        const dim3 sgrid((L.n + 3) / 4, bt.B);
        float* d2s = L.at<float>(ws, L.d2s);
        if (vec)
            launch_k(gram_split_kernel<true>, sgrid, 256, 0, s, X, L.n, L.d, L.dp, Ph, Pl, nrm, st, rc, bt.x, bt.ws);
        else
            launch_k(gram_split_kernel<false>, sgrid, 256, 0, s, X, L.n, L.d, L.dp, Ph, Pl, nrm, st, rc, bt.x, bt.ws);
        if (t256) {
            launch_k(H ? gram_pk2_kernel<true> : gram_pk2_kernel<false>,
                     dim3(unsigned(nt2 - tail)), 512, 0, s, Ph, Pl, nrm, L.n, L.dp, T2, D2,
                     L.ldD, bt.ws, d2s);
            if (tail > 0 && sub == 4)
                launch_k(H ? gram_pk_kernel<true, 128> : gram_pk_kernel<false, 128>,
                         dim3(unsigned(4 * tail)), 256, 0, s, Ph, Pl, nrm, L.n, L.dp, T, D2, L.ldD,
                         bt.ws, d2s, int(nt2 - tail));
            else if (tail > 0)
                launch_k(H ? gram_pk_kernel<true, 64> : gram_pk_kernel<false, 64>,
                         dim3(unsigned(16 * tail)), 256, 0, s, Ph, Pl, nrm, L.n, L.dp,
                         (L.n + 63) / 64, D2, L.ldD, bt.ws, d2s, int(nt2 - tail));
        } else {
            launch_k(H ? gram_pk_kernel<true, 128> : gram_pk_kernel<false, 128>,
                     dim3(unsigned(bt.B * T * (T + 1) / 2)), 256, 0, s, Ph, Pl, nrm, L.n, L.dp, T,
                     D2, L.ldD, bt.ws, d2s, -1);
        }
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(pk)");
    }
    if (int64_t(bt.B) * T * (T + 1) / 2 >= 512) {
        const dim3 grid(T * (T + 1) / 2, bt.B);
        prof_begin(GLL_K_GRAM, s);
        if (vec)
            launch_k(gram_bf3w_kernel<true>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws, 0, 0);
        else
            launch_k(gram_bf3w_kernel<false>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc, bt.x, bt.ws, 0, 0);
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(bf3w)");
    }
    const int T64 = (L.n + 63) / 64;
    const dim3 grid(T64 * (T64 + 1) / 2, bt.B);
    prof_begin(GLL_K_GRAM, s);
    if (L.d <= kHP) {   // 1024-thread tile 17.4 -> 9.5 us at FullySup (profiles/r06v_ab_*.txt)
        if (vec)
            launch_k(gram_bf3h_kernel<true>, grid, 512, 0, s, X, L.n, L.d, T64, D2, L.ldD, st, rc, bt.x, bt.ws);
        else
            launch_k(gram_bf3h_kernel<false>, grid, 512, 0, s, X, L.n, L.d, T64, D2, L.ldD, st, rc, bt.x, bt.ws);
        prof_end(GLL_K_GRAM, s);
        return launch_status("knn.hip:launch_gram(bf3h)");
    }
    if (vec)
        launch_k(gram_bf3_kernel<true>, grid, 1024, 0, s, X, L.n, L.d, T64, D2, L.ldD, st, rc, bt.x, bt.ws);
    else
        launch_k(gram_bf3_kernel<false>, grid, 1024, 0, s, X, L.n, L.d, T64, D2, L.ldD, st, rc, bt.x, bt.ws);
    prof_end(GLL_K_GRAM, s);
    return launch_status("knn.hip:launch_gram(bf3)");
}

// One row panel of the Gram (build_graph's panel mode, single graphs): rows r0 .. r0 + rows - 1
// against every column on the inline-split 128-tile kernel (rectangular tiles: twice the flops
// of the triangle, for an O(panel x n) buffer).
hipError_t launch_gram_panel(const Layout& L, void* ws, const float* X, bool vec, int r0, int rows,
                             hipStream_t s) {
    float* D2 = L.at<float>(ws, L.D2);
    int32_t* st = L.at<int32_t>(ws, L.status);
    int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
    const int T = (L.n + 127) / 128, pt = (rows + 127) / 128;
    if (r0 % 128 || pt <= 0) return hipErrorInvalidValue;
    const dim3 grid(unsigned(int64_t(pt) * T));
    prof_begin(GLL_K_GRAM, s);
    if (vec)
        launch_k(gram_bf3w_kernel<true>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc,
                 size_t(0), size_t(0), r0, pt);
    else
        launch_k(gram_bf3w_kernel<false>, grid, 1024, 0, s, X, L.n, L.d, T, D2, L.ldD, st, rc,
                 size_t(0), size_t(0), r0, pt);
    prof_end(GLL_K_GRAM, s);
    return launch_status("knn.hip:launch_gram_panel");
}

hipError_t launch_select(const Layout& L, const Batch& bt, void* ws, const float* X,
                         float eps_fixed, bool auto_eps, bool vec, int32_t* status_pub,
                         hipStream_t s, int r0, int rows) {
    if (rows < 0) rows = L.n - r0;
    const int n = L.n, K = L.K;
    // candidate list capacity: smallest of {16, 32, 64} leaving a re-rank margin >= 4
    const int need = K - 1 + 4;
    const int KC = need <= 16 ? 16 : (need <= 32 ? 32 : 64);
    if (K - 1 > kMaxKm1Huge) return hipErrorInvalidValue;
    int margin = KC - (K - 1);
    if (margin > 8) margin = 8;
    int kc = K - 1 + margin;
    if (kc > n - 1) kc = n - 1;
    const size_t plane = size_t(n) * L.ldD;
    const int planes = gram_planes(L, bt.B);
    dim3 grid((rows + 3) / 4, bt.B);
    const bool h16 = planes == 1 && d2_half(L, bt);   // the Gram stored D2 as fp16 x s
    const float* d2s = L.at<float>(ws, L.d2s);
    const int32_t* perm = (locality_order(L, bt) && r0 == 0 && rows == n)
                              ? L.at<int32_t>(ws, L.perm) : nullptr;
    if (K - 1 > kMaxKm1) {   // k past one candidate per lane: LDS lists (knn_select_wide_kernel)
        if (h16) return hipErrorInvalidValue;   // d2_half keeps fp32 rows for it
        const int kcw = min(K - 1 + 8, n - 1);
        prof_begin(GLL_K_SELECT, s);
#define GLL_SELW(V, NPV)                                                                       \
        do {                                                                                   \
            if (K - 1 > kMaxKm1Wide)                                                           \
                GLL_SELW_(V, NPV, 512, kMaxKm1Huge, 5);                                        \
            else                                                                               \
                GLL_SELW_(V, NPV, 256, kMaxKm1Wide, 4);                                        \
        } while (0)
#define GLL_SELW_(V, NPV, CAP, KMX, TOP)                                                       \
        launch_k(knn_select_wide_kernel<V, NPV, CAP, KMX, TOP>, grid, 256, 0, s,                 \
                 L.at<float>(ws, L.D2), L.ldD,                                                 \
                 plane, X, n, L.d, K, kcw, eps_fixed, auto_eps ? 1 : 0, L.RCAP,                \
                 L.at<int32_t>(ws, L.knn_idx), L.at<float>(ws, L.knn_d2), L.at<float>(ws, L.eps), \
                 L.at<int32_t>(ws, L.rev_cnt), L.at<int32_t>(ws, L.rev_idx),                   \
                 L.at<float>(ws, L.rev_d2), L.at<int32_t>(ws, L.ovf), L.at<int32_t>(ws, L.status), \
                 status_pub, bt.x, bt.ws, bt.st, r0, r0 + rows, perm)
        if (vec) {
            if (planes == 2) GLL_SELW(true, 2);
            else GLL_SELW(true, 1);
        } else {
            if (planes == 2) GLL_SELW(false, 2);
            else GLL_SELW(false, 1);
        }
#undef GLL_SELW
#undef GLL_SELW_
        prof_end(GLL_K_SELECT, s);
        return launch_status("knn.hip:launch_select(wide)");
    }
    // the latency form (PG = 2 candidate groups in flight, NU = 16, ~200 VGPRs: 2 waves per SIMD)
    // for a single graph whose rows fill at most one such round of the chip; larger graphs (and
    // batches) run the occupancy form below.  Stress (n = 8,192): 2,048 workgroups, four rounds
    // of the latency form (profiles/r04c_trace_stress.txt: the last workgroup starts at +200 of
    // 255 us).  GLL_KNOB_SEL_FORM 1 / 2 forces either (tests, A/B).
    const int form = knob(GLL_KNOB_SEL_FORM);
    const bool lat = bt.B == 1 && (form == 1 || (form == 0 && rows <= 2048));
    prof_begin(GLL_K_SELECT, s);
// Batched launches (PG = 1) stage x_i in LDS (XQ quarters of 256 features, d <= 1024): round 2
// measured B = 64 NS select 259 -> 214 us at 6 waves per SIMD (XQ = 2, NU = 8; the NU = 16
// batch of loads held 120 VGPRs, 4 waves).  Round 4 (x_i by LDS-DMA, no registers held for it):
// NU = 4 at 8 waves per SIMD, B = 64 NS 183 -> 174 us, FullySup B = 64 349 -> 339, stress
// 169 -> 168 (profiles/r04q_ab_sel.txt).  NU: 32-feature steps per exact-distance load batch
// (16 for the latency form, whose two waves per SIMD have registers to spare); the loads of
// steps past d are clamped to row 0 and masked.
// Batched launches number blocks XCD-contiguously (R = true: each XCD works through a run of
// graphs): NS B = 64 220 -> 213 us, FullySup B = 64 440 -> 429 us (profiles/r02h_xcd_ab.txt),
// once the kernel took its graph index once instead of per pointer.
#define GLL_SEL6(KCV, V, NPV, NUS, NUB, XQV, CHV, HV)                                          \
    launch_k((lat ? knn_select_kernel<KCV, V, NPV, 2, NUS, 0, false, CHV, HV>            \
                        : knn_select_kernel<KCV, V, NPV, 1, NUB, (V ? XQV : 0), true, CHV, HV>), grid, 256, 0, s, \
        L.at<float>(ws, L.D2), L.ldD, plane, X, n, L.d, K, kc, eps_fixed, auto_eps ? 1 : 0,     \
        L.RCAP,                                                                                \
        L.at<int32_t>(ws, L.knn_idx), L.at<float>(ws, L.knn_d2), L.at<float>(ws, L.eps),       \
        L.at<int32_t>(ws, L.rev_cnt), L.at<int32_t>(ws, L.rev_idx), L.at<float>(ws, L.rev_d2), \
        L.at<int32_t>(ws, L.ovf), L.at<int32_t>(ws, L.status), status_pub, bt.x, bt.ws, bt.st,       \
        r0, r0 + rows, d2s, perm)
#define GLL_SEL5(KCV, V, NPV, NUS, NUB, XQV, CHV)                                              \
    do {                                                                                       \
        if (h16) GLL_SEL6(KCV, V, NPV, NUS, NUB, XQV, CHV, (NPV == 1));                        \
        else GLL_SEL6(KCV, V, NPV, NUS, NUB, XQV, CHV, false);                                 \
    } while (0)
// the threshold scan holds rows of <= 2048 columns in registers (KC <= 32, aligned d)
#define GLL_SEL4(KCV, V, NPV, NUS, NUB, XQV)                                                   \
    do {                                                                                       \
        if (KCV <= 32 && V && n <= 1024 && rows == n) GLL_SEL5(KCV, V, NPV, NUS, NUB, XQV, (KCV <= 32 && V ? 1 : 0)); \
        else if (KCV <= 32 && V && n <= 2048 && rows == n) GLL_SEL5(KCV, V, NPV, NUS, NUB, XQV, (KCV <= 32 && V ? 2 : 0)); \
        else GLL_SEL5(KCV, V, NPV, NUS, NUB, XQV, 0);                                          \
    } while (0)
#define GLL_SEL(KCV, V)                                                                        \
    do {                                                                                       \
        if (planes == 2) GLL_SEL4(KCV, V, 2, 16, 16, 0);                                       \
        else if (L.d <= 128) GLL_SEL4(KCV, V, 1, 4, 4, 1);                                     \
        else if (L.d <= 256) GLL_SEL4(KCV, V, 1, 16, 4, 1);                                    \
        else if (L.d <= 512) GLL_SEL4(KCV, V, 1, 16, 4, 2);                                    \
        else if (L.d <= 1024) GLL_SEL4(KCV, V, 1, 16, 4, 4);                                   \
        else GLL_SEL4(KCV, V, 1, 16, 16, 0);                                                   \
    } while (0)
    if (KC == 16) { if (vec) GLL_SEL(16, true); else GLL_SEL(16, false); }
    else if (KC == 32) { if (vec) GLL_SEL(32, true); else GLL_SEL(32, false); }
    else { if (vec) GLL_SEL(64, true); else GLL_SEL(64, false); }
#undef GLL_SEL
#undef GLL_SEL4
#undef GLL_SEL5
#undef GLL_SEL6
    prof_end(GLL_K_SELECT, s);
    return launch_status("knn.hip:launch_select");
}

}  // namespace gll
