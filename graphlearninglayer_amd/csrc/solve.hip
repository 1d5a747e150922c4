// solve.hip -- Jacobi-preconditioned conjugate gradients on Luu (and on a general CSR).
//
// Replaces the SuperLU `spsolve(Luu, -Lul Y)` of the forward (/root/reference/GLL.py:53)
// and `spsolve(Luu, grad_output)` of the backward (GLL.py:93); the algorithm is the
// per-column masked CG of stable_conjgrad (GLL.py:247-276) with a Jacobi preconditioner
// (the reference's commented-out variant, GLL.py:55-64), WITHOUT its `p = r` aliasing
// quirk.  Each right-hand-side column is an independent system, so
// one workgroup owns one column: no inter-workgroup traffic, no host synchronisation, the
// iteration loop and the convergence test live on the device.
//
// Luu is never materialised: row u (graph row i = base + u) is
//     diag[u] * p_u - sum_{e in row i, col_e >= base} w_e * p_{col_e - base}
// over the sorted CSR of the symmetric kNN graph (labeled columns first, so the U block of
// a row is a suffix of the row).
//
// Per-column kernels (cg_dispatch picks one; single graphs with m > 2048 take the whole-GPU
// CG of gridcg.hip):
//   cg_ell_kernel (short U rows, m <= 4096): a thread owns R rows and keeps everything about
//     them in registers, including the first S entries of each U row as an ELL slice; entries
//     past S are compacted into LDS.  Single-reduction (Chronopoulos-Gear) PCG: one fused
//     three-value exchange and one publish barrier per iteration.
//   cg_vr_kernel (long U rows: K = 25, the FullySup shape): the U block cut into "virtual
//     rows" of 8 entries dealt out evenly to the threads (see its comment).
//   cg_lds_kernel: vectors in LDS or global memory, for systems larger than either.
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_set>

#include "gll_internal.h"
#include "grad_common.h"

namespace gll {

GLL_TRACE_UNIT(solve)
#ifdef GLL_TRACE
// fused backward, per gradient wave (row): [0] release seen, [1] w loaded + first coefficients,
// [2] products done, [3] stored, [4] (row length) | (CU id << 16) | (XCC id << 24)
static __device__ unsigned long long g_fz[5 * 4096];
void trace_read_fz(unsigned long long* out) {
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fz), sizeof(g_fz));
}
#define GLL_FZ(slot, wv, val)                                                                  \
    do {                                                                                       \
        if (lane_id() == 0 && (wv) < 4096) g_fz[(slot) * 4096 + (wv)] = (val);                 \
    } while (0)
#else
#define GLL_FZ(slot, wv, val) do {} while (0)
#endif

static constexpr size_t kLdsLimit = 160 * 1024;
static constexpr size_t kLdsDyn = kLdsLimit - 1024;   // dynamic share, room for static LDS
constexpr int kSc1W = 16;   // buffer aux bit sc1 (write-through / L2-coherent)

// Opt a kernel into all of the 160 KiB of LDS its static allocation leaves for dynamic use,
// once per kernel (host-side cost).  The attribute call's status is consumed here: a failure
// must not linger as the thread's last error and surface at an unrelated launch.
void allow_full_lds(const void* fn) {
    static std::mutex mu;
    static std::unordered_set<const void*> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert(fn).second) {
        hipFuncAttributes at{};
        size_t stat = 0;
        if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int(kLdsLimit - stat));
        (void)hipGetLastError();
    }
}

// Block-wide sum of two values; every thread gets the totals (fixed order -> deterministic).
template <int NT>
__device__ __forceinline__ void block_sum2(float& a, float& b, float* red, int& phase) {
    wave_sum2_dpp(a, b);
    if constexpr (NT > kWave) {
        constexpr int NW = NT / kWave;
        float* q = red + phase * 2 * NW;
        phase ^= 1;
        if (lane_id() == 0) {
            q[threadIdx.x >> 6] = a;
            q[NW + (threadIdx.x >> 6)] = b;
        }
        __syncthreads();
        a = 0.f;
        b = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            a += q[w];
            b += q[NW + w];
        }
    }
}


// Block-wide sum of three values in one LDS exchange (the single-reduction CG).  Partials
// are laid out [value][wave] so each total is read with 16-B loads; fixed order everywhere.
// Block-wide sum of three values in two halves: post (DPP, partials to LDS, barrier) and read
// (totals from LDS), so the pipelined CG can put independent work between them.  Partials
// are laid out [value][wave] so each total is read with 16-B loads; fixed order everywhere.
template <int NT>
__device__ __forceinline__ const float* block_sum3_post(float& a, float& b, float& c, float* red,
                                                        int& phase) {
    a = dpp_add<0xB1, 0xf>(a); b = dpp_add<0xB1, 0xf>(b); c = dpp_add<0xB1, 0xf>(c);
    a = dpp_add<0x4E, 0xf>(a); b = dpp_add<0x4E, 0xf>(b); c = dpp_add<0x4E, 0xf>(c);
    a = dpp_add<0x141, 0xf>(a); b = dpp_add<0x141, 0xf>(b); c = dpp_add<0x141, 0xf>(c);
    a = dpp_add<0x140, 0xf>(a); b = dpp_add<0x140, 0xf>(b); c = dpp_add<0x140, 0xf>(c);
    a = dpp_add<0x142, 0xa>(a); b = dpp_add<0x142, 0xa>(b); c = dpp_add<0x142, 0xa>(c);
    a = dpp_add<0x143, 0xc>(a); b = dpp_add<0x143, 0xc>(b); c = dpp_add<0x143, 0xc>(c);
    if constexpr (NT == kWave) {
        a = readlane_f(a, 63);
        b = readlane_f(b, 63);
        c = readlane_f(c, 63);
        return red;
    } else {
        constexpr int NW = NT / kWave;
        constexpr int NQ = NW < 4 ? 4 : NW;
        float* q = red + phase * 3 * NQ;
        phase ^= 1;
        if (lane_id() == 63) {
            const int w = threadIdx.x >> 6;
            q[w] = a;
            q[NQ + w] = b;
            q[2 * NQ + w] = c;
        }
        __syncthreads();
        return q;
    }
}

template <int NT>
__device__ __forceinline__ void block_sum3_read(const float* q, float& a, float& b, float& c) {
    if constexpr (NT > kWave) {
        constexpr int NW = NT / kWave;
        constexpr int NQ = NW < 4 ? 4 : NW;
        a = b = c = 0.f;
        if constexpr (NW == 2 || NW == 4 || NW == 8 || NW == 16) {
            // one ds_read_b32 per lane (lane l < 3 NW: partial l % NW of value l / NW) and DPP
            // sums over aligned groups of NW lanes, instead of 3 NW / 4 ds_read_b128 that every
            // lane of every wave repeats (8 LDS cycles each, all waves right after the barrier)
            const int lane = lane_id();
            const int idx = (lane / NW) * NQ + lane % NW;
            const float t = q[lane < 3 * NW ? idx : 0];
            float v = lane < 3 * NW ? t : 0.f;
            v = dpp_add<0xB1, 0xf>(v);                              // pairs
            if constexpr (NW >= 4) v = dpp_add<0x4E, 0xf>(v);       // quads
            if constexpr (NW >= 8) v = dpp_add<0x141, 0xf>(v);      // half rows
            if constexpr (NW >= 16) v = dpp_add<0x140, 0xf>(v);     // rows
            a = readlane_f(v, 0);
            b = readlane_f(v, NW);
            c = readlane_f(v, 2 * NW);
        } else if constexpr (NW % 4 == 0) {
#pragma unroll
            for (int w = 0; w < NW; w += 4) {
                const f32x4 va = *reinterpret_cast<const f32x4*>(q + w);
                const f32x4 vb = *reinterpret_cast<const f32x4*>(q + NQ + w);
                const f32x4 vc = *reinterpret_cast<const f32x4*>(q + 2 * NQ + w);
                a += va.x; a += va.y; a += va.z; a += va.w;
                b += vb.x; b += vb.y; b += vb.z; b += vb.w;
                c += vc.x; c += vc.y; c += vc.z; c += vc.w;
            }
        } else {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                a += q[w];
                b += q[NQ + w];
                c += q[2 * NQ + w];
            }
        }
    }
}

// Block-wide sum of three values in one LDS exchange (the single-reduction CG).  Partials
// are laid out [value][wave] so each total is read with 16-B loads; fixed order everywhere.
template <int NT>
__device__ __forceinline__ void block_sum3(float& a, float& b, float& c, float* red, int& phase) {
    const float* q = block_sum3_post<NT>(a, b, c, red, phase);
    block_sum3_read<NT>(q, a, b, c);
}

// Wave-uniform maximum of a small non-negative int (setup only).
__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int o = __shfl_xor(v, off);
        v = o > v ? o : v;
    }
    return __builtin_amdgcn_readfirstlane(v);
}


// Exclusive prefix sum of one int per thread over the block; `total` gets the block sum.
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* scratch, int& total) {
    const int lane = lane_id();
    int incl = v;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
    }
    if constexpr (NT == kWave) {
        total = __shfl(incl, kWave - 1);
        return incl - v;
    } else {
        constexpr int NW = NT / kWave;
        const int w = threadIdx.x >> 6;
        if (lane == kWave - 1) scratch[w] = incl;
        __syncthreads();
        int before = 0, all = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            const int sw = scratch[q];
            before += q < w ? sw : 0;
            all += sw;
        }
        total = all;
        return before + incl - v;
    }
}

// MODE: 3 Chronopoulos-Gear with a first-order Neumann preconditioner (below; the default where
// a thread owns one row), 1 Chronopoulos-Gear (one reduction, two barriers per iteration).
// (Measured and removed in round 4, DESIGN.md §3.2: the classic two-reduction form and the
// pipelined Ghysels-Vanroose form.)
// The kernel body: `gxy` = (column, graph); `fsync` (the fused backward, cg_grad_fused_kernel)
// non-null: the solution is stored write-through (sc1) and, once every wave has drained its
// stores, thread 0 adds 1 to fsync[0] -- the feature-gradient workgroups of the same launch
// wait for C arrivals (the hand-off protocol of DESIGN.md §3.5).
template <int NT, int R, int S, typename TB, int MODE>
__device__ __forceinline__ void cg_ell_body(
    int2 gxy, unsigned* fsync,
    int m, int C, int base, const int32_t* __restrict__ row_start,
    const int32_t* __restrict__ row_len, const int32_t* __restrict__ ucnt,
    const int32_t* __restrict__ col, const float* __restrict__ wv, const float* __restrict__ diag,
    const TB* __restrict__ bsrc, double* __restrict__ out64, float* __restrict__ out32,
    float rtol, int max_iter, int mat_cap, int32_t* __restrict__ st_nonconv,
    int32_t* __restrict__ st_iters, const int4* __restrict__ ell, size_t wss, size_t bs,
    size_t us, size_t sts) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    ell = gshift_at(ell, wss, gxy.y);
    row_start = gshift_br_at(row_start, wss, gxy.y);   // batched launches: graph blockIdx.y
    row_len = gshift_br_at(row_len, wss, gxy.y);
    ucnt = gshift_at(ucnt, wss, gxy.y);
    col = gshift_br_at(col, wss, gxy.y);
    wv = gshift_br_at(wv, wss, gxy.y);
    diag = gshift_at(diag, wss, gxy.y);
    bsrc = gshift_at(bsrc, bs, gxy.y);
    out64 = gshift_br_at(out64, us, gxy.y);
    out32 = gshift_br_at(out32, wss, gxy.y);
    st_nonconv = gshift_br_at(st_nonconv, sts, gxy.y);
    st_iters = gshift_br_at(st_iters, sts, gxy.y);
    const int c = gxy.x;
    const int tid = threadIdx.x;
    float* red = smem;                                  // 96 floats of reduction scratch
    int* scan = reinterpret_cast<int*>(smem + 96);      // 16 ints of scan scratch
    const int mp4 = (m + 3) & ~3;
    float* P_ = smem + 128;                             // gathered vector (x2 for MODE 3)
    int* lcol = reinterpret_cast<int*>(P_ + (MODE == 3 ? 2 : 1) * mp4);   // overflow, compacted
    float* lw = reinterpret_cast<float*>(lcol + mat_cap);
    // (Ordering rows by length so each wave's slot bound tracks its own rows was measured:
    // no gain per iteration at NS, +1.5 us of setup from the permuted ELL loads.)
    int urow[R];   // the row each thread slot handles
#pragma unroll
    for (int q = 0; q < R; ++q) urow[q] = tid + NT * q;
    int ec[R][S];
    float ew[R][S];
    int ost[R], olen[R];
    float x[R], r[R], p[R], ap[R], mi[R], dg[R];
    float rz = 0.f, bb = 0.f;
    int tov = 0;
    GLL_TRACE_SCOPE(0);
    GLL_TRACE_PT(0);
    // Every global load of the setup is issued before the first barrier (the U-block lengths,
    // the ELL slices, the diagonal and the right-hand side), so the prologue pays one memory
    // latency, not one per dependent step.
    int ulen[R];
    float bv[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int u = urow[q];
        const int uc = u < m ? u : 0;
        ulen[q] = ucnt[uc];
        static_assert(S % 2 == 0, "two ELL slots per 16-B record");
#pragma unroll
        for (int s2 = 0; s2 < S / 2; ++s2) {   // column-major ELL records (row_build): coalesced
            const int4 v = ell[size_t(s2) * m + uc];
            ec[q][2 * s2] = v.x;
            ew[q][2 * s2] = __int_as_float(v.y);
            ec[q][2 * s2 + 1] = v.z;
            ew[q][2 * s2 + 1] = __int_as_float(v.w);
        }
        dg[q] = diag[uc];
        bv[q] = to_f32(bsrc[size_t(uc) * C + c]);
    }
    // entries past the S ELL slots exist only when some U block is longer than S: one
    // workgroup-wide OR (a single barrier) decides, so the usual case skips the overflow scan
    int longer = 0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        if (urow[q] >= m) ulen[q] = 0;
        longer |= ulen[q] > S ? 1 : 0;
    }
    const bool has_ovf = __syncthreads_or(longer) != 0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int u = urow[q];
        x[q] = r[q] = p[q] = ap[q] = mi[q] = 0.f;
        if (u >= m) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
                ec[q][s] = 0;
                ew[q][s] = 0.f;
            }
            dg[q] = 0.f;
        }
        ost[q] = 0;
        olen[q] = 0;
        if (has_ovf && u < m) {
            const int len = ulen[q];   // U block = sorted suffix of graph row base + u
            ost[q] = row_start[base + u] + row_len[base + u] - len + S;
            olen[q] = len - S;
            tov += olen[q] > 0 ? olen[q] : 0;
        }
        if (u < m) {
            mi[q] = dg[q] > 0.f ? 1.f / dg[q] : 0.f;
            r[q] = mi[q] > 0.f ? bv[q] : 0.f;   // zero-diagonal rows are decoupled: x = 0
            p[q] = mi[q] * r[q];
            P_[u] = p[q];
            rz += r[q] * p[q];
            bb += r[q] * r[q];
        }
    }
    GLL_TRACE_PT(1);
    // entries beyond the ELL slices: compact them into LDS when they fit
    int ov_total = 0;
    int ooff = has_ovf ? block_excl_scan<NT>(tov, scan, ov_total) : 0;
    const bool matl = ov_total <= mat_cap;
    if (has_ovf && matl) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            for (int t = 0; t < olen[q]; ++t) {
                const int e = ost[q] + t;
                lcol[ooff + t] = col[e] - base;
                lw[ooff + t] = wv[e];
            }
            if (olen[q] > 0) {
                ost[q] = ooff;
                ooff += olen[q];
            }
        }
    }
    GLL_TRACE_PT(2);
    int phase = 0;
    if constexpr (NT > kWave) __syncthreads();
    int it = 0;
    bool conv;
    static_assert(MODE == 1 || MODE == 3, "MODE: 1 Chronopoulos-Gear, 3 with Neumann-1");
    {
        // Each wave gathers only the ELL slots some row of its own holds (wave-uniform bound
        // in groups of 4: rows average ~6 of the 24 slots at NS).
        int smax[R];
#pragma unroll
        for (int q = 0; q < R; ++q) smax[q] = wave_max_int(ulen[q] < S ? ulen[q] : S);
        auto spmv = [&](int q, float pq, const float* Pb) {
            float pv[S];
#pragma unroll
            for (int s0 = 0; s0 < S; s0 += 4) {
                if (s0 < smax[q]) {
#pragma unroll
                    for (int t = 0; t < 4 && s0 + t < S; ++t) pv[s0 + t] = Pb[ec[q][s0 + t]];
                } else {
#pragma unroll
                    for (int t = 0; t < 4 && s0 + t < S; ++t) pv[s0 + t] = 0.f;
                }
            }
            // slots past the wave's bound hold weight 0: their products are skipped, not summed
            float acc = 0.f;
#pragma unroll
            for (int s0 = 0; s0 < S; s0 += 4)
                if (s0 < smax[q]) {
#pragma unroll
                    for (int t = 0; t < 4 && s0 + t < S; ++t) acc += ew[q][s0 + t] * pv[s0 + t];
                }
            if (matl) {
                // four entries per step, every LDS read issued before use (same summation
                // order as one at a time); rows past the slots are long at K = 25
                const int e0 = ost[q], no = olen[q];
                int t = 0;
                for (; t + 4 <= no; t += 4) {
                    int c4[4];
                    float w4[4], p4[4];
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        c4[v] = lcol[e0 + t + v];
                        w4[v] = lw[e0 + t + v];
                    }
#pragma unroll
                    for (int v = 0; v < 4; ++v) p4[v] = Pb[c4[v]];
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc += w4[v] * p4[v];
                }
                for (; t < no; ++t) acc += lw[e0 + t] * Pb[lcol[e0 + t]];
            } else {   // from the CSR (L2), four entries in flight per step
                const int e0 = ost[q], no = olen[q];
                int t = 0;
                for (; t + 4 <= no; t += 4) {
                    int c4[4];
                    float w4[4], p4[4];
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        c4[v] = col[e0 + t + v];
                        w4[v] = wv[e0 + t + v];
                    }
#pragma unroll
                    for (int v = 0; v < 4; ++v) p4[v] = Pb[c4[v] - base];
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc += w4[v] * p4[v];
                }
                for (; t < no; ++t) acc += wv[e0 + t] * Pb[col[e0 + t] - base];
            }
            return dg[q] * pq - acc;   // (Luu u)_row = (deg + tau) u_row - sum_j W_rowj u_j
        };
        {
        // Chronopoulos-Gear single-reduction PCG: one fused (r.u, w.u, r.r) exchange and one
        // publish barrier per iteration (classic PCG: two exchanges + publish = 3 barriers).
        // s = A p by recurrence; u = M^-1 r is what is published and multiplied.
        // MODE 3: M^-1 = D^-1 + D^-1 N D^-1 (A = D - N, N the off-diagonal weights W_uj >= 0:
        // the first two terms of the Neumann series of A^-1), applied as y = D^-1 r published,
        // u = y + D^-1 (N y) -- one more gather and barrier per iteration.  It is SPD where
        // D^-1/2 A D^-1/2 has its spectrum in (0, 2), which diagonal dominance gives, and turns
        // that spectrum [l, h] into {x (2 - x)}: at NS [0.44, 1.32] -> [0.69, 1], 11 -> 6
        // iterations, so each iteration's fixed reduction and step-size latency is paid about
        // half as often (tools/ab_flags.py).
        constexpr bool NEU = MODE == 3;
        float* P2_ = P_ + mp4;   // y = D^-1 r (MODE 3)
        if constexpr (NEU) {
            // setup left y0 = D^-1 r0 in P_ (as p) and rz = (r0, y0): u0 = y0 + D^-1 N y0
            rz = 0.f;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const float t = -spmv(q, 0.f, P_);   // (N y0)_row
                p[q] = p[q] + mi[q] * t;
                rz += r[q] * p[q];
            }
            __syncthreads();   // every gather of y0 is done before u0 overwrites it
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int u = urow[q];
                if (u < m) P_[u] = p[q];
            }
            __syncthreads();
        }
        // pre-step: w0 = A u0 (u0 = p, already published), gamma0 = (r,u), delta0 = (w,u)
        float sv[R];
        float dl = 0.f;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            sv[q] = spmv(q, p[q], P_);
            dl += p[q] * sv[q];
        }
        block_sum3<NT>(rz, bb, dl, red, phase);
        GLL_TRACE_PT(3);
        const float tol2 = rtol * rtol * bb;
        conv = !(bb > 0.f);
        float gam = rz;
        float alpha = dl > 0.f ? gam / dl : 0.f;
        if (!(dl > 0.f)) alpha = -1.f;   // breakdown before the first step
#ifdef GLL_TRACE
#define GLL_TRACE_CYC(i)                                                                       \
    do {                                                                                       \
        if (it == 3 && blockIdx.x == 0 && threadIdx.x == 0) g_trace[i] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define GLL_TRACE_CYC(i) do {} while (0)
#endif
        while (!conv && alpha > 0.f && it < max_iter) {
            ++it;
            GLL_TRACE_CYC(10);
#pragma unroll
            for (int q = 0; q < R; ++q) {
                x[q] += alpha * p[q];
                r[q] -= alpha * sv[q];
                ap[q] = mi[q] * r[q];                       // u = M^-1 r (MODE 3: y)
                const int u = urow[q];
                if (u < m) (NEU ? P2_ : P_)[u] = ap[q];
            }
            if constexpr (NEU) {   // u = y + D^-1 (N y)
                __syncthreads();
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    ap[q] += mi[q] * -spmv(q, 0.f, P2_);
                    const int u = urow[q];
                    if (u < m) P_[u] = ap[q];
                }
            }
            GLL_TRACE_CYC(11);
            if constexpr (NT > kWave) __syncthreads();
            if (it == 1) GLL_TRACE_PT(4);
            GLL_TRACE_CYC(12);
            float gn = 0.f, de = 0.f, rr = 0.f;
            float w[R];
#pragma unroll
            for (int q = 0; q < R; ++q) {
                w[q] = spmv(q, ap[q], P_);
                gn += r[q] * ap[q];
                de += w[q] * ap[q];
                rr += r[q] * r[q];
            }
#ifdef GLL_TRACE
            if (it == 3 && blockIdx.x == 0 && threadIdx.x == 0 && de == 12345.f) g_trace[9] = 0;
#endif
            GLL_TRACE_CYC(13);
            block_sum3<NT>(gn, de, rr, red, phase);
            GLL_TRACE_CYC(14);
            if (it == 1) GLL_TRACE_PT(6);
            if (rr <= tol2) {
                conv = true;
                break;
            }
            // one reciprocal on the critical path: alpha' = gn / (de - beta gn / alpha)
            //                                             = gn alpha / (alpha de - beta gn)
            const float beta = gn * __builtin_amdgcn_rcpf(gam);
            const float den = alpha * de - beta * gn;
            if (!(den > 0.f)) break;   // breakdown or NaN: reported as non-converged
            alpha = (gn * alpha) * __builtin_amdgcn_rcpf(den);
            gam = gn;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                p[q] = ap[q] + beta * p[q];
                sv[q] = w[q] + beta * sv[q];
            }
            GLL_TRACE_CYC(15);
        }
        }
    }
    GLL_TRACE_PT(8);
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int u = urow[q];
        if (u < m) {
            if (out64) out64[size_t(u) * C + c] = double(x[q]);
            if (out32) {
                if (fsync)
                    __hip_atomic_store(out32 + size_t(u) * C + c, x[q], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);   // global_store ... sc1
                else
                    out32[size_t(u) * C + c] = x[q];
            }
        }
    }
    if (tid == 0) {
        if (st_iters && (sts != 0 || gxy.y == 0 || !conv)) atomicMax(st_iters, it);   // sink: see gll.h
        if (!conv && st_nonconv) atomicAdd(st_nonconv, 1);
    }
    if (fsync) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // the column completing the count writes the release word the gradient blocks poll
        // (on its own line: the pollers never read the line the arrivals add to)
        if (tid == 0 &&
            __hip_atomic_fetch_add(fsync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u ==
                unsigned(C))
            __hip_atomic_store(fsync + 96, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    GLL_TRACE_PT(9);
}

// The batched geometry (256 x 2, MODE 1: B x C > 256 column workgroups) must keep three
// workgroups per CU -- B = 64 NS is 640 of them, all resident at once -- so <= 168 VGPRs.
template <int NT, int R, int S, typename TB, int MODE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 && R == 2 && MODE == 1 ? 3 : 1)))
void cg_ell_kernel(
    int m, int C, int base, const int32_t* __restrict__ row_start,
    const int32_t* __restrict__ row_len, const int32_t* __restrict__ ucnt,
    const int32_t* __restrict__ col, const float* __restrict__ wv, const float* __restrict__ diag,
    const TB* __restrict__ bsrc, double* __restrict__ out64, float* __restrict__ out32,
    float rtol, int max_iter, int mat_cap, int32_t* __restrict__ st_nonconv,
    int32_t* __restrict__ st_iters, const int4* __restrict__ ell, size_t wss, size_t bs,
    size_t us, size_t sts) {
    // batch_xy once: per pointer it re-reads gridDim and divides
    cg_ell_body<NT, R, S, TB, MODE>(batch_xy<true>(), nullptr, m, C, base, row_start, row_len,
                                    ucnt, col, wv, diag, bsrc, out64, out32, rtol, max_iter,
                                    mat_cap, st_nonconv, st_iters, ell, wss, bs, us, sts);
}

// --------------------------------------------------------------------------------------
// Balanced per-column CG for long U rows (cg_vr_kernel).
//
// At K = 25 (the FullySup caller, FullySup.py:156) a U row of Luu holds 27 entries on average
// and up to ~75, so a thread-per-row SpMV loops every wave to its longest row, and past the
// register slots each entry costs three LDS operations (column, weight, gathered value).
// Here the U block is cut into "virtual rows" of kVS = 8 consecutive entries (a row of L
// entries gives ceil(L/8)), which row_build writes pre-packed (16-bit LDS byte offsets of the
// columns, then the weights; gll_internal.h kVrSlot).  The virtual rows -- not the rows -- are
// dealt out to the threads, v = j * NT + tid for j < RV, and held in registers for the whole
// solve.  An SpMV is then one LDS gather per entry, the same count for every thread, plus one
// partial sum per virtual row written to LDS.
//
// The row sums of A u are needed only after the iteration's reduction barrier (for the
// recurrence s = w + beta s), so they are read there from the partials -- no extra barrier.
// The (w, u) product the reduction needs before that barrier is formed per virtual row
// instead: (w, u) = sum_rows diag u^2 - sum_v u_row(v) part_v.
// Fixed partition and fixed summation order: deterministic.  Virtual rows past the register
// capacity NT x RV (an underestimated size) or past the VRM slots of a row (hubs) are summed
// by their row's thread from the CSR.
// --------------------------------------------------------------------------------------
template <int NT, int R, int RV, typename TB>
__global__ __launch_bounds__(NT) void cg_vr_kernel(
    int m, int C, int base, int VRM, const int32_t* __restrict__ row_start,
    const int32_t* __restrict__ row_len, const int32_t* __restrict__ ucnt,
    const int32_t* __restrict__ col, const float* __restrict__ wv, const float* __restrict__ diag,
    const char* __restrict__ vrs, const TB* __restrict__ bsrc, double* __restrict__ out64,
    float* __restrict__ out32, float rtol, int max_iter, int32_t* __restrict__ st_nonconv,
    int32_t* __restrict__ st_iters, size_t wss, size_t bs, size_t us, size_t sts) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int2 gxy = batch_xy<true>();   // once: per pointer it re-reads gridDim and divides
    row_start = gshift_at(row_start, wss, gxy.y);
    row_len = gshift_at(row_len, wss, gxy.y);
    ucnt = gshift_at(ucnt, wss, gxy.y);
    col = gshift_at(col, wss, gxy.y);
    wv = gshift_at(wv, wss, gxy.y);
    diag = gshift_at(diag, wss, gxy.y);
    vrs = gshift_at(vrs, wss, gxy.y);
    bsrc = gshift_at(bsrc, bs, gxy.y);
    out64 = gshift_br_at(out64, us, gxy.y);
    out32 = gshift_br_at(out32, wss, gxy.y);
    st_nonconv = gshift_br_at(st_nonconv, sts, gxy.y);
    st_iters = gshift_br_at(st_iters, sts, gxy.y);
    constexpr int VCAP = NT * RV;
    const int c = gxy.x;
    const int tid = threadIdx.x;
    const int mp4 = (m + 3) & ~3;
    float* red = smem;                                   // 96 floats of reduction scratch
    int* scan = reinterpret_cast<int*>(smem + 96);       // 16 ints of scan scratch
    float* P_ = smem + 128;                              // the published vector u
    // partial sums, row-padded: row u's at vpart[vpad_u ..), vpad_u 16-B aligned, so the row
    // sums read them four at a time
    float* vpart = P_ + mp4;                             // VCAP + 4 mp4
    int* vmap = reinterpret_cast<int*>(vpart + VCAP + 4 * mp4);   // VCAP: (row << 10) | (j << 4) | len
    int* vpad = vmap + VCAP;                             // mp4: row u's first partial
    GLL_TRACE_SCOPE(0);
    GLL_TRACE_PT(0);

    // ---- rows this thread owns (u = tid + NT q): setup loads all issued together
    int ulen[R], est[R], vs[R], nvc[R], sps[R], spe[R], vp[R];
    float dg[R], bv[R], mi[R], x[R], r[R], p[R], sv[R], uu[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int u = tid + NT * q;
        const int uc = u < m ? u : 0;
        ulen[q] = ucnt[uc];
        est[q] = row_start[base + uc] + row_len[base + uc];
        dg[q] = diag[uc];
        bv[q] = to_f32(bsrc[size_t(uc) * C + c]);
    }
    int tv = 0, tp = 0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        if (tid + NT * q >= m) {
            ulen[q] = 0;
            dg[q] = 0.f;
        }
        est[q] -= ulen[q];   // the U block is the row's sorted suffix
        const int nv = min((ulen[q] + kVS - 1) / kVS, VRM);
        tv += nv;
        tp += (nv + 3) & ~3;
    }
    int V = 0, VP = 0;
    int v0 = block_excl_scan<NT>(tv, scan, V);
    __syncthreads();   // the scan scratch is reused
    int p0 = block_excl_scan<NT>(tp, scan, VP);
    float rz = 0.f, bb = 0.f;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int u = tid + NT * q;
        const int nv = min((ulen[q] + kVS - 1) / kVS, VRM);
        vs[q] = v0;
        vp[q] = p0;
        if (u < m) vpad[u] = p0;
        p0 += (nv + 3) & ~3;
        for (int j = 0; j < nv && v0 + j < VCAP; ++j)
            vmap[v0 + j] = (u << 10) | (j << 4) | min(kVS, ulen[q] - kVS * j);
        nvc[q] = v0 + nv <= VCAP ? nv : (v0 < VCAP ? VCAP - v0 : 0);
        if (nvc[q] == 0) vp[q] = 0;   // no partials held (past the capacity): stay in bounds
        sps[q] = est[q] + kVS * nvc[q];   // entries past the held virtual rows: from the CSR
        spe[q] = est[q] + ulen[q];
        v0 += nv;
        mi[q] = dg[q] > 0.f ? 1.f / dg[q] : 0.f;
        r[q] = mi[q] > 0.f ? bv[q] : 0.f;   // zero-diagonal rows are decoupled: x = 0
        x[q] = sv[q] = 0.f;
        p[q] = uu[q] = mi[q] * r[q];
        if (u < m) P_[u] = uu[q];
        rz += r[q] * uu[q];
        bb += r[q] * r[q];
    }
    // wave-uniform bound of the partial sums each row reads after the reduction
    int nvmax[R];
#pragma unroll
    for (int q = 0; q < R; ++q) nvmax[q] = wave_max_int(nvc[q]);
    GLL_TRACE_PT(1);
    __syncthreads();
    // ---- this thread's virtual rows, packed by row_build: 3 x 16-B loads each, consecutive
    // threads on consecutive virtual rows
    uint32_t cpk[RV][kVS / 2];
    float ew[RV][kVS];
    int vrow[RV], vmax[RV], pidx[RV];
    const int Vlive = V < VCAP ? V : VCAP;
#pragma unroll
    for (int j = 0; j < RV; ++j) {
        const int v = j * NT + tid;
        const int info = vmap[v < Vlive ? v : 0];
        const int len = v < Vlive ? (info & 15) : 0;
        vrow[j] = v < Vlive ? (info >> 10) : 0;
        pidx[j] = v < Vlive ? vpad[info >> 10] + ((info >> 4) & 63) : VCAP + 4 * mp4 - 1;
        const int slot = v < Vlive ? (info >> 10) * VRM + ((info >> 4) & 63) : 0;
        const uint4 cw = *reinterpret_cast<const uint4*>(vrs + size_t(slot) * kVrSlot);
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(vrs + size_t(slot) * kVrSlot + 16);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(vrs + size_t(slot) * kVrSlot + 32);
        // a dead slot loads virtual row 0: masked through an opaque mask (a select on the
        // loaded values would let the compiler sink the loads into a branch)
        uint32_t mk = v < Vlive ? 0xffffffffu : 0u;
        asm volatile("" : "+v"(mk));
        cpk[j][0] = cw.x & mk;
        cpk[j][1] = cw.y & mk;
        cpk[j][2] = cw.z & mk;
        cpk[j][3] = cw.w & mk;
        ew[j][0] = __uint_as_float(__float_as_uint(w0.x) & mk);
        ew[j][1] = __uint_as_float(__float_as_uint(w0.y) & mk);
        ew[j][2] = __uint_as_float(__float_as_uint(w0.z) & mk);
        ew[j][3] = __uint_as_float(__float_as_uint(w0.w) & mk);
        ew[j][4] = __uint_as_float(__float_as_uint(w1.x) & mk);
        ew[j][5] = __uint_as_float(__float_as_uint(w1.y) & mk);
        ew[j][6] = __uint_as_float(__float_as_uint(w1.z) & mk);
        ew[j][7] = __uint_as_float(__float_as_uint(w1.w) & mk);
        vmax[j] = wave_max_int(len);
    }
    GLL_TRACE_PT(3);
    const char* Pb = reinterpret_cast<const char*>(P_);
    // A u over this thread's virtual rows: partials to LDS, returns sum_v u_row(v) part_v
    auto spmv = [&]() {
        float dl = 0.f;
        // the packed offsets are "redefined" here so the compiler cannot hoist their unpacked
        // halves out of the iteration loop (that doubles the registers they take)
#pragma unroll
        for (int j = 0; j < RV; ++j)
#pragma unroll
            for (int h = 0; h < kVS / 2; ++h) asm volatile("" : "+v"(cpk[j][h]));
#pragma unroll
        for (int j = 0; j < RV; ++j) {
            if (vmax[j] > 0) {
                float pv[kVS];
#pragma unroll
                for (int k0 = 0; k0 < kVS; k0 += 4) {
                    if (k0 < vmax[j]) {
#pragma unroll
                        for (int k = k0; k < k0 + 4; ++k) {
                            const uint32_t off = (k & 1) ? (cpk[j][k >> 1] >> 16)
                                                         : (cpk[j][k >> 1] & 0xffffu);
                            pv[k] = *reinterpret_cast<const float*>(Pb + off);
                        }
                    } else {
#pragma unroll
                        for (int k = k0; k < k0 + 4; ++k) pv[k] = 0.f;
                    }
                }
                const float ur = P_[vrow[j]];
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < kVS; ++k) acc += ew[j][k] * pv[k];
                vpart[pidx[j]] = acc;
                dl += ur * acc;
            }
            // one virtual row's gathers in flight at a time: hoisting all RV x 8 spills
            __builtin_amdgcn_sched_barrier(0);
        }
        return dl;
    };
    // entries past the held virtual rows (rare): this row's thread sums them from the CSR
    auto spill = [&](int q) {
        float acc = 0.f;
        for (int e = sps[q]; e < spe[q]; ++e) acc += wv[e] * P_[col[e] - base];
        return acc;
    };
    // after the reduction barrier: (A u)_row = diag u - sum of the row's partials; the loads
    // of every row of the thread are issued together, four partials per row per step
    // the first 8 of a row's partials (rows up to 64 entries) come in two 16-B loads per row,
    // every row's issued before any is used; longer rows loop over the rest
    const int vplim = VCAP + 4 * mp4 - 4;
    auto rowsums = [&](float* wr, const float* spl) {
        f32x4 pv[R][2];
#pragma unroll
        for (int q = 0; q < R; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                pv[q][h] = *reinterpret_cast<const f32x4*>(vpart + min(vp[q] + 4 * h, vplim));
#pragma unroll
        for (int q = 0; q < R; ++q) {
            float acc = 0.f;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                acc += 4 * h + 0 < nvc[q] ? pv[q][h].x : 0.f;
                acc += 4 * h + 1 < nvc[q] ? pv[q][h].y : 0.f;
                acc += 4 * h + 2 < nvc[q] ? pv[q][h].z : 0.f;
                acc += 4 * h + 3 < nvc[q] ? pv[q][h].w : 0.f;
            }
            for (int t = 8; t < nvmax[q]; ++t) acc += t < nvc[q] ? vpart[vp[q] + t] : 0.f;
            wr[q] = dg[q] * uu[q] - (acc + spl[q]);
        }
    };

    int phase = 0;
    int it = 0;
    bool conv;
    // pre-step: w0 = A u0, gamma0 = (r,u), delta0 = (w,u)
    float spl[R];
    float dl = -spmv();
#pragma unroll
    for (int q = 0; q < R; ++q) {
        spl[q] = spill(q);
        dl += dg[q] * uu[q] * uu[q] - uu[q] * spl[q];
    }
    block_sum3<NT>(rz, bb, dl, red, phase);
    rowsums(sv, spl);
    GLL_TRACE_PT(4);
    const float tol2 = rtol * rtol * bb;
    conv = !(bb > 0.f);
    float gam = rz;
    float alpha = dl > 0.f ? gam / dl : 0.f;
    if (!(dl > 0.f)) alpha = -1.f;   // breakdown before the first step
    while (!conv && alpha > 0.f && it < max_iter) {
        ++it;
        GLL_TRACE_CYC(10);
#pragma unroll
        for (int q = 0; q < R; ++q) {
            x[q] += alpha * p[q];
            r[q] -= alpha * sv[q];
            uu[q] = mi[q] * r[q];                       // u = M^-1 r
            const int u = tid + NT * q;
            if (u < m) P_[u] = uu[q];
        }
        GLL_TRACE_CYC(11);
        __syncthreads();
        GLL_TRACE_CYC(12);
        float gn = 0.f, de = -spmv(), rr = 0.f;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            spl[q] = spill(q);
            gn += r[q] * uu[q];
            de += dg[q] * uu[q] * uu[q] - uu[q] * spl[q];
            rr += r[q] * r[q];
        }
#ifdef GLL_TRACE
        if (it == 3 && blockIdx.x == 0 && threadIdx.x == 0 && de == 12345.f) g_trace[9] = 0;
#endif
        GLL_TRACE_CYC(13);
        block_sum3<NT>(gn, de, rr, red, phase);
        GLL_TRACE_CYC(14);
        float w[R];
        rowsums(w, spl);
        if (rr <= tol2) {
            conv = true;
            break;
        }
        const float beta = gn * __builtin_amdgcn_rcpf(gam);
        const float den = alpha * de - beta * gn;
        if (!(den > 0.f)) break;   // breakdown or NaN: reported as non-converged
        alpha = (gn * alpha) * __builtin_amdgcn_rcpf(den);
        gam = gn;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            p[q] = uu[q] + beta * p[q];
            sv[q] = w[q] + beta * sv[q];
        }
        GLL_TRACE_CYC(15);
    }
    GLL_TRACE_PT(8);
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int u = tid + NT * q;
        if (u < m) {
            if (out64) out64[size_t(u) * C + c] = double(x[q]);
            if (out32) out32[size_t(u) * C + c] = x[q];
        }
    }
    if (tid == 0) {
        if (st_iters && (sts != 0 || gxy.y == 0 || !conv)) atomicMax(st_iters, it);   // sink: see gll.h
        if (!conv && st_nonconv) atomicAdd(st_nonconv, 1);
    }
}

// Large systems: vectors in LDS (<= 160 KiB) or in the workspace.
template <int NT, typename TB>
__global__ __launch_bounds__(NT) void cg_lds_kernel(
    int m, int C, int base, const int32_t* __restrict__ row_start,
    const int32_t* __restrict__ row_len, const int32_t* __restrict__ ucnt,
    const int32_t* __restrict__ col,
    const float* __restrict__ wv, const float* __restrict__ diag, const TB* __restrict__ bsrc,
    double* __restrict__ out64, float* __restrict__ out32, float rtol, int max_iter,
    float* __restrict__ gvec, int vec_in_lds, int32_t* __restrict__ st_nonconv,
    int32_t* __restrict__ st_iters, size_t wss, size_t bs, size_t us, size_t sts) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int2 gxy = batch_xy<true>();   // once: per pointer it re-reads gridDim and divides
    row_start = gshift_at(row_start, wss, gxy.y);
    row_len = gshift_at(row_len, wss, gxy.y);
    ucnt = gshift_at(ucnt, wss, gxy.y);
    col = gshift_at(col, wss, gxy.y);
    wv = gshift_at(wv, wss, gxy.y);
    diag = gshift_at(diag, wss, gxy.y);
    bsrc = gshift_at(bsrc, bs, gxy.y);
    out64 = gshift_at(out64, us, gxy.y);
    out32 = gshift_at(out32, wss, gxy.y);
    gvec = gshift_at(gvec, wss, gxy.y);
    st_nonconv = gshift_at(st_nonconv, sts, gxy.y);
    st_iters = gshift_at(st_iters, sts, gxy.y);
    const int c = gxy.x;
    const int tid = threadIdx.x;
    float* red = smem;
    float* vb = vec_in_lds ? smem + 64 : gvec + size_t(c) * 5 * m;
    float *X_ = vb, *R_ = vb + m, *P_ = vb + 2 * m, *A_ = vb + 3 * m, *M_ = vb + 4 * m;
    float rz = 0.f, bb = 0.f;
    for (int u = tid; u < m; u += NT) {
        const float dg = diag[u];
        const float mi = dg > 0.f ? 1.f / dg : 0.f;
        const float bu = to_f32(bsrc[size_t(u) * C + c]);
        const float rb = mi > 0.f ? bu : 0.f;
        X_[u] = 0.f;
        R_[u] = rb;
        M_[u] = mi;
        P_[u] = mi * rb;
        rz += rb * mi * rb;
        bb += rb * rb;
    }
    int phase = 0;
    __syncthreads();
    block_sum2<NT>(rz, bb, red, phase);
    const float tol2 = rtol * rtol * bb;
    int it = 0;
    bool conv = !(bb > 0.f);
    while (!conv && it < max_iter) {
        ++it;
        float pap = 0.f, unused = 0.f;
        for (int u = tid; u < m; u += NT) {
            const int i = base + u;
            const int end = row_start[i] + row_len[i];
            float acc = 0.f;
            for (int e = end - ucnt[u]; e < end; ++e) acc += wv[e] * P_[col[e] - base];
            const float ap = diag[u] * P_[u] - acc;
            A_[u] = ap;
            pap += P_[u] * ap;
        }
        block_sum2<NT>(pap, unused, red, phase);
        if (!(pap > 0.f)) break;
        const float alpha = rz / pap;
        float rr = 0.f, rzn = 0.f;
        for (int u = tid; u < m; u += NT) {
            X_[u] += alpha * P_[u];
            const float ru = R_[u] - alpha * A_[u];
            R_[u] = ru;
            rr += ru * ru;
            rzn += ru * M_[u] * ru;
        }
        block_sum2<NT>(rr, rzn, red, phase);
        if (rr <= tol2) {
            conv = true;
            break;
        }
        const float beta = rzn / rz;
        rz = rzn;
        for (int u = tid; u < m; u += NT) P_[u] = M_[u] * R_[u] + beta * P_[u];
        __syncthreads();
    }
    for (int u = tid; u < m; u += NT) {
        if (out64) out64[size_t(u) * C + c] = double(X_[u]);
        if (out32) out32[size_t(u) * C + c] = X_[u];
    }
    if (tid == 0) {
        if (st_iters && (sts != 0 || gxy.y == 0 || !conv)) atomicMax(st_iters, it);   // sink: see gll.h
        if (!conv && st_nonconv) atomicAdd(st_nonconv, 1);
    }
}


template <int NT, int R, int S, typename TB, int MODE>
static hipError_t run_ell(const Layout& L, const Batch& bt, void* ws, const TB* b, size_t bs,
                          double* out64, float* out32, float rtol, int max_iter,
                          int32_t* st_nonconv, int32_t* st_iters, hipStream_t s) {
    size_t lds = 128 * 4 + size_t((L.m + 3) & ~3) * 4 * (MODE == 3 ? 2 : 1);
    // entries past the ELL slices are compacted into LDS up to kOvfLds of them, the rest read
    // from the CSR; batched launches cap them so 4 workgroups still share a CU (a full-LDS
    // request would pin one per CU); a single graph's C workgroups take all the LDS there is
    // (K = 25 rows overflow 16 slots by ~14K entries at m = 1250)
    const int64_t kOvfLds = bt.B == 1 ? int64_t(1) << 30 : 2048;
    const int64_t eu_bound = int64_t(L.m + L.n) * (L.K - 1);
    int64_t cap = int64_t(kLdsDyn - lds) / 8;
    if (cap > eu_bound) cap = eu_bound;
    if (cap > kOvfLds) cap = kOvfLds;
    if (cap < 0) cap = 0;
    lds += size_t(cap) * 8;
    // the kernel holds the first S of the ell_emit(L, B) slots row_build wrote in registers
    // (entries past S come from the CSR through the LDS overflow)
    if (S > ell_emit(L, bt.B)) return hipErrorInvalidValue;
    auto fn = cg_ell_kernel<NT, R, S, TB, MODE>;
    allow_full_lds(reinterpret_cast<const void*>(fn));
    launch_k(fn, dim3(L.C, bt.B), NT, lds, s,
        L.m, L.C, L.base, L.at<int32_t>(ws, L.row_start), L.at<int32_t>(ws, L.row_len),
        L.at<int32_t>(ws, L.ucnt), L.at<int32_t>(ws, L.col), L.at<float>(ws, L.w),
        L.at<float>(ws, L.diag), b, out64, out32, rtol, max_iter, int(cap), st_nonconv, st_iters,
        L.at<int4>(ws, L.ell), bt.ws, bs, bt.u, bt.st);
    return launch_status("solve.hip:run_ell");
}

// ---------------------------------------------------------------------------------------
// Fused backward of one small graph (gll_backward, B = 1, fixed eps, C = 10, m <= 512: the
// north-star shape).  The adjoint solve occupies C workgroups of the GPU for ~15 us while the
// feature gradient waits behind a kernel boundary: dispatch, a gap and then cold loads of X
// rows, the CSR and P.  Here both run in ONE launch: blocks 0..C-1 are the per-column CG
// (cg_ell_body), blocks C.. the whole-row gradient (grad_spmm_kernel's register form, one wave
// per row).  A gradient wave loads everything that does not depend on the solve -- x_i, its
// edges, P_i and P_j, the first EB neighbour rows x_j -- then waits for the C columns (one
// counter, the columns' solution stored write-through), loads w_i, w_j with sc1 loads and
// finishes: the same fma order as grad_spmm_kernel, so the results agree bitwise.  All
// C + n / (NT / 64) workgroups are co-resident (checked against the occupancy at launch), so
// a waiting gradient wave never holds a CU a solve needs.  The last gradient workgroup
// re-arms the counters for the next backward on the same workspace.
struct EllCgArgs {
    int m, C, base;
    const int32_t* row_start;
    const int32_t* row_len;
    const int32_t* ucnt;
    const int32_t* col;
    const float* wv;
    const float* diag;
    const void* b;
    float* out32;
    float rtol;
    int max_iter, mat_cap;
    int32_t* st_nonconv;
    int32_t* st_iters;
    const int4* ell;
};

template <int NT, int S, typename TB, int ND>
__global__ __launch_bounds__(NT) void cg_grad_fused_kernel(EllCgArgs c, EdgeArgs a,
                                                           const float* __restrict__ X,
                                                           float* __restrict__ out,
                                                           unsigned* fsync, int32_t* st_failed) {
    const int C = c.C;
    if (int(blockIdx.x) < C) {
        cg_ell_body<NT, 1, S, TB, 3>(int2{int(blockIdx.x), 0}, fsync, c.m, C, c.base,
                                     c.row_start, c.row_len, c.ucnt, c.col, c.wv, c.diag,
                                     static_cast<const TB*>(c.b), nullptr, c.out32, c.rtol,
                                     c.max_iter, c.mat_cap, c.st_nonconv, c.st_iters, c.ell,
                                     0, 0, 0, 0);
        return;
    }
    // ---- gradient role: one wave per row (C = 10 classes, fixed eps)
    constexpr int NC = 10;
    constexpr int EB = ND <= 2 ? 16 : 8;   // grad_spmm_kernel's single-graph (WIDE) batch
    __shared__ int s_ok;
    const int lane = lane_id();
    // XCD-local rows (round 6).  A row's gradient gathers its neighbours' X rows, and ~86% of
    // kNN edges join rows of one class, so the rows are taken in class order --
    // argmax of P = [Y; U], the forward's output -- and each XCD's workgroups (block b runs on
    // XCD b % 8: dispatch order, §3.5, a speed assumption only) take a contiguous run of that
    // order: an XCD then gathers mostly the X rows of one or two classes, which its L2 holds,
    // instead of every XCD refilling all of X (16 MB of counter bytes for a 2 MB X at NS,
    // profiles/r05zzzz_pmc_ns.json).  Each gradient workgroup sorts the rows itself (a stable
    // counting sort in its LDS) while the adjoint solves run; a row's result does not depend on
    // which wave computes it, so the gradient is bitwise that of the row-index order.
    int i0;
    {
        extern __shared__ __attribute__((aligned(16))) float smem[];
        int* srt = reinterpret_cast<int*>(smem);   // [n] rows in class order
        int* crk = srt + a.n;                      // [n] class << 16 | rank in its 64-row chunk
        const int nch = (a.n + kWave - 1) / kWave;
        int* cnt = crk + a.n;                      // [nch][NC] rows per (chunk, class)
        constexpr int NW = NT / kWave;
        const int w = threadIdx.x >> 6;
        for (int q = w; q < nch; q += NW) {   // wave-uniform
            const int i = q * kWave + lane;
            int cls = -1;
            if (i < a.n) {
                float bv = -3.0e38f;
                cls = 0;
#pragma unroll
                for (int k = 0; k < NC; k += 2) {
                    const f32x2 v = *reinterpret_cast<const f32x2*>(a.P + size_t(i) * NC + k);
                    if (v.x > bv) bv = v.x, cls = k;
                    if (v.y > bv) bv = v.y, cls = k + 1;
                }
            }
            int rnk = 0;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const uint64_t mk = __ballot(cls == k);
                if (cls == k) rnk = lanes_below(mk);
                if (lane == k) cnt[q * NC + k] = __popcll(mk);
            }
            if (i < a.n) crk[i] = (cls << 16) | rnk;
        }
        __syncthreads();
        if (threadIdx.x < NC) {   // each (chunk, class) run's first position, class-major
            const int k = threadIdx.x;
            int before = 0;
            for (int kk = 0; kk < k; ++kk)
                for (int q = 0; q < nch; ++q) before += cnt[q * NC + kk];
            for (int q = 0; q < nch; ++q) {
                const int c0 = cnt[q * NC + k];
                cnt[q * NC + k] = before;
                before += c0;
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < a.n; i += NT) {
            const int v = crk[i];
            srt[cnt[(i / kWave) * NC + (v >> 16)] + (v & 0xffff)] = i;
        }
        __syncthreads();
        // this workgroup's rank in XCD-major order of the gradient workgroups
        const int G = int(gridDim.x) - C, b = int(blockIdx.x), x = b & 7;
        int ord = 0;
#pragma unroll
        for (int xx = 0; xx < 8; ++xx) {
            const int f = C + ((xx - C % 8 + 8) & 7);   // first gradient block on XCD xx
            const int cx = f < C + G ? (C + G - 1 - f) / 8 + 1 : 0;
            if (xx < x) ord += cx;
        }
        ord += (b - (C + ((x - C % 8 + 8) & 7))) >> 3;
        const int pos = ord * NW + w;
        i0 = pos < a.n ? srt[pos] : a.n;
    }
    const bool live = i0 < a.n;
    const int i = live ? i0 : 0;
    const int d = a.d;
    const int beg = a.row_start[i];
    const int end = live ? beg + a.row_len[i] : beg;
    const float ei = a.eps_fixed;
    const float* xi = X + size_t(i) * d;
    f32x4 xv[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) xv[q] = load4_raw<true>(xi, 4 * lane + 4 * kWave * q, d);
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    float pi[NC];
#pragma unroll
    for (int q = 0; q < NC; q += 2) {
        const f32x2 v = *reinterpret_cast<const f32x2*>(a.P + size_t(i) * NC + q);
        pi[q] = v.x, pi[q + 1] = v.y;
    }
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.Wadj), 0, a.n * NC * 4, 0x00020000);
    // edge e's neighbour, weight and P row (forward data: plain loads)
    auto edge_pre = [&](int e, int& cj, float& we, float* pj) {
        const bool el = e < end;
        cj = el ? a.col[e] : i;
        we = el ? a.w[e] : 0.f;
#pragma unroll
        for (int q = 0; q < NC; q += 2) {
            const f32x2 v = *reinterpret_cast<const f32x2*>(a.P + size_t(cj) * NC + q);
            pj[q] = v.x, pj[q + 1] = v.y;
        }
    };
    // its coefficient once w is complete (edge_gv_r's order)
    float wi[NC];
    auto edge_coef = [&](int e, int cj, float we, const float* pj) -> float {
        float wj[NC];
#pragma unroll
        for (int q = 0; q < NC; ++q)
            wj[q] = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(rw, (cj * NC + q) * 4, 0, kSc1W));
        float g = 0.f;
#pragma unroll
        for (int q = 0; q < NC; ++q) g = __builtin_fmaf(wi[q] - wj[q], pj[q] - pi[q], g);
        const float ej = a.eps_fixed;
        const float v = -8.f * we / (ei * ej);   // GLL.py:217/234
        return e < end ? g * v : 0.f;
    };
    int cj;
    float we, pj[NC];
    edge_pre(beg + lane, cj, we, pj);
    const int cnt0 = min(kWave, end - beg);
#ifdef GLL_TRACE
    const bool tr = int(blockIdx.x) == C && threadIdx.x == 0;   // the first gradient block
    if (tr) g_trace[16] = __builtin_amdgcn_s_memrealtime();
#endif
    f32x4 v[EB][ND];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
        const int t = u < cnt0 ? u : 0;
        const float* xj = X + size_t(readlane_i(cj, t)) * d;
#pragma unroll
        for (int q = 0; q < ND; ++q) v[u][q] = load4_raw<true>(xj, 4 * lane + 4 * kWave * q, d);
    }
    // ---- wait for the C column solves (bounded: a lost solve surfaces as NaN + status)
    if (threadIdx.x == 0) {
        // a workspace whose previous fused backward lost a solve stays poisoned (its counter may
        // be stale) until the next forward rebuilds it: NaN again, never a stale hand-off
        int ok = __hip_atomic_load(fsync + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
        unsigned spins = 0;
        const unsigned long long t0 = wall_ticks();
        // the release word (fsync[96]) sits on a line no arrival adds to, so the 125 pollers
        // may poll it closely (round 4 polled the counter line itself with ~1,000 cycles
        // between polls, so as not to queue the columns' adds behind the loads)
        while (ok && __hip_atomic_load(fsync + 96, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               0u) {
            __builtin_amdgcn_s_sleep(2);
            if ((++spins & 15u) == 0 && wall_ticks() - t0 > kWaitTicks) {   // 1 s of wall clock
                ok = 0;
                break;
            }
        }
        s_ok = ok;
    }
    __syncthreads();
    const bool ok = s_ok != 0;
#ifdef GLL_TRACE
    if (tr) g_trace[17] = __builtin_amdgcn_s_memrealtime();
    GLL_FZ(0, i0, __builtin_amdgcn_s_memrealtime());
#endif
#pragma unroll
    for (int q = 0; q < NC; ++q)
        wi[q] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rw, (i * NC + q) * 4, 0, kSc1W));
    f32x4 acc[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int e0 = beg; e0 < end; e0 += kWave) {
        if (e0 != beg) edge_pre(e0 + lane, cj, we, pj);   // rows past 64 edges (hubs)
        const float cf = edge_coef(e0 + lane, cj, we, pj);
#ifdef GLL_TRACE
        if (e0 == beg) {
            float cfo = cf;
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(cfo)::"memory");
            if (cfo == 12345.f) g_trace[9] = 0;
            GLL_FZ(1, i0, __builtin_amdgcn_s_memrealtime());
        }
#endif
        const int cnt = min(kWave, end - e0);
        for (int t0 = 0; t0 < cnt; t0 += EB) {
            float sv[EB];
            if (e0 != beg || t0 != 0) {
#pragma unroll
                for (int u = 0; u < EB; ++u) {
                    const int t = t0 + u < cnt ? t0 + u : t0;
                    const float* xj = X + size_t(readlane_i(cj, t)) * d;
#pragma unroll
                    for (int q = 0; q < ND; ++q) v[u][q] = load4_raw<true>(xj, 4 * lane + 4 * kWave * q, d);
                }
            }
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                const int t = t0 + u < cnt ? t0 + u : t0;
                sv[u] = t0 + u < cnt ? readlane_f(cf, t) : 0.f;
            }
#pragma unroll
            for (int u = 0; u < EB; ++u) {
#pragma unroll
                for (int q = 0; q < ND; ++q) acc[q] += sv[u] * (xv[q] - v[u][q]);
            }
        }
    }
#ifdef GLL_TRACE
    {
        f32x4 ao = acc[0];
        asm volatile("" : "+v"(ao));
        if (ao.x == 12345.f) g_trace[9] = 0;
        GLL_FZ(2, i0, __builtin_amdgcn_s_memrealtime());
    }
#endif
    if (live) {
        const float nanf_ = __builtin_nanf("");
        float* oi = out + size_t(i) * d;
#pragma unroll
        for (int q = 0; q < ND; ++q) {
            const int k = 4 * lane + 4 * kWave * q;
            const f32x4 r = ok ? acc[q] : f32x4{nanf_, nanf_, nanf_, nanf_};
            if (k < d) __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(oi + k));
        }
    }
#ifdef GLL_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    GLL_FZ(3, i0, __builtin_amdgcn_s_memrealtime());
    {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        GLL_FZ(4, i0, (unsigned long long)(end - beg) | ((unsigned long long)((hw >> 8) & 0xffff) << 16) |
                          ((unsigned long long)(xcc & 0xff) << 40));
    }
#endif
    __syncthreads();
#ifdef GLL_TRACE
    if (tr) g_trace[18] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) atomicMax(&g_trace[19], __builtin_amdgcn_s_memrealtime());
#endif
    if (threadIdx.x == 0) {
        // the last gradient workgroup re-arms the counters for a second backward over the same
        // workspace (retain_graph) -- unless some workgroup gave up on the solves: then CG
        // workgroups may still add to fsync[0] after a reset, so the workspace is poisoned
        // instead (fsync[64], cleared by the next forward's row build)
        // Relaxed agent-scope atomics throughout (all performed at the coherence point, §3.5):
        // an acquire-release count made every one of the 125 gradient workgroups write back and
        // invalidate its XCD's L2 (buffer_wbl2 / buffer_inv) on its way out.  The poison is
        // performed before this workgroup's count (the vmcnt wait on the returning atomic), so
        // the last workgroup, whose count follows every other, reads it.
        if (!ok) {
            __hip_atomic_fetch_or(fsync + 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st_failed) atomicOr(st_failed, 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const unsigned ng = gridDim.x - unsigned(C);
        const unsigned old = __hip_atomic_fetch_add(fsync + 32, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1u == ng &&
            __hip_atomic_load(fsync + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
            __hip_atomic_store(fsync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(fsync + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(fsync + 96, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int NT, int ND, typename TB>
static hipError_t run_fused(const Layout& L, void* ws, const TB* b, const float* X,
                            float eps_fixed, float* gradX, float rtol, int max_iter,
                            int32_t* st_nonconv, int32_t* st_iters, int32_t* st_failed,
                            hipStream_t s) {
    constexpr int S = 24;
    size_t lds = 128 * 4 + size_t((L.m + 3) & ~3) * 4 * 2;   // MODE 3: P and y
    const int64_t eu_bound = int64_t(L.m + L.n) * (L.K - 1);
    int64_t cap = int64_t(kLdsDyn - lds) / 8;
    if (cap > eu_bound) cap = eu_bound;
    if (cap < 0) cap = 0;
    lds += size_t(cap) * 8;
    // the gradient workgroups' counting sort of the rows (class order): 2 n ints + the chunk table
    const size_t sort_lds = size_t(L.n) * 8 + size_t((L.n + kWave - 1) / kWave) * 10 * 4;
    if (sort_lds > kLdsDyn) return hipErrorNotSupported;
    if (lds < sort_lds) lds = sort_lds;
    auto fn = cg_grad_fused_kernel<NT, S, TB, ND>;
    allow_full_lds(reinterpret_cast<const void*>(fn));
    const int G = L.C + (L.n + NT / kWave - 1) / (NT / kWave);
    // (cached per kernel and device: a HIP query per call is host time on the step's path)
    const int nb = occupancy_blocks(reinterpret_cast<const void*>(fn), NT, lds);
    if (int64_t(nb) * device_cus() < G) return hipErrorNotSupported;   // not co-resident: two launches
    EllCgArgs c;
    c.m = L.m;
    c.C = L.C;
    c.base = L.base;
    c.row_start = L.at<int32_t>(ws, L.row_start);
    c.row_len = L.at<int32_t>(ws, L.row_len);
    c.ucnt = L.at<int32_t>(ws, L.ucnt);
    c.col = L.at<int32_t>(ws, L.col);
    c.wv = L.at<float>(ws, L.w);
    c.diag = L.at<float>(ws, L.diag);
    c.b = b;
    c.out32 = L.at<float>(ws, L.Wadj) + size_t(L.base) * L.C;
    c.rtol = rtol;
    c.max_iter = max_iter;
    c.mat_cap = int(cap);
    c.st_nonconv = st_nonconv;
    c.st_iters = st_iters;
    c.ell = L.at<int4>(ws, L.ell);
    const EdgeArgs a = make_edge_args(L, 0, ws, eps_fixed);
    prof_begin(GLL_K_BWD, s);
    launch_k(fn, dim3(unsigned(G)), NT, lds, s, c, a, X, gradX, L.at<unsigned>(ws, L.fsync),
             st_failed);
    prof_end(GLL_K_BWD, s);
    return launch_status("solve.hip:run_fused");
}

hipError_t launch_cg_grad_fused(const Layout& L, void* ws, const void* gbar, int g_dtype,
                                const float* X, float eps_fixed, float* gradX, float rtol,
                                int max_iter, int32_t* st_nonconv, int32_t* st_iters,
                                int32_t* st_failed, bool vec, hipStream_t s) {
    const int m = L.m;
    if (L.C != 10 || !(eps_fixed > 0.f) || !vec || m < 1 || m > 512 || L.RV != 0 ||
        ell_emit(L, 1) != 24 || L.d > 1024)
        return hipErrorNotSupported;
    if (L.flags & (GLL_FLAG_BWD_UNFUSED | GLL_FLAG_CG_GRID | GLL_FLAG_GRAD_CHUNK))
        return hipErrorNotSupported;
    if (size_t(L.n) * L.d * 4 > (size_t(4) << 20)) return hipErrorNotSupported;   // chunked
    const int nd = (L.d + 255) / 256;
#define GLL_FUSED(NT_)                                                                       \
    {                                                                                        \
        if (g_dtype == GLL_DT_F32) {                                                         \
            const float* b = static_cast<const float*>(gbar);                                \
            if (nd <= 1) return run_fused<NT_, 1>(L, ws, b, X, eps_fixed, gradX, rtol, max_iter, st_nonconv, st_iters, st_failed, s); \
            if (nd <= 2) return run_fused<NT_, 2>(L, ws, b, X, eps_fixed, gradX, rtol, max_iter, st_nonconv, st_iters, st_failed, s); \
            return run_fused<NT_, 4>(L, ws, b, X, eps_fixed, gradX, rtol, max_iter, st_nonconv, st_iters, st_failed, s); \
        }                                                                                    \
        const double* b = static_cast<const double*>(gbar);                                  \
        if (nd <= 1) return run_fused<NT_, 1>(L, ws, b, X, eps_fixed, gradX, rtol, max_iter, st_nonconv, st_iters, st_failed, s); \
        if (nd <= 2) return run_fused<NT_, 2>(L, ws, b, X, eps_fixed, gradX, rtol, max_iter, st_nonconv, st_iters, st_failed, s); \
        return run_fused<NT_, 4>(L, ws, b, X, eps_fixed, gradX, rtol, max_iter, st_nonconv, st_iters, st_failed, s); \
    }
    if (m <= 64) GLL_FUSED(64);
    if (m <= 128) GLL_FUSED(128);
    if (m <= 256) GLL_FUSED(256);
    GLL_FUSED(512);
#undef GLL_FUSED
}

template <int NT, int R, int RV, typename TB>
static hipError_t run_vr(const Layout& L, const Batch& bt, void* ws, const TB* b, size_t bs,
                         double* out64, float* out32, float rtol, int max_iter,
                         int32_t* st_nonconv, int32_t* st_iters, hipStream_t s) {
    if (L.m > NT * R || L.RV != RV || L.VRM <= 0 || L.VRM > 63) {   // row_build's packing
        (void)hipGetLastError();
        return hipErrorInvalidValue;
    }
    const size_t mp4 = size_t((L.m + 3) & ~3);
    const size_t lds = 128 * 4 + mp4 * 4 + (size_t(NT) * RV + 4 * mp4) * 4 +
                       size_t(NT) * RV * 4 + mp4 * 4;
    auto fn = cg_vr_kernel<NT, R, RV, TB>;
    allow_full_lds(reinterpret_cast<const void*>(fn));
    launch_k(fn, dim3(L.C, bt.B), NT, lds, s,
        L.m, L.C, L.base, L.VRM, L.at<int32_t>(ws, L.row_start), L.at<int32_t>(ws, L.row_len),
        L.at<int32_t>(ws, L.ucnt), L.at<int32_t>(ws, L.col), L.at<float>(ws, L.w),
        L.at<float>(ws, L.diag), L.at<char>(ws, L.vr), b, out64, out32, rtol, max_iter,
        st_nonconv, st_iters, bt.ws, bs, bt.u, bt.st);
    return launch_status("solve.hip:run_vr");
}

template <typename TB>
static hipError_t cg_dispatch(const Layout& L, const Batch& bt, void* ws, const TB* b, size_t bs,
                              double* out64, float* out32, float rtol, int max_iter,
                              int32_t* st_nonconv, int32_t* st_iters, int32_t* st_failed,
                              hipStream_t s) {
    const int m = L.m;
    // one persistent launch over the whole GPU (gridcg.hip) for a single graph past the
    // per-column register kernels' sweet spot (m > 2048: 4 ELL slots); measured at stress
    // (m 4096, K 30): 209 us against 288 us per solve, while at the FullySup shape (m 1250,
    // K 25) the per-column kernel with 16 slots and the LDS overflow wins.  Batches keep the
    // per-column kernels (B x C workgroups already fill the GPU).
    if (grid_cg_route(L, bt)) {
        const int b_dtype = sizeof(TB) == 8 ? GLL_DT_F64 : GLL_DT_F32;
        const hipError_t e = launch_cg_grid_luu(L, ws, b, b_dtype, out64, out32, rtol, 0.f,
                                                max_iter, st_nonconv, st_iters, st_failed, s);
        if (e != hipErrorNotSupported) return e;
        // no grid configuration holds it: per-column kernels below (any m)
    }
    // the Neumann form (MODE 3) wherever a thread owns one row; with two or more rows per thread
    // one SpMV per iteration (MODE 3 at 256 x 2 takes 220 VGPRs, two waves per SIMD instead of
    // three: B = 64 NS CG 21.8 -> 34.2 us, profiles/r03l_cg_neumann_ab.txt; at 1024 x 2 it
    // spilled 144 B per lane: FullySup single graph forced onto this kernel 174 -> 135 us per
    // solve with MODE 1, profiles/r04p_ab_ell2.txt).
#define GLL_ELL(NT, R, S)                                                                   \
    return (R > 1)                                                                          \
               ? run_ell<NT, R, S, TB, 1>(L, bt, ws, b, bs, out64, out32, rtol, max_iter,   \
                                          st_nonconv, st_iters, s)                          \
               : run_ell<NT, R, S, TB, 3>(L, bt, ws, b, bs, out64, out32, rtol, max_iter,   \
                                          st_nonconv, st_iters, s)
    if (L.RV > 0) {   // the balanced kernel (row_build packed its virtual rows)
#define GLL_VR(T_, R_, V_) \
        if (L.RV == V_) return run_vr<T_, R_, V_, TB>(L, bt, ws, b, bs, out64, out32, rtol,   \
                                                      max_iter, st_nonconv, st_iters, s)
        if (m <= 512) { GLL_VR(512, 1, 4); GLL_VR(512, 1, 8); GLL_VR(512, 1, 10); }
        if (m <= 1024) { GLL_VR(512, 2, 4); GLL_VR(512, 2, 8); GLL_VR(512, 2, 10); }
        if (m <= 1536) { GLL_VR(512, 3, 4); GLL_VR(512, 3, 8); GLL_VR(512, 3, 10); }
        GLL_VR(512, 4, 4); GLL_VR(512, 4, 8); GLL_VR(512, 4, 10);
#undef GLL_VR
        return hipErrorInvalidValue;
    }
    if (m <= 64) GLL_ELL(64, 1, 24);
    if (m <= 128) GLL_ELL(128, 1, 24);
    if (m <= 256) GLL_ELL(256, 1, 24);
    // m <= 512: one row per thread is the lower latency for a single graph; batches run more
    // workgroups per CU with 4 waves x 2 rows (B = 64: 44.7 -> 36.6 us per launch).  Batches of
    // at most one column workgroup per CU (B x C <= 256) run the single-graph geometry, 512 x 1
    // with the Neumann form: NS B = 8 18.6 -> 15.9 us per launch; with more workgroups than CUs
    // 256 x 2 (MODE 1) keeps the lead: B = 64 21.9 against 28.2 us
    // (profiles/r03t_cg_batched_geometry_ab.txt).  Round 4 swept nine batched geometries (128 /
    // 256 / 512 threads x 4 / 2 / 1 rows, 8-24 register ELL slots, MODE 1 and 3) at B = 64:
    // none beat 256 x 2 x 24 MODE 1 (21.9 us; the best Neumann form 28.2 us,
    // profiles/r04c_ab_geom.txt), and the variants were removed.  (Column pairs -- two right-hand sides per
    // workgroup -- measured slower at B = 64 and 8 and were removed in round 4:
    // profiles/r03s_cg_pairs_ab.txt.)
    if (m <= 512 && (bt.B == 1 || int64_t(bt.B) * L.C <= 256)) GLL_ELL(512, 1, 24);
    if (m <= 512) GLL_ELL(256, 2, 24);
    if (m <= 1024) GLL_ELL(1024, 1, 16);
    if (m <= 2048) GLL_ELL(1024, 2, 16);
    if (m <= 4096) GLL_ELL(1024, 4, 4);
#undef GLL_ELL
    const size_t vec_bytes = size_t(5) * m * sizeof(float);
    const bool vec_lds = 64 * 4 + vec_bytes <= kLdsDyn;
    const size_t lds = 64 * 4 + (vec_lds ? vec_bytes : 0);
    auto fn = cg_lds_kernel<1024, TB>;
    allow_full_lds(reinterpret_cast<const void*>(fn));
    launch_k(fn, dim3(L.C, bt.B), 1024, lds, s,
        m, L.C, L.base, L.at<int32_t>(ws, L.row_start), L.at<int32_t>(ws, L.row_len),
        L.at<int32_t>(ws, L.ucnt), L.at<int32_t>(ws, L.col), L.at<float>(ws, L.w),
        L.at<float>(ws, L.diag), b, out64, out32, rtol, max_iter, L.at<float>(ws, L.cgv),
        vec_lds ? 1 : 0, st_nonconv, st_iters, bt.ws, bs, bt.u, bt.st);
    return launch_status("solve.hip:cg_dispatch");
}

hipError_t launch_cg_luu(const Layout& L, const Batch& bt, void* ws, const void* b,
                         size_t b_stride, int b_dtype, double* out64, float* out32, float rtol,
                         int max_iter, int32_t* st_nonconv, int32_t* st_iters,
                         int32_t* st_failed, hipStream_t s) {
    if (L.m <= 0) return hipSuccess;
    hipError_t e;
    prof_begin(GLL_K_CG, s);
    if (b_dtype == GLL_DT_F32)
        e = cg_dispatch(L, bt, ws, static_cast<const float*>(b), b_stride, out64, out32, rtol,
                        max_iter, st_nonconv, st_iters, st_failed, s);
    else if (b_dtype == GLL_DT_F64)
        e = cg_dispatch(L, bt, ws, static_cast<const double*>(b), b_stride, out64, out32, rtol,
                        max_iter, st_nonconv, st_iters, st_failed, s);
    else
        return hipErrorInvalidValue;
    prof_end(GLL_K_CG, s);
    return e;
}

// --------------------------------------------------------------------------------------
// General SPD CSR (stable_conjgrad replacement, absolute tolerance like GLL.py:259)
// --------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void cg_csr_kernel(int m, int C, const int32_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col,
                                                    const float* __restrict__ val,
                                                    const float* __restrict__ b,
                                                    float* __restrict__ x, float atol,
                                                    int max_iter, float* __restrict__ gvec,
                                                    int vec_in_lds, int32_t* __restrict__ iters,
                                                    int32_t* __restrict__ nonconv) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int c = bx<true>();
    const int tid = threadIdx.x;
    float* red = smem;
    float* vb = vec_in_lds ? smem + 64 : gvec + size_t(c) * 5 * m;
    float *X_ = vb, *R_ = vb + m, *P_ = vb + 2 * m, *A_ = vb + 3 * m, *M_ = vb + 4 * m;
    float rz = 0.f, rr0 = 0.f;
    for (int u = tid; u < m; u += NT) {
        float dg = 0.f;
        for (int e = rp[u]; e < rp[u + 1]; ++e)
            if (col[e] == u) dg += val[e];
        const float mi = dg > 0.f ? 1.f / dg : 0.f;
        const float bu = b[size_t(u) * C + c];
        X_[u] = 0.f;
        R_[u] = bu;
        M_[u] = mi;
        P_[u] = mi * bu;
        rz += bu * mi * bu;
        rr0 += bu * bu;
    }
    int phase = 0;
    __syncthreads();
    block_sum2<NT>(rz, rr0, red, phase);
    const float tol2 = atol * atol;
    int it = 0;
    bool conv = rr0 <= tol2;
    while (!conv && it < max_iter) {
        ++it;
        float pap = 0.f, unused = 0.f;
        for (int u = tid; u < m; u += NT) {
            float acc = 0.f;
            for (int e = rp[u]; e < rp[u + 1]; ++e) acc += val[e] * P_[col[e]];
            A_[u] = acc;
            pap += P_[u] * acc;
        }
        block_sum2<NT>(pap, unused, red, phase);
        if (!(pap > 0.f)) break;
        const float alpha = rz / pap;
        float rr = 0.f, rzn = 0.f;
        for (int u = tid; u < m; u += NT) {
            X_[u] += alpha * P_[u];
            const float ru = R_[u] - alpha * A_[u];
            R_[u] = ru;
            rr += ru * ru;
            rzn += ru * M_[u] * ru;
        }
        block_sum2<NT>(rr, rzn, red, phase);
        if (rr <= tol2) {
            conv = true;
            break;
        }
        const float beta = rzn / rz;
        rz = rzn;
        for (int u = tid; u < m; u += NT) P_[u] = M_[u] * R_[u] + beta * P_[u];
        __syncthreads();
    }
    for (int u = tid; u < m; u += NT) x[size_t(u) * C + c] = X_[u];
    if (tid == 0) {
        if (iters) atomicMax(iters, it);
        if (!conv && nonconv) atomicAdd(nonconv, 1);
    }
}

hipError_t launch_cg_csr(int m, int C, const int32_t* row_ptr, const int32_t* col,
                         const float* val, const float* b, float* x, float atol, int max_iter,
                         int32_t* iters, int32_t* nonconv, float* gvec, hipStream_t s) {
    const size_t vec_bytes = size_t(5) * m * sizeof(float);
    const bool vec_lds = 64 * 4 + vec_bytes <= kLdsDyn;
    if (!vec_lds && gvec == nullptr) return hipErrorInvalidValue;
    const size_t lds = 64 * 4 + (vec_lds ? vec_bytes : 0);
    auto fn = cg_csr_kernel<256>;
    allow_full_lds(reinterpret_cast<const void*>(fn));
    prof_begin(GLL_K_CG, s);
    launch_k(fn, C, 256, lds, s, m, C, row_ptr, col, val, b, x, atol, max_iter, gvec, vec_lds ? 1 : 0,
                           iters, nonconv);
    prof_end(GLL_K_CG, s);
    return launch_status("solve.hip:launch_cg_csr");
}

}  // namespace gll
