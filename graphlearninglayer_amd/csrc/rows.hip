// rows.hip -- symmetric kNN graph rows + weights, degree and Laplace right-hand side.
//
// Replaces the scipy COO/CSR work of knn_sym_dist (/root/reference/GLL.py:192-238:
// coo->csr, symmetric max, sparse.find, W values) and csgraph.laplacian + the Luu/Lul
// split (GLL.py:29,37-38,48).  One wave per graph row i (K3 row_build_kernel):
//   * forward entries: i's own kNN list (valid = d > 0; sparse.find drops zeros, GLL.py:198);
//   * reverse entries: every l that listed i (pushed by knn_select_kernel onto i's reverse
//     list, spilling to the overflow list past RCAP); a reverse entry already in i's own list
//     (a mutual pair) keeps max(d_ij, d_ji): the union-max of GLL.py:197.  (The two
//     distances agree bitwise unless one row refined its ranking in float64, knn.hip);
//   * the row is staged in LDS (global scratch for hub rows), rank-sorted by column --
//     deterministic whatever order the atomics produced -- and written to its slot
//     (row_start, row_len; hub rows take a bump-allocated range);
//   * W_ij = exp(-4 d_ij^2 / (eps_i eps_j)) (GLL.py:216/233), degree, and for unlabeled rows
//     the Luu diagonal deg + tau, the U-block length, and rhs = W_ul Y (= -Lul Y, GLL.py:53);
//     labeled rows write P = Y and w = 0 for the backward (GLL.py:104,109).
#include "gll_internal.h"

namespace gll {

GLL_TRACE_UNIT(rows)

// Row checkpoints (trace builds): slots 1.. for row `base` (the first unlabeled row), 11.. for a
// hub row (reverse list past RCAP; the last one to get there), 20 / 21 the longest wave among
// every 16th row / among the hub rows (s_memrealtime ticks, atomicMax).
#ifdef GLL_TRACE
#define GLL_ROW_PT(q)                                                                         \
    do {                                                                                     \
        if (lane_id() == 0 && tslot >= 0) g_trace[tslot + (q)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define GLL_ROW_PT(q) do {} while (0)
#endif

constexpr int kStage = 256;      // per-wave LDS staging capacity (entries)
constexpr int kMaxCPerLane = 4;  // classes per lane in the rhs accumulation (C <= 256)
constexpr int kYPre = 16;        // label prefetch: classes held per staged entry (C <= 16)

struct RowArgs {
    int n, base, C, K, RCAP, Wcap;
    int64_t bump_base;
    float tau;
    float eps_fixed;   // > 0: fixed epsilon, no eps gathers
    const int32_t* knn_idx;
    const float* knn_d2;
    const int32_t* rev_cnt;
    const int32_t* rev_idx;
    const float* rev_d2;
    const int32_t* ovf;
    int32_t* status;
    const float* eps;
    int32_t* tmp_col;
    float* tmp_d2;
    int32_t* row_start;
    int32_t* row_len;
    int32_t* col;
    float* w;
    float* d2e;
    float* deg;
    int32_t* ucnt;
    float* diag;
    float* rhs;
    float* P;
    float* Wadj;
    int32_t* ell;       // [SE/2][m] x (col, w, col, w): column-major U slices for the CG
    int SE, m;
    char* vr;           // [m][VRM] packed virtual rows of the balanced CG (VRM = 0: none)
    int VRM;
    unsigned* fsync;    // fused backward counters (solve.hip cg_grad_fused_kernel): zeroed here
    unsigned* gsync;    // whole-GPU CG sync words (gridcg.hip), zeroed here; null: not used
    size_t wss;   // batched launches: workspace stride between graphs (bytes)

    template <bool FLAT>
    __device__ void to_graph(int g) {   // move every workspace pointer to graph g
        knn_idx = FLAT ? gshift_flat_at(knn_idx, wss, g) : gshift_at(knn_idx, wss, g);
        knn_d2 = FLAT ? gshift_flat_at(knn_d2, wss, g) : gshift_at(knn_d2, wss, g);
        rev_cnt = FLAT ? gshift_flat_at(rev_cnt, wss, g) : gshift_at(rev_cnt, wss, g);
        rev_idx = FLAT ? gshift_flat_at(rev_idx, wss, g) : gshift_at(rev_idx, wss, g);
        rev_d2 = FLAT ? gshift_flat_at(rev_d2, wss, g) : gshift_at(rev_d2, wss, g);
        ovf = FLAT ? gshift_flat_at(ovf, wss, g) : gshift_at(ovf, wss, g);
        status = FLAT ? gshift_flat_at(status, wss, g) : gshift_at(status, wss, g);
        eps = FLAT ? gshift_flat_at(eps, wss, g) : gshift_at(eps, wss, g);
        tmp_col = FLAT ? gshift_flat_at(tmp_col, wss, g) : gshift_at(tmp_col, wss, g);
        tmp_d2 = FLAT ? gshift_flat_at(tmp_d2, wss, g) : gshift_at(tmp_d2, wss, g);
        row_start = FLAT ? gshift_flat_at(row_start, wss, g) : gshift_at(row_start, wss, g);
        row_len = FLAT ? gshift_flat_at(row_len, wss, g) : gshift_at(row_len, wss, g);
        col = FLAT ? gshift_flat_at(col, wss, g) : gshift_at(col, wss, g);
        w = FLAT ? gshift_flat_at(w, wss, g) : gshift_at(w, wss, g);
        d2e = FLAT ? gshift_flat_at(d2e, wss, g) : gshift_at(d2e, wss, g);
        deg = FLAT ? gshift_flat_at(deg, wss, g) : gshift_at(deg, wss, g);
        ucnt = FLAT ? gshift_flat_at(ucnt, wss, g) : gshift_at(ucnt, wss, g);
        diag = FLAT ? gshift_flat_at(diag, wss, g) : gshift_at(diag, wss, g);
        rhs = FLAT ? gshift_flat_at(rhs, wss, g) : gshift_at(rhs, wss, g);
        P = FLAT ? gshift_flat_at(P, wss, g) : gshift_at(P, wss, g);
        Wadj = FLAT ? gshift_flat_at(Wadj, wss, g) : gshift_at(Wadj, wss, g);
        ell = FLAT ? gshift_flat_at(ell, wss, g) : gshift_at(ell, wss, g);
        vr = FLAT ? gshift_flat_at(vr, wss, g) : gshift_at(vr, wss, g);
        fsync = FLAT ? gshift_flat_at(fsync, wss, g) : gshift_at(fsync, wss, g);
    }
};

template <typename TY>
__device__ __forceinline__ float yval(const TY* Y, int j, int C, int c) {
    return to_f32(Y[size_t(j) * C + c]);
}

// Build row i.  LDS: staging and sorted copies live in the wave's LDS slices; otherwise the
// staging is tmp_col/tmp_d2 and the sorted copy is the output itself (agent fences order them).
// pri / prd: this lane's slot of the first 64 reverse entries, loaded with the kNN list (one
// memory round trip for both).  Rows staged in LDS with C <= kYPre also issue the label loads
// of their first 64 staged entries right after staging, so the loads overlap the sort and the
// weights; the sums still run in sorted-column order (t_idx maps a sorted slot to its staged
// entry), so results are unchanged.
// FH: 64-entry parts of the forward list (K - 1 <= 64 FH): entry 64 h + lane of row i's kNN list
// sits in lane `lane` of fi[h]; its valid entries are staged part after part.
template <bool LDS, bool PRE, typename TY, int FH>
__device__ __forceinline__ void build_row(const RowArgs& a, const TY* __restrict__ Y, int i,
                                          int start, const int (&fi)[FH], const float (&fd)[FH],
                                          const bool (&fval)[FH], const uint64_t (&fmask)[FH],
                                          int nf, int rc, float ei, int pri,
                                          float prd, int* s_col, float* s_d2, int* t_col,
                                          float* t_d2, float* t_w, int* t_idx, float* ybuf,
                                          int tslot) {
    const int lane = lane_id();
    (void)tslot;
    int* scol = LDS ? s_col : a.tmp_col + start;
    float* sd2 = LDS ? s_d2 : a.tmp_d2 + start;
    int* ocol = LDS ? t_col : a.col + start;
    float* od2 = LDS ? t_d2 : a.d2e + start;
    float* ow = LDS ? t_w : a.w + start;
    const int Km1 = a.K - 1;
    int fself[FH];
    int fbase[FH];   // staged position of each half's first valid entry
    // forward entries
#pragma unroll
    for (int h = 0; h < FH; ++h) {
        fself[h] = fval[h] ? fi[h] : -2;
        fbase[h] = h == 0 ? 0 : fbase[h - 1] + __popcll(fmask[h - 1]);
        if (fval[h]) {
            const int p = fbase[h] + lanes_below(fmask[h]);
            scol[p] = fi[h];
            sd2[p] = fd[h];
        }
    }
    // the staged position of forward entry t (a valid one): its half's base + valid entries
    // before it in that half
    auto fpos = [&](int t) {
        int p = 0;
#pragma unroll
        for (int h = 0; h < FH; ++h)
            if ((t >> 6) == h) p = fbase[h] + __popcll(fmask[h] & ((1ull << (t & 63)) - 1ull));
        return p;
    };
    // the staged position of the forward entry equal to column ri, or -1.  LDS rows scan the
    // staged forward list [0, nf) with 16-B broadcast reads (no cross-lane chain); global-
    // staged rows compare against the lanes' list registers
    auto fmatch_pos = [&](int ri) {
        if constexpr (LDS) {
            int p = -1;
            const int nf4 = nf & ~3;
#pragma unroll 2
            for (int u = 0; u < nf4; u += 4) {
                const int4 v = *reinterpret_cast<const int4*>(scol + u);
                p = v.x == ri ? u : p;
                p = v.y == ri ? u + 1 : p;
                p = v.z == ri ? u + 2 : p;
                p = v.w == ri ? u + 3 : p;
            }
#pragma unroll 1
            for (int u = nf4; u < nf; ++u) p = scol[u] == ri ? u : p;
            return p;
        } else {
            return -1;   // not used
        }
    };
    auto fmatch = [&](int ri) {   // the forward entry equal to column ri, or -1
        int tpos = -1;
#pragma unroll
        for (int h = 0; h < FH; ++h) {
            const int tn = min(Km1 - 64 * h, kWave);
            for (int t = 0; t < tn; ++t) tpos = (ri == readlane_i(fself[h], t)) ? 64 * h + t : tpos;
        }
        return tpos;
    };
    int L = nf;
    // reverse entries, deduplicated against the forward list (mutual pairs)
    const int nr = min(rc, a.RCAP);
    for (int r0 = 0; r0 < nr; r0 += kWave) {
        const int r = r0 + lane;
        const bool live = r < nr;
        const int ri = !live ? -1 : (r0 == 0 ? pri : a.rev_idx[size_t(i) * a.RCAP + r]);
        const float rd = !live ? 0.f : (r0 == 0 ? prd : a.rev_d2[size_t(i) * a.RCAP + r]);
        const int tpos = LDS ? fmatch_pos(ri) : fmatch(ri);
        const bool keep = live && tpos < 0;
        const uint64_t mk = __ballot(keep);
        if (keep) {
            const int p = L + lanes_below(mk);
            scol[p] = ri;
            sd2[p] = rd;
        }
        if (live && tpos >= 0) {   // mutual pair: union-max (non-negative float bits order)
            if constexpr (!LDS) __threadfence();
            atomicMax(reinterpret_cast<unsigned*>(sd2) + (LDS ? tpos : fpos(tpos)),
                      __float_as_uint(rd));
        }
        L += __popcll(mk);
    }
    GLL_ROW_PT(9);
    if (rc > a.RCAP) {  // hub row: the remaining reverse entries sit in the overflow list
        const int novf = __hip_atomic_load(&a.status[kStOvfCount], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        GLL_ROW_PT(8);
#ifdef GLL_TRACE
        if (tslot == 10 && lane == 0) g_trace[22] = novf;
#endif
        // the whole list is scanned by every hub row: OB chunks of 64 triples are loaded
        // before any is matched (one memory round trip per 512 entries, not per 64: a stress
        // hub row spent 22 of its 43 us here, profiles/r05t_trace_stress.txt); entries are
        // still taken in list order
        constexpr int OB = 8;
        for (int q0 = 0; q0 < novf; q0 += OB * kWave) {
            int ojs[OB], ois[OB];
            float ods[OB];
#pragma unroll
            for (int b = 0; b < OB; ++b) {
                const int q = q0 + b * kWave + lane;
                const bool live = q < novf;
                ojs[b] = live ? a.ovf[3 * q] : -1;
                ois[b] = live ? a.ovf[3 * q + 1] : -1;
                ods[b] = live ? __int_as_float(a.ovf[3 * q + 2]) : 0.f;
            }
#pragma unroll
            for (int b = 0; b < OB; ++b) {
                if (q0 + b * kWave >= novf) break;   // wave-uniform
                const int oj = ojs[b], oi = ois[b];
                const float od = ods[b];
                const bool mine_e = oj == i;   // dead slots hold -1
                const int tpos = __ballot(mine_e) ? (LDS ? fmatch_pos(oi) : fmatch(oi)) : -1;
                const bool keep = mine_e && tpos < 0;
                const uint64_t mk = __ballot(keep);
                if (keep) {
                    const int p = L + lanes_below(mk);
                    scol[p] = oi;
                    sd2[p] = od;
                }
                if (mine_e && tpos >= 0) {   // mutual pair: union-max
                    if constexpr (!LDS) __threadfence();
                    atomicMax(reinterpret_cast<unsigned*>(sd2) + (LDS ? tpos : fpos(tpos)),
                              __float_as_uint(od));
                }
                L += __popcll(mk);
            }
#ifdef GLL_TRACE
            if (tslot == 10 && lane == 0 && q0 == 0) g_trace[23] = __builtin_amdgcn_s_memrealtime();
#endif
        }
    }
    if constexpr (!LDS) __threadfence();
    GLL_ROW_PT(2);
    // label prefetch (unlabeled rows): lane e < 64 loads Y of staged entry e when labeled
    const bool ypre = LDS && PRE && i >= a.base && a.C <= kYPre;
    float yreg[kYPre];
    if (ypre) {
        const int col0 = lane < L ? scol[lane] : a.base;
        const bool lab = lane < L && col0 < a.base;
#pragma unroll
        for (int c = 0; c < kYPre; ++c) yreg[c] = (lab && c < a.C) ? yval(Y, col0, a.C, c) : 0.f;
    }
    // rank sort by column (columns are unique within a row).  LDS rows are read four columns
    // per 16-B broadcast load, past L padded with INT_MAX (never below a column): a quarter of
    // the LDS reads (a stress hub row of ~230 entries spent 5-9 us here)
    if constexpr (LDS) {
        const int L16 = (L + 15) & ~15;   // <= kStage, a multiple of 16
        if (L + lane < L16) scol[L + lane] = 0x7fffffff;
        __builtin_amdgcn_wave_barrier();   // a wave's LDS ops run in order
        asm volatile("" ::: "memory");
        for (int e = lane; e < L; e += kWave) {
            const int c = scol[e];
            int rank = 0;
            for (int u = 0; u < L16; u += 16) {   // four loads in flight per step
                int4 v[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const int4*>(scol + u + 4 * q);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    rank += (v[q].x < c ? 1 : 0) + (v[q].y < c ? 1 : 0) + (v[q].z < c ? 1 : 0) +
                            (v[q].w < c ? 1 : 0);
            }
            ocol[rank] = c;
            od2[rank] = sd2[e];
            if constexpr (PRE) t_idx[rank] = e;
        }
    } else {
        for (int e = lane; e < L; e += kWave) {
            const int c = scol[e];
            int rank = 0;
            for (int u = 0; u < L; ++u) rank += scol[u] < c ? 1 : 0;
            ocol[rank] = c;
            od2[rank] = sd2[e];
        }
    }
    if constexpr (!LDS) __threadfence();
    GLL_ROW_PT(3);
    // sorted pass: weights, degree, labeled-prefix length
    float dsum = 0.f;
    int nlab = 0;
    for (int e = lane; e < L; e += kWave) {
        const int c = ocol[e];
        const float dd = od2[e];
        const float ec = a.eps_fixed > 0.f ? a.eps_fixed : a.eps[c];
        const float we = expf(-4.f * dd / (ei * ec));   // GLL.py:216/233
        ow[e] = we;
        if constexpr (LDS) {
            a.col[start + e] = c;
            a.d2e[start + e] = dd;
            a.w[start + e] = we;
        }
        dsum += we;
        nlab += c < a.base ? 1 : 0;
    }
    if constexpr (!LDS) __threadfence();
    dsum = wave_sum_dpp(dsum);
    nlab = wave_sum_i(nlab);
    GLL_ROW_PT(4);
    // rhs_i = sum_{j < base} W_ij Y_j over the sorted labeled prefix, lanes over classes
    float racc[kMaxCPerLane];
#pragma unroll
    for (int q = 0; q < kMaxCPerLane; ++q) racc[q] = 0.f;
    if (i >= a.base && a.SE > 0) {   // column-major ELL slice of the U block for the CG
        const int u = i - a.base, nu = L - nlab;
        if (lane < a.SE) {
            const bool live = lane < nu;
            const int e = nlab + (live ? lane : 0);
            const int c = live ? ocol[e] - a.base : 0;
            const float we = live ? ow[e] : 0.f;
            int32_t* rec = a.ell + (size_t(lane >> 1) * a.m + u) * 4 + (lane & 1) * 2;
            rec[0] = c;
            rec[1] = __float_as_int(we);
        }
    }
    if (i >= a.base && a.VRM > 0) {
        // the U block as packed virtual rows of kVS entries for the balanced CG (solve.hip
        // cg_vr_kernel): 16-bit LDS byte offsets of the columns, then the weights, the last
        // one zero-padded; rows past VRM of them keep their tail in the CSR only
        const int u = i - a.base, nu = L - nlab;
        const int nv = min((nu + kVS - 1) / kVS, a.VRM);
        char* slots = a.vr + size_t(u) * a.VRM * kVrSlot;
        for (int q = lane; q < nv * kVS; q += kWave) {
            const bool live = q < nu;
            const int e = nlab + (live ? q : 0);
            const int cu = ocol[e] - a.base;
            const float we = ow[e];
            char* sl = slots + size_t(q / kVS) * kVrSlot;
            reinterpret_cast<uint16_t*>(sl)[q % kVS] = live ? uint16_t(cu * 4) : uint16_t(0);
            reinterpret_cast<float*>(sl + kVS * 2)[q % kVS] = live ? we : 0.f;
        }
    }
    GLL_ROW_PT(5);
    if (ypre) {
        // prefetched labels: staged entry e's row of Y at ybuf[e][.], summed in sorted order
        if (lane < L && lane < kWave) {
#pragma unroll
            for (int c = 0; c < kYPre; ++c) ybuf[lane * kYPre + c] = yreg[c];
        }
        __builtin_amdgcn_wave_barrier();   // a wave's LDS ops run in order
        asm volatile("" ::: "memory");
        if (L <= kWave) {   // every staged entry's labels were prefetched
            // 16 entries per step: their staged indices, then their labels and weights, all
            // read before the first product (one entry at a time was two dependent LDS round
            // trips per labeled neighbour); same summation order
            for (int e0 = 0; e0 < nlab; e0 += 16) {
                int ev[16];
#pragma unroll
                for (int t = 0; t < 16; ++t) ev[t] = t_idx[e0 + t < nlab ? e0 + t : e0];
                float yv[16], wv[16];
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    yv[t] = lane < a.C ? ybuf[ev[t] * kYPre + lane] : 0.f;
                    wv[t] = ow[e0 + t < nlab ? e0 + t : e0];
                }
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    if (e0 + t < nlab) racc[0] += wv[t] * yv[t];
            }
        } else {
            // rows of hub nodes (more than 64 staged entries): 32 labeled neighbours per step,
            // all of a step's label loads in flight before any is used (one at a time they
            // were 15 of a stress hub row's 43 us, profiles/r05t_trace_stress.txt); the same
            // values in the same order as the prefetched form
            constexpr int NB = 32;
            for (int e0 = 0; e0 < nlab; e0 += NB) {
                float yv[NB];
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const int es = e0 + t < nlab ? e0 + t : e0;
                    yv[t] = yval(Y, ocol[es], a.C, lane < a.C ? lane : 0);
                }
#pragma unroll
                for (int t = 0; t < NB; ++t)
                    if (e0 + t < nlab) racc[0] += ow[e0 + t] * (lane < a.C ? yv[t] : 0.f);
            }
        }
    } else if (i >= a.base) {
        // 8 labeled neighbours per step, their label loads all in flight before any is used
        for (int e0 = 0; e0 < nlab; e0 += 8) {
            float we[8], yv[8][kMaxCPerLane];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const bool live = e0 + t < nlab;
                const int j = ocol[live ? e0 + t : e0];
                we[t] = live ? ow[e0 + t] : 0.f;
#pragma unroll
                for (int q = 0; q < kMaxCPerLane; ++q) {
                    const int c = lane + q * kWave;
                    yv[t][q] = c < a.C ? yval(Y, j, a.C, c) : 0.f;
                }
            }
#pragma unroll
            for (int t = 0; t < 8; ++t)
#pragma unroll
                for (int q = 0; q < kMaxCPerLane; ++q) racc[q] += we[t] * yv[t][q];
        }
    }
#pragma unroll
    for (int q = 0; q < kMaxCPerLane; ++q) {
        const int c = lane + q * kWave;
        if (c < a.C) {
            if (i >= a.base) {
                a.rhs[size_t(i - a.base) * a.C + c] = racc[q];
            } else {
                a.P[size_t(i) * a.C + c] = yval(Y, i, a.C, c);
                a.Wadj[size_t(i) * a.C + c] = 0.f;
            }
        }
    }
    GLL_ROW_PT(6);
    if (lane == 0) {
        a.row_start[i] = start;
        a.row_len[i] = L;
        a.deg[i] = dsum;
        if (i >= a.base) {
            a.diag[i - a.base] = dsum + a.tau;   // Luu + tau I (GLL.py:48)
            a.ucnt[i - a.base] = L - nlab;       // the U block is the row's sorted suffix
        }
    }
}

// PRE: label prefetch (single-graph launches; its 20 KiB of LDS halves the workgroups per CU
// that batches need: B = 64 NS 72 -> 90 us with it)
template <typename TY, bool PRE, bool FLAT, bool R = false, int FH = 1>
__global__ __launch_bounds__(256) void row_build_kernel(RowArgs a, const TY* __restrict__ Y,
                                                        size_t ys) {
    GLL_TRACE_SCOPE(0);
    const int2 gxy = batch_xy<R>();   // once (per pointer it re-reads gridDim and divides)
    a.to_graph<FLAT>(gxy.y);
    Y = gshift_at(Y, ys, gxy.y);
    __shared__ __attribute__((aligned(16))) int s_col[4][kStage];
    __shared__ float s_d2[4][kStage];
    __shared__ int t_col[4][kStage];
    __shared__ float t_d2[4][kStage];
    __shared__ float t_w[4][kStage];
    __shared__ int t_idx[4][PRE ? kStage : 1];
    __shared__ float ybuf[4][PRE ? kWave * kYPre : 1];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    const int i = gxy.x * 4 + wv;
    if (i >= a.n) return;
#ifdef GLL_TRACE
    const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
#endif
    if (i == 0 && lane == 0) {   // the backward's hand-off counters start at zero
        a.fsync[0] = 0u;
        a.fsync[32] = 0u;
        a.fsync[64] = 0u;   // a poisoned workspace (lost solve) is rebuilt here
        a.fsync[96] = 0u;
    }
    if (i == 0 && a.gsync)   // single graphs only (grid_cg_route)
        for (int t = lane; t < kGridSyncWords; t += kWave) a.gsync[t] = 0u;
    const int Km1 = a.K - 1;
    int fi[FH];
    float fd[FH];
    bool fval[FH];
    uint64_t fmask[FH];
    int nf = 0;
#pragma unroll
    for (int h = 0; h < FH; ++h) {
        const int t = 64 * h + lane;
        fi[h] = -1;
        fd[h] = 0.f;
        if (t < Km1) {
            fi[h] = a.knn_idx[size_t(i) * a.K + 1 + t];
            fd[h] = a.knn_d2[size_t(i) * a.K + 1 + t];
        }
        fval[h] = t < Km1 && fd[h] > 0.f && fi[h] != i && fi[h] >= 0 && fi[h] < a.n;
        fmask[h] = __ballot(fval[h]);
        nf += __popcll(fmask[h]);
    }
    const int rc = a.rev_cnt[i];
    const float ei = a.eps_fixed > 0.f ? a.eps_fixed : a.eps[i];   // issued with the lists
    int pri = -1;   // the first 64 reverse-list slots, speculatively with the kNN list
    float prd = 0.f;
    if (lane < a.RCAP) {
        pri = a.rev_idx[size_t(i) * a.RCAP + lane];
        prd = a.rev_d2[size_t(i) * a.RCAP + lane];
    }
    const int lbound = nf + rc;
    int tslot = -1;
#ifdef GLL_TRACE
    if (gxy.y == 0) tslot = i == a.base ? 0 : (rc > a.RCAP ? 10 : -1);
    if (tslot >= 0 && lane == 0) g_trace[tslot] = t_entry;
    GLL_ROW_PT(1);
#endif
    int start = i * a.Wcap;
    if (lbound > a.Wcap) {
        int s0 = 0;
        if (lane == 0) s0 = int(a.bump_base) + atomicAdd(&a.status[kStBump], lbound);
        start = readlane_i(s0, 0);
    }
    if (lbound <= kStage)
        build_row<true, PRE, TY, FH>(a, Y, i, start, fi, fd, fval, fmask, nf, rc, ei, pri, prd,
                                     s_col[wv], s_d2[wv], t_col[wv], t_d2[wv], t_w[wv], t_idx[wv],
                                     ybuf[wv], tslot);
    else
        build_row<false, PRE, TY, FH>(a, Y, i, start, fi, fd, fval, fmask, nf, rc, ei, pri, prd,
                                      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                      nullptr, tslot);
#ifdef GLL_TRACE
    if (lane_id() == 0 && gxy.y == 0) {
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t_entry;
        if ((i & 15) == 0) atomicMax(&g_trace[20], dt);
        if (rc > a.RCAP) atomicMax(&g_trace[21], dt);
        if (tslot >= 0) g_trace[tslot + 7] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

hipError_t launch_finalize(const Layout& L, const Batch& bt, void* ws, const void* Y,
                           int y_dtype, float tau, float eps_fixed, hipStream_t s) {
    if (L.C > kMaxCPerLane * kWave) return hipErrorInvalidValue;
    RowArgs a;
    a.n = L.n;
    a.base = L.base;
    a.C = L.C;
    a.K = L.K;
    a.RCAP = L.RCAP;
    a.Wcap = L.Wcap;
    a.bump_base = int64_t(L.n) * L.Wcap;
    a.tau = tau;
    a.eps_fixed = eps_fixed;
    a.knn_idx = L.at<int32_t>(ws, L.knn_idx);
    a.knn_d2 = L.at<float>(ws, L.knn_d2);
    a.rev_cnt = L.at<int32_t>(ws, L.rev_cnt);
    a.rev_idx = L.at<int32_t>(ws, L.rev_idx);
    a.rev_d2 = L.at<float>(ws, L.rev_d2);
    a.ovf = L.at<int32_t>(ws, L.ovf);
    a.status = L.at<int32_t>(ws, L.status);
    a.eps = L.at<float>(ws, L.eps);
    a.tmp_col = L.at<int32_t>(ws, L.tmp_col);
    a.tmp_d2 = L.at<float>(ws, L.tmp_d2);
    a.row_start = L.at<int32_t>(ws, L.row_start);
    a.row_len = L.at<int32_t>(ws, L.row_len);
    a.col = L.at<int32_t>(ws, L.col);
    a.w = L.at<float>(ws, L.w);
    a.d2e = L.at<float>(ws, L.d2e);
    a.deg = L.at<float>(ws, L.deg);
    a.ucnt = L.at<int32_t>(ws, L.ucnt);
    a.diag = L.at<float>(ws, L.diag);
    a.rhs = L.at<float>(ws, L.rhs);
    a.P = L.at<float>(ws, L.P);
    a.Wadj = L.at<float>(ws, L.Wadj);
    a.ell = L.at<int32_t>(ws, L.ell);
    a.SE = ell_emit(L, bt.B);
    a.m = L.m;
    a.vr = L.at<char>(ws, L.vr);
    a.VRM = L.VRM;
    a.fsync = L.at<unsigned>(ws, L.fsync);
    a.gsync = grid_cg_route(L, bt) ? L.at<unsigned>(ws, L.cgv) : nullptr;
    a.wss = bt.ws;
    dim3 grid((L.n + 3) / 4, bt.B);
    // label prefetch: single graphs (its LDS halves the resident workgroups, which batches need)
    const int kp = knob(GLL_KNOB_ROW_PRE);
    const bool pre = kp == 1 || (kp == 0 && bt.B == 1);
    prof_begin(GLL_K_FINALIZE, s);
    // Batched launches address the workspace through flat pointers (integer-shifted, so the
    // compiler cannot prove them global): measured faster there (NS B = 64 68 -> 63 us, FullySup
    // B = 64 127 -> 116 us, profiles/r02h_rows_flat_ab.txt), while the single-graph kernel is
    // as fast or faster with global loads (6.5 -> 6.4 us).  XCD-contiguous numbering (R) measured
    // slower here even with the graph index taken once (NS B = 64 62 -> 66 us, FullySup B = 64
    // 116 -> 125 us, profiles/r02h_xcd_ab.txt).
// (K - 1 > 64: the forward list in 64-entry parts, FH = 2 up to K - 1 = 128, 4 up to 256)
#define GLL_ROWS_FH(T, FHV)                                                                  \
    do {                                                                                     \
        if (bt.B == 1)                                                                       \
            launch_k(row_build_kernel<T, true, false, false, FHV>, grid, 256, 0, s, a,       \
                     static_cast<const T*>(Y), bt.y);                                        \
        else                                                                                 \
            launch_k(row_build_kernel<T, false, true, false, FHV>, grid, 256, 0, s, a,       \
                     static_cast<const T*>(Y), bt.y);                                        \
    } while (0)
#define GLL_ROWS(T)                                                                          \
    do {                                                                                     \
        if (L.K - 1 > 2 * kWave)                                                             \
            GLL_ROWS_FH(T, 4);                                                               \
        else if (L.K - 1 > kWave)                                                            \
            GLL_ROWS_FH(T, 2);                                                               \
        else if (pre)                                                                        \
            launch_k(row_build_kernel<T, true, false>, grid, 256, 0, s, a, static_cast<const T*>(Y), bt.y);  \
        else if (bt.B == 1)                                                                  \
            launch_k(row_build_kernel<T, false, false>, grid, 256, 0, s, a, static_cast<const T*>(Y), bt.y); \
        else                                                                                 \
            launch_k(row_build_kernel<T, false, true>, grid, 256, 0, s, a, static_cast<const T*>(Y), bt.y); \
    } while (0)
    if (y_dtype == GLL_DT_F32) GLL_ROWS(float);
    else if (y_dtype == GLL_DT_F64) GLL_ROWS(double);
    else if (y_dtype == GLL_DT_I64) GLL_ROWS(int64_t);
    else return hipErrorInvalidValue;
#undef GLL_ROWS
#undef GLL_ROWS_FH
    prof_end(GLL_K_FINALIZE, s);
    return launch_status("rows.hip:launch_finalize");
}

}  // namespace gll
