// gll_internal.h -- workspace layout, device helpers and launcher declarations shared by
// the HIP translation units of libgll.  CDNA4 (gfx950) only: wave64, fp32 MFMA.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "gll.h"

namespace gll {

constexpr int kWave = 64;
constexpr int kMaxKm1 = 56;      // K - 1 <= 56: knn_select_kernel (one candidate per lane; the
                                 // rescan keeps >= 8 lanes of a wave free)
constexpr int kMaxKm1Wide = 128; // K - 1 <= 128: knn_select_wide_kernel, 256 candidate slots
constexpr int kMaxKm1Huge = 256; // K - 1 <= 256: the same kernel with 512 slots (k <= 257)

// ---------------------------------------------------------------------------------------
// Workspace layout.  One block per forward/backward pair, carved into 256-B aligned arrays.
// All sizes are functions of (n, d, base, C, K) only, so forward and backward agree.
//
// Graph storage ("padded rows"): row i of the symmetric kNN graph holds row_len[i] entries
// (col, w, d2) starting at row_start[i], sorted by column.  Ordinary rows sit in a fixed slot
// i * Wcap (Wcap = 5(K-1) + 8); rows longer than that (hubs) get their storage from a bump
// region behind the slots.  No prefix sum over rows is ever needed.
// ---------------------------------------------------------------------------------------
constexpr int kStOvfCount = 8;   // internal status words: overflow-list length
constexpr int kStBump = 9;       //                        bump-region cursor
constexpr int kStPermValid = 11; //                        1: this forward wrote the locality
                                 //                        order (order_perm_kernel); the Gram
                                 //                        zeroes it, so a backward never reads
                                 //                        a perm its forward did not write
constexpr int kPiv = 64;         // pivot rows of the locality order (order_pid_kernel)
constexpr int kStWords = GLL_ST_NWORDS;   // words the Gram kernels zero per call

// ELL slice width of the per-column CG kernels for m unlabeled rows (solve.hip dispatch);
// row_build emits that many column-major (col, w) slots per U row, 0 when no ELL kernel runs.
// Even: two slots per 16-B record (Layout::ell).
inline int ell_slots(int m) {
    return m <= 512 ? 24 : (m <= 2048 ? 16 : (m <= 4096 ? 4 : 0));
}

// Balanced per-column CG (solve.hip cg_vr_kernel): the U block of each row cut into "virtual
// rows" of kVS entries.  row_build writes them pre-packed for it, kVrSlot bytes per virtual
// row (kVS 16-bit LDS byte offsets of the columns, then kVS fp32 weights, zero-padded), at
// most kVrMax(K) of them per U row (row u's j-th at slot u * kVrMax + j); longer rows keep
// their tail in the CSR only.  vr_threads(L) > 0 <=> the per-column solves of this problem
// run that kernel (with vr_threads(L) virtual rows per thread): a host-side function of the
// problem alone, so row_build and the CG agree without a device round trip.
constexpr int kVS = 8;
constexpr int kVrSlot = kVS * 2 + kVS * 4;   // 48 B
// threads of the balanced kernel: 512, up to 10 virtual rows each in 256 VGPRs (1024 threads
// hold at most 5 in 128 VGPRs and spilled: 118 against 66 us per FullySup solve)
constexpr int kVrNT = 512;
// Virtual-row slots per U row: enough for a row of Layout::Wcap = 5(K-1)+8 entries (the row
// slot); hub rows in the bump region can be longer, and so can rows at k > 101, where the
// 6-bit slot field of the CG's virtual-row map caps this at 63: their tail stays in the CSR and
// the balanced kernel's spill path sums it (tests force both: the VRM clamp and the spill).
inline int vr_max_per_row(int K) {
    const int v = ((K - 1) + 4 * (K - 1) + 8 + kVS - 1) / kVS;
    return v < 63 ? v : 63;
}

// Process-wide test knobs (gll_set_knob, include/gll.h): each forces a code path, never a result.
// An atomic load, not a getenv per call (host time on the step's critical path).
int knob(int id);
// Set GLL_DEBUG=1 in the environment to print launch failures (read once).
bool debug_log();
// Device facts the launchers need, queried once per device / kernel and cached for the process.
int device_cus();                                          // CUs of the current device
int occupancy_blocks(const void* fn, int nt, size_t lds);  // resident blocks per CU
size_t static_lds_bytes(const void* fn);                   // the kernel's static LDS

inline int vr_threads(int n, int m, int K, int flags) {
    if (m <= 0 || m > 4 * kVrNT || (flags & GLL_FLAG_CG_ELL)) return 0;
    // kNN union rows hold ~1.4 (K-1) entries, a fraction m/n of them in the U block
    const double len = 1.4 * (K - 1) * double(m) / double(n);
    if (len <= 12.0 && !(flags & GLL_FLAG_CG_VR)) return 0;
    const double v = m * (len / kVS + 0.5);
    int rv = int((v + kVrNT - 1) / kVrNT);
    // tests: force the register capacity (4 at K = 25 puts most rows on the CSR spill path)
    if (knob(GLL_KNOB_VR_RV) > 0) rv = knob(GLL_KNOB_VR_RV);
    return rv <= 4 ? 4 : (rv <= 8 ? 8 : (rv <= 10 ? 10 : 0));
}

// ---------------------------------------------------------------------------------------
// In-kernel timestamps (diagnostic builds only: build.py --trace defines GLL_TRACE and
// writes libgll_trace.so; the product library compiles these to nothing).  Per translation
// unit, 64 words of s_memrealtime (100 MHz): [0,24) checkpoints of block 0 / thread 0,
// [24,32) last workgroup entry of kernel k < 8, [32,64) (first entry, last exit) pairs of up
// to 16 kernels over all workgroups.
// ---------------------------------------------------------------------------------------
#ifdef GLL_TRACE
#define GLL_TRACE_UNIT(name)                                                                 \
    static __device__ unsigned long long g_trace[64];                                       \
    static __device__ unsigned long long g_wg[2 * 3 * 4096]; /* kernels 0-1: entry, exit, cu */ \
    void trace_read_##name(unsigned long long* out) {                                       \
        (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), sizeof(g_trace));               \
    }                                                                                        \
    void trace_read_wg_##name(unsigned long long* out) {                                    \
        (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg), sizeof(g_wg));                     \
    }                                                                                        \
    void trace_reset_##name() {                                                              \
        unsigned long long h[64];                                                            \
        for (int i = 0; i < 64; ++i) h[i] = (i >= 32 && (i & 1) == 0) ? ~0ull : 0ull;       \
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_trace), h, sizeof(h));                         \
    }                                                                                        \
    struct TraceScope {                                                                      \
        int k;                                                                               \
        /* sampled (every 16th workgroup): a global atomic per workgroup of a 640-workgroup   \
           launch serialises at the memory side and distorts what it measures */              \
        __device__ explicit TraceScope(int k_) : k(k_) {                                     \
            if (threadIdx.x == 0 && ((blockIdx.x | blockIdx.y) & 15) == 0) {                 \
                const unsigned long long t = __builtin_amdgcn_s_memrealtime();               \
                atomicMin(&g_trace[32 + 2 * k], t);                                          \
                atomicMax(&g_trace[24 + k], t);                                              \
                if (k < 2 && blockIdx.x < 4096 && blockIdx.y == 0) {                         \
                    g_wg[k * 3 * 4096 + blockIdx.x] = t;                                     \
                    g_wg[k * 3 * 4096 + 2 * 4096 + blockIdx.x] = __smid();                   \
                }                                                                            \
            }                                                                                \
        }                                                                                    \
        __device__ ~TraceScope() {                                                           \
            if (threadIdx.x == 0 && ((blockIdx.x | blockIdx.y) & 15) == 0) {                 \
                const unsigned long long t = __builtin_amdgcn_s_memrealtime();               \
                atomicMax(&g_trace[33 + 2 * k], t);                                          \
                if (k < 2 && blockIdx.x < 4096 && blockIdx.y == 0)                           \
                    g_wg[k * 3 * 4096 + 4096 + blockIdx.x] = t;                              \
            }                                                                                \
        }                                                                                    \
    };
#define GLL_TRACE_SCOPE(k) TraceScope gll_trace_scope_(k)
#define GLL_TRACE_PT(i)                                                                      \
    do {                                                                                     \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_trace[i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define GLL_TRACE_ENTER(k)                                                                   \
    do {                                                                                     \
        if (threadIdx.x == 0) atomicMin(&g_trace[32 + 2 * (k)], __builtin_amdgcn_s_memrealtime()); \
    } while (0)
#define GLL_TRACE_EXIT(k)                                                                    \
    do {                                                                                     \
        if (threadIdx.x == 0) atomicMax(&g_trace[33 + 2 * (k)], __builtin_amdgcn_s_memrealtime()); \
    } while (0)
#else
#define GLL_TRACE_UNIT(name)
#define GLL_TRACE_SCOPE(k) do {} while (0)
#define GLL_TRACE_PT(i) do {} while (0)
#define GLL_TRACE_ENTER(k) do {} while (0)
#define GLL_TRACE_EXIT(k) do {} while (0)
#endif

// D2 planes.  A single small graph (T = ceil(n / 64) <= 16 tiles a side, 256 < d <= 512)
// runs the split-phase Gram (gram_bf3s_kernel): T^2 workgroups, each off-diagonal tile as two
// feature-phase halves writing partial planes that the select kernel adds in a fixed order.
// Batches already fill the chip and keep one plane (the layout still reserves two, which is
// 4 MB a graph at most).  (Evenly split fp32 tiles were measured before: 21.5 / 23.5 us for
// KS = 2 / 4 against 16.9 us unsplit, profiles/r01_gram_dispatch.txt -- 2 T(T+1)/2
// workgroups overflow the 256 CUs; T^2 does not.)
inline int gram_splits(int n, int d) {
    return ((n + 63) / 64 <= 16 && d > 256 && d <= 512) ? 2 : 1;
}

// Rows of the squared-distance buffer: n (the whole n x n matrix), or a panel of PR rows when
// the matrix would pass 32 GiB (panels of 8 GiB) or GLL_FLAG_KNN_PANEL asks for panels of 1,024
// rows.  The kNN is then built panel by panel: rectangular Gram tiles of the panel's rows
// against every column, then the select of those rows (api.hip build_graph).  A multiple of 128
// (the Gram tile), < n in panel mode.
inline int panel_rows(int n, int flags) {
    const size_t row_bytes = size_t((n + 3) & ~3) * 4;
    int64_t pr = n;
    if (flags & GLL_FLAG_KNN_PANEL) pr = 1024;
    else if (size_t(n) * row_bytes > (size_t(32) << 30)) pr = int64_t((size_t(8) << 30) / row_bytes);
    if (pr >= n) return n;
    pr = (pr / 128) * 128;
    if (pr < 128) pr = 128;
    return pr < n ? int(pr) : n;
}

size_t grid_cg_workspace_floats(int m, int C);
// The whole-GPU CG's sync words at the start of its region (gridcg.hip kSyncWords): row_build
// zeroes them before a forward whose solves take that kernel (grid_cg_route), and each solve
// leaves them zero, so its launch needs no memset.
constexpr int kGridSyncWords = 2048;   // >= gridcg.hip kSyncWords
struct Layout;
int ell_emit(const Layout& L, int B);

struct Layout {
    int n, d, base, m, C, K;
    int flags;        // gll_problem.flags
    int KS;           // Gram split planes (gram_splits)
    int ldD;          // leading dimension of the n x n squared-distance matrix
    int PR;           // rows of the distance buffer (panel_rows: n, or a panel < n)
    int RCAP;         // reverse-list capacity per row
    int Wcap;         // slot width of a row
    int64_t Etot;     // entry capacity: n Wcap slots + 2 n (K-1) bump region
    size_t status, D2, knn_idx, knn_d2, eps, rev_cnt, rev_idx, rev_d2, ovf, row_start, row_len;
    size_t tmp_col, tmp_d2, col, w, d2e, deg, ucnt, diag, rhs, P, Wadj, S, b, cgv, total;
    int SE;           // ELL slots per U row (ell_slots; even)
    size_t ell;       // [SE/2][m] 16-B records (col_2s, w_2s, col_2s+1, w_2s+1)
    int RV;           // balanced CG: virtual rows per thread (vr_threads), 0 = not used
    int VRM;          // balanced CG: virtual-row slots per U row (vr_max_per_row)
    size_t vr;        // [m][VRM] packed virtual rows (kVrSlot bytes each)
    int dp;           // split-Gram planes: d rounded up to 64
    size_t xhi, xlo, xnrm;   // [n][dp] bf16 hi / lo planes of x - x_0, and |x - x_0|^2
    size_t fsync;     // fused backward: [0] solved columns, [32] finished gradient blocks,
                      // [64] poison (a lost solve: the counters may be stale), [96] release
                      // (set by the last column to arrive; the gradient blocks poll it)
    size_t d2s;       // float: the fp16 D2 scale of the pre-split GEMM (knn.hip tile_d2_scale)
    size_t pid, perm; // locality order (order_rows): nearest pivot of each row, the row order
    size_t ohist;     // locality order: rows per pivot of each 64-row block ([ceil(n/64)][64])

    explicit Layout(const gll_problem& p) {
        n = p.n; d = p.d; base = p.base; C = p.C;
        flags = p.flags;
        K = p.K < p.n ? p.K : p.n;
        m = n - base;
        ldD = (n + 3) & ~3;
        PR = panel_rows(n, flags);
        KS = PR < n ? 1 : gram_splits(n, d);
        // reverse-list capacity: past it a row's reverse entries go to the global overflow
        // list, which each such (hub) row then scans whole -- at stress (K = 30) 4(K-1)+8 left
        // 39 hubs scanning 742 entries, 14 of their 35 us (profiles/r05w_trace_stress.txt)
        RCAP = 8 * (K - 1) + 8;
        // A row's slot holds its forward list and up to 4(K-1)+8 reverse entries (~1.4(K-1)
        // entries on average); longer rows -- hubs -- take their storage from the bump region,
        // which holds every row at once if it must (all rows together have at most 2n(K-1)
        // entries).  The slot width is kept apart from RCAP: the six Etot arrays cost 24 B a
        // slot, and a 9(K-1)+8-wide slot made them 60% larger for every graph.
        Wcap = (K - 1) + 4 * (K - 1) + 8;
        Etot = int64_t(n) * Wcap + 2LL * n * (K - 1);
        size_t off = 0;
        auto take = [&](size_t bytes) {
            size_t at = off;
            off += (bytes + 255) & ~size_t(255);
            return at;
        };
        status = take(size_t(kStWords) * 4);
        D2 = take(size_t(KS) * PR * ldD * 4);  // KS partial planes (or one panel)
        knn_idx = take(size_t(n) * K * 4);
        knn_d2 = take(size_t(n) * K * 4);
        eps = take(size_t(n) * 4);
        rev_cnt = take(size_t(n) * 4);
        rev_idx = take(size_t(n) * RCAP * 4);
        rev_d2 = take(size_t(n) * RCAP * 4);
        ovf = take(size_t(n) * (K - 1) * 12);   // (row, col, d2) triples past RCAP
        row_start = take(size_t(n) * 4);
        row_len = take(size_t(n) * 4);
        tmp_col = take(size_t(Etot) * 4);       // staging of rows too long for LDS
        tmp_d2 = take(size_t(Etot) * 4);
        col = take(size_t(Etot) * 4);
        w = take(size_t(Etot) * 4);
        d2e = take(size_t(Etot) * 4);
        deg = take(size_t(n) * 4);
        ucnt = take(size_t(m) * 4);        // U-block entries per unlabeled row
        diag = take(size_t(m) * 4);
        rhs = take(size_t(m) * C * 4);
        SE = ell_slots(m);
        // U-block columns (U index) and weights W_uj of each U row's first SE entries, 0-padded,
        // two slots per 16-B record: one dwordx4 load brings two slots of a row (the CG's setup
        // issues SE/2 loads per row instead of 2 SE)
        ell = take(size_t(SE) * m * 8);
        RV = vr_threads(n, m, K, flags);
        VRM = RV ? vr_max_per_row(K) : 0;
        vr = take(size_t(m) * VRM * kVrSlot);
        dp = (d + 63) & ~63;
        xhi = take(size_t(n) * dp * 2);
        xlo = take(size_t(n) * dp * 2);
        xnrm = take(size_t(n) * 4);
        fsync = take(512);   // four words on their own 128-B lines, zeroed by row_build
        d2s = take(256);     // fp16 D2 scale of the pre-split Gram (knn.hip tile_d2_scale)
        pid = take(size_t(n) * 4);
        perm = take(size_t(n) * 4);
        ohist = take(size_t((n + 63) / 64) * 64 * 4);
        P = take(size_t(n) * C * 4);       // [Y; U] as fp32 (backward's P, GLL.py:109)
        Wadj = take(size_t(n) * C * 4);    // [0; Luu^-1 gbar] (backward's w, GLL.py:104)
        S = take(size_t(Etot) * 4);        // per-edge coefficient (auto eps / chunked gradient)
        b = take(size_t(n) * 4);           // auto-eps b_i (GLL.py:126)
        // CG vectors when they do not fit in LDS (per-column kernels) / of the grid-wide CG
        const size_t gf = grid_cg_workspace_floats(m, C);
        cgv = take((gf > size_t(5) * m * C ? gf : size_t(5) * m * C) * 4);
        total = off;
    }
    template <typename T>
    T* at(void* ws, size_t o) const { return reinterpret_cast<T*>(static_cast<char*>(ws) + o); }
};

// ELL slots row_build writes and the per-column CG reads for a launch over B graphs: the
// region's L.SE.  (Round 3 measured narrower slices for batches -- 12 or 16 of the 24 slots,
// the longer rows' tails in the LDS overflow -- and dropped them: B = 64 NS CG 21.6 us at 24
// slots against 26.9 at 16 and 29.6 at 12, profiles/r03j_batched_ell_width_ab.txt.)
inline int ell_emit(const Layout& L, int B) {
    (void)B;
    return L.SE;
}

// Planes the Gram kernel of a launch over B graphs writes (= planes the select kernel sums).
inline int gram_planes(const Layout& L, int B) { return (L.KS == 2 && B == 1) ? 2 : 1; }

// ---------------------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Wall-clock bound of the in-launch waits (grid barriers, the fused backward's hand-off):
// s_memrealtime ticks at a constant 100 MHz whatever the shader clock, so 1e8 ticks = 1 s.
constexpr unsigned long long kWaitTicks = 100000000ull;
__device__ __forceinline__ unsigned long long wall_ticks() {
    return __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Wave64 sum through DPP (no LDS round trips): quad butterflies, half-row and row mirrors,
// then row_bcast15/31 carry the row sums up to lane 63, which is broadcast via readlane.
// Fixed combination order -> deterministic; the result is wave-uniform (scalar).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add(float v) {
    const int s = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf,
                                              false);
    return v + __builtin_bit_cast(float, s);
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v = dpp_add<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]
    v = dpp_add<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]
    v = dpp_add<0x141, 0xf>(v);   // row_half_mirror
    v = dpp_add<0x140, 0xf>(v);   // row_mirror
    v = dpp_add<0x142, 0xa>(v);   // row_bcast15 -> rows 1, 3
    v = dpp_add<0x143, 0xc>(v);   // row_bcast31 -> rows 2, 3
    return readlane_f(v, 63);
}
// two independent sums interleaved (ILP across the two DPP chains)
__device__ __forceinline__ void wave_sum2_dpp(float& a, float& b) {
    a = dpp_add<0xB1, 0xf>(a); b = dpp_add<0xB1, 0xf>(b);
    a = dpp_add<0x4E, 0xf>(a); b = dpp_add<0x4E, 0xf>(b);
    a = dpp_add<0x141, 0xf>(a); b = dpp_add<0x141, 0xf>(b);
    a = dpp_add<0x140, 0xf>(a); b = dpp_add<0x140, 0xf>(b);
    a = dpp_add<0x142, 0xa>(a); b = dpp_add<0x142, 0xa>(b);
    a = dpp_add<0x143, 0xc>(a); b = dpp_add<0x143, 0xc>(b);
    a = readlane_f(a, 63);
    b = readlane_f(b, 63);
}

// Wave64 minimum of a 64-bit key through DPP; result broadcast to every lane.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_min_u64(uint64_t k) {
    const uint32_t lo = __builtin_amdgcn_update_dpp(0xFFFFFFFFu, uint32_t(k), CTRL, ROW_MASK, 0xf,
                                                    false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0xFFFFFFFFu, uint32_t(k >> 32), CTRL,
                                                    ROW_MASK, 0xf, false);
    const uint64_t o = (uint64_t(hi) << 32) | lo;
    return o < k ? o : k;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t k) {
    k = dpp_min_u64<0xB1, 0xf>(k);
    k = dpp_min_u64<0x4E, 0xf>(k);
    k = dpp_min_u64<0x141, 0xf>(k);
    k = dpp_min_u64<0x140, 0xf>(k);
    k = dpp_min_u64<0x142, 0xa>(k);
    k = dpp_min_u64<0x143, 0xc>(k);
    const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(k), 63);
    const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(k >> 32), 63);
    return (uint64_t(hi) << 32) | lo;
}
// Sum over each aligned group of 8 lanes (result in all 8 lanes of the group).
__device__ __forceinline__ float group8_sum(float v) {
    v = dpp_add<0xB1, 0xf>(v);
    v = dpp_add<0x4E, 0xf>(v);
    v = dpp_add<0x141, 0xf>(v);
    return v;
}
// Number of set bits of `mask` below this lane (wave-level compaction).
__device__ __forceinline__ int lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi(uint32_t(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo(uint32_t(mask), 0));
}

template <typename T>
__device__ __forceinline__ float to_f32(T v) { return static_cast<float>(v); }

// Load 4 consecutive floats p[k..k+3] (zeros beyond `lim`).  VEC: 16-B vector load, needs
// lim % 4 == 0 and 16-B alignment; otherwise scalar loads.  Branch-free: out-of-range lanes
// load p[0..] (p must be readable) and select zero, so hipcc keeps exact vmcnt counting and
// prefetches stay in flight (a predicated load becomes a branch + vmcnt(0) drain).
template <bool VEC>
__device__ __forceinline__ f32x4 load4(const float* __restrict__ p, int k, int lim) {
    f32x4 v;
    if constexpr (VEC) {
        const bool in = k < lim;
        v = *reinterpret_cast<const f32x4*>(p + (in ? k : 0));
        v = in ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
        const float a = p[k + 0 < lim ? k + 0 : 0];
        const float b = p[k + 1 < lim ? k + 1 : 0];
        const float c = p[k + 2 < lim ? k + 2 : 0];
        const float e = p[k + 3 < lim ? k + 3 : 0];
        v.x = k + 0 < lim ? a : 0.f;
        v.y = k + 1 < lim ? b : 0.f;
        v.z = k + 2 < lim ? c : 0.f;
        v.w = k + 3 < lim ? e : 0.f;
    }
    return v;
}

// load4 split in two halves for software pipelining: the load (address clamped into the
// row, never branched) and the zero-mask of the lanes past `lim`, applied where the value
// is consumed -- a mask right after the load would make the wave wait for it there.
template <bool VEC>
__device__ __forceinline__ f32x4 load4_raw(const float* __restrict__ p, int k, int lim) {
    f32x4 v;
    if constexpr (VEC) {
        v = *reinterpret_cast<const f32x4*>(p + (k < lim ? k : 0));
    } else {
        v.x = p[k + 0 < lim ? k + 0 : 0];
        v.y = p[k + 1 < lim ? k + 1 : 0];
        v.z = p[k + 2 < lim ? k + 2 : 0];
        v.w = p[k + 3 < lim ? k + 3 : 0];
    }
    return v;
}
template <bool VEC>
__device__ __forceinline__ f32x4 mask4(f32x4 v, int k, int lim) {
    if constexpr (VEC) {
        return k < lim ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
        v.x = k + 0 < lim ? v.x : 0.f;
        v.y = k + 1 < lim ? v.y : 0.f;
        v.z = k + 2 < lim ? v.z : 0.f;
        v.w = k + 3 < lim ? v.w : 0.f;
        return v;
    }
}

// ---------------------------------------------------------------------------------------
// Batched launches: B independent graphs of the same shape in one launch per kernel, graph
// g = blockIdx.y.  Every pointer a kernel receives is graph 0's; gshift moves it to graph g
// by a per-array byte stride (0 = shared by all graphs, e.g. a status sink).
// ---------------------------------------------------------------------------------------
struct Batch {
    int B = 1;
    size_t ws = 0;   // workspace block
    size_t x = 0;    // X (n x d fp32)
    size_t y = 0;    // label matrix (base x C, its dtype)
    size_t u = 0;    // U output (m x C fp64)
    size_t g = 0;    // upstream gradient (m x C, its dtype)
    size_t gx = 0;   // gradX output (n x d fp32)
    size_t st = 0;   // public status words: ws when they live in the workspace, 0 for a sink
};

// XCD-aware block numbering of batched launches.  Blocks are dealt round-robin over the 8 XCDs
// in dispatch order (linear index L = y * gridDim.x + x, XCD = L % 8; DESIGN.md §3.5: a
// speed assumption, never a correctness one).  For gridDim.y = B > 1 graphs, block (x, y) is
// renumbered so that each XCD works through a contiguous run of the graph-major sequence: a
// graph's blocks share one XCD's L2 (its X rows, its D2, its CSR) instead of each of the 8
// XCDs refilling every graph.  batch_xy() = (block within the graph, graph); single graphs keep
// (blockIdx.x, 0).  Every kernel that runs batched takes its block and graph from here.
template <bool R = false>
__device__ __forceinline__ int2 batch_xy() {
    if (!R || gridDim.y == 1) return int2{int(blockIdx.x), int(blockIdx.y)};
    const int nb = gridDim.x, nt = nb * gridDim.y;
    const int L = blockIdx.y * nb + blockIdx.x;
    const int x = L & 7, q = L >> 3, per = nt >> 3, extra = nt & 7;
    const int idx = x * per + (x < extra ? x : extra) + q;
    return int2{idx % nb, idx / nb};
}
// R = true only where it measured faster (tools/ab_flags.py, B = 64 / 8): the per-column CG
// (NS B = 64 32 -> 24 us, stress B = 64 2.0 -> 1.1 ms) and the whole-row feature gradient (NS
// B = 64 198 -> 178 us, FullySup B = 64 347 -> 305 us), and -- once kernels took batch_xy once
// instead of per pointer (gshift_at) -- the select (NS B = 64 220 -> 213 us).  The row build
// still runs slower with it (62 -> 66 us), and the chunked gradient needs block % 8 = chunk.
// A kernel computes batch_xy ONCE: per call it re-reads gridDim and divides.
template <bool R = false>
__device__ __forceinline__ int bx() { return batch_xy<R>().x; }
template <bool R = false>
__device__ __forceinline__ int bg() { return batch_xy<R>().y; }

// Branch-free on purpose: a branch per pointer splits the prologue into basic blocks with an
// s_waitcnt each, serialising the kernel-argument loads (~13 dependent scalar loads, ~0.5 us
// at the start of every kernel); selects let them all be in flight at once.
// Pointer (not integer) arithmetic: an integer round trip loses the pointer's provenance, and
// with it the compiler's proof that it points to global memory -- every access through it
// became a flat instruction (no scalar base, waits on both the vector and LDS counters).
template <bool R = false, typename T>
__device__ __forceinline__ T* gshift(T* p, size_t stride) {
    using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    const size_t off = size_t(bg<R>()) * stride;
    return reinterpret_cast<T*>(reinterpret_cast<B*>(p) + (p != nullptr ? off : size_t(0)));
}

// Integer-arithmetic form: the result is a generic (flat) pointer to the compiler.  Kept for
// the batched row build, where flat accesses measured faster (rows.hip launch_finalize).
template <typename T>
__device__ __forceinline__ T* gshift_flat_at(T* p, size_t stride, int g) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uintptr_t off = uintptr_t(g) * stride;
    return reinterpret_cast<T*>(a + (a != 0 ? off : uintptr_t(0)));
}

// The same with the graph index already known (a kernel shifting many pointers computes
// batch_xy once: per pointer, the batched numbering re-reads gridDim and divides each time).
template <typename T>
__device__ __forceinline__ T* gshift_at(T* p, size_t stride, int g) {
    using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    const size_t off = size_t(g) * stride;
    return reinterpret_cast<T*>(reinterpret_cast<B*>(p) + (p != nullptr ? off : size_t(0)));
}

// Branching form for the register-tight Gram kernels (four pointers, no long load chain):
// the select form costs them 36-84 B more of scratch spills.
template <bool R = false, typename T>
__device__ __forceinline__ T* gshift_br(T* p, size_t stride) {
    if (p == nullptr || stride == 0) return p;
    using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    return reinterpret_cast<T*>(reinterpret_cast<B*>(p) + size_t(bg<R>()) * stride);
}

template <typename T>
__device__ __forceinline__ T* gshift_br_at(T* p, size_t stride, int g) {
    if (p == nullptr || stride == 0) return p;
    using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    return reinterpret_cast<T*>(reinterpret_cast<B*>(p) + size_t(g) * stride);
}

// Launch-error report (GLL_DEBUG=1 in the environment): which launcher failed and why.
hipError_t launch_status(const char* what);

// Opt a kernel into all of the 160 KiB of LDS its static allocation leaves for dynamic use
// (once per kernel; solve.hip).
void allow_full_lds(const void* fn);

// Every kernel goes out through launch_k.  When prof_begin has armed an event pair for the next
// launch (gll_prof_enable: bench.py times its dominant kernel inside the timed region), the
// events ride in the dispatch packet itself (hipExtLaunchKernelGGL start / stop), so they time
// the kernel the way rocprofv3 does rather than the queue between two separate event packets.
struct ArmedLaunch {
    int kid = -1;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int span = 1;   // launches the timed phase spans: the first records e0, the last e1
};
extern thread_local ArmedLaunch g_armed;

// A timed phase made of `n` consecutive launches (e.g. the Gram's split + GEMM): call right
// after prof_begin.
inline void prof_span(int n) {
    if (g_armed.kid >= 0) g_armed.span = n;
}

template <typename F, typename... Args>
inline void launch_k(F fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args) {
    if (g_armed.kid >= 0 && g_armed.span > 1) {
        const hipEvent_t e0 = g_armed.e0;
        g_armed.e0 = nullptr;
        --g_armed.span;
        hipExtLaunchKernelGGL(fn, grid, block, uint32_t(lds), s, e0, nullptr, 0u, args...);
    } else if (g_armed.kid >= 0) {
        const hipEvent_t e0 = g_armed.e0, e1 = g_armed.e1;
        g_armed.kid = -1;
        g_armed.span = 1;
        hipExtLaunchKernelGGL(fn, grid, block, uint32_t(lds), s, e0, e1, 0u, args...);
    } else {
        fn<<<grid, block, lds, s>>>(args...);
    }
}

// ---------------------------------------------------------------------------------------
// Launchers (host side, one per translation unit)
// ---------------------------------------------------------------------------------------
void prof_begin(int kid, hipStream_t s);
void prof_end(int kid, hipStream_t s);

hipError_t launch_gram(const Layout& L, const Batch& bt, void* ws, const float* X, bool vec,
                       hipStream_t s);
// rows r0 .. r0 + rows - 1 of the graph (a panel, D2 holding only them); rows < 0: every row
hipError_t launch_select(const Layout& L, const Batch& bt, void* ws, const float* X,
                         float eps_fixed, bool auto_eps, bool vec, int32_t* status_pub,
                         hipStream_t s, int r0 = 0, int rows = -1);
hipError_t launch_gram_panel(const Layout& L, void* ws, const float* X, bool vec, int r0, int rows,
                             hipStream_t s);
// Locality order of the rows of one large graph (knn.hip order_rows): rows grouped by their
// nearest of kPiv pivot rows under the Gram distances, so each XCD's share of the select and of
// the chunked gradient is a run of rows whose neighbours mostly lie in the same run -- the X rows
// those kernels gather then stay in that XCD's 4 MB L2 instead of streaming from the MALL.  Speed
// only: every row's result is independent of the order.  Single graphs whose X exceeds an XCD's
// L2 (n d 4 B > 4 MB), with the whole n x n distance matrix (no row panels).
inline bool locality_order(const Layout& L, const Batch& bt) {
    return bt.B == 1 && L.PR == L.n && L.n >= 16 * kPiv &&
           size_t(L.n) * L.d * 4 > (size_t(4) << 20) && !(L.flags & GLL_FLAG_ROW_ORDER_OFF);
}
hipError_t launch_order(const Layout& L, void* ws, hipStream_t s);
// The Luu solves of this problem try the whole-GPU CG first (solve.hip cg_dispatch): single
// graphs past the per-column kernels' sweet spot (m > 2048), or forced by GLL_FLAG_CG_GRID.
inline bool grid_cg_route(const Layout& L, const Batch& bt) {
    return bt.B == 1 && L.C <= 16 && !(L.flags & GLL_FLAG_CG_PERCOL) &&
           (L.m > 2048 || (L.flags & GLL_FLAG_CG_GRID));
}
hipError_t launch_finalize(const Layout& L, const Batch& bt, void* ws, const void* Y,
                           int y_dtype, float tau, float eps_fixed, hipStream_t s);
// b: right-hand sides of graph 0, `b_stride` bytes apart (the workspace rhs or gbar)
// st_failed: the public GLL_ST_SOLVE_FAILED word (whole-GPU CG barrier failure)
hipError_t launch_cg_luu(const Layout& L, const Batch& bt, void* ws, const void* b,
                         size_t b_stride, int b_dtype, double* out64, float* out32, float rtol,
                         int max_iter, int32_t* st_nonconv, int32_t* st_iters,
                         int32_t* st_failed, hipStream_t s);
// The whole-GPU CG returns hipErrorNotSupported when no grid configuration holds the system
// (C > 16 or more rows than the co-resident workgroups can keep in registers): callers then
// run the per-column kernels with the Krylov vectors in the workspace.
hipError_t launch_cg_grid_luu(const Layout& L, void* ws, const void* b, int b_dtype,
                              double* out64, float* out32, float rtol, float atol,
                              int max_iter, int32_t* st_nonconv, int32_t* st_iters,
                              int32_t* st_failed, hipStream_t s);
hipError_t launch_cg_grid_csr(int m, int C, const int32_t* row_ptr, const int32_t* col,
                              const float* val, int64_t nnz, const float* b, float* x,
                              float atol, int max_iter, int32_t* iters, int32_t* nonconv,
                              int32_t* failed, float* ws, hipStream_t s);
hipError_t launch_cg_csr(int m, int C, const int32_t* row_ptr, const int32_t* col,
                         const float* val, const float* b, float* x, float atol, int max_iter,
                         int32_t* iters, int32_t* nonconv, float* gvec, hipStream_t s);
hipError_t launch_backward_grad(const Layout& L, const Batch& bt, void* ws, const float* X,
                                bool auto_eps, float eps_fixed, float* gradX, bool vec,
                                hipStream_t s);
// One small graph, fixed eps: the adjoint CG and the feature gradient in one launch
// (solve.hip cg_grad_fused_kernel); hipErrorNotSupported when the shape does not qualify.
hipError_t launch_cg_grad_fused(const Layout& L, void* ws, const void* gbar, int g_dtype,
                                const float* X, float eps_fixed, float* gradX, float rtol,
                                int max_iter, int32_t* st_nonconv, int32_t* st_iters,
                                int32_t* st_failed, bool vec, hipStream_t s);

}  // namespace gll
