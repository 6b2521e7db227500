// orbit_hip.hip — MI355X (gfx950 / CDNA4) kernels for the per-snapshot orbit-tagging
// hot path of s-balu/nbody-orbit-analysis, behind the C ABI of include/orbit_hip.h.
//
// Reference path (paths under /root/reference/orbitanalysis/):
//   region_frame               track_orbits.py:247-290    -> k_step phase 1
//   compare_radial_velocities  track_orbits.py:293-327    -> k_step phase 2
//   calc_angles                track_orbits.py:330-351    -> k_step phase 2
//   result assembly            track_orbits.py:199-227    -> k_step (direct records), or
//                                                            k_scan_slots, k_gather_*
//   bulk velocity (sum/mean)   track_orbits.py:262-284    -> k_bulk
//   large halos                (same functions)           -> k_part_scatter, k_part_join;
//                                                            k_big_frame, k_big_join
//   on-the-fly driver          track_orbits_onthefly.py   -> k_step<..., OTF>, k_big_*
//   module-level helpers       track_orbits.py:293-351    -> k_match_*, k_compare_pairs,
//                                                            k_angle_add
//
// Design: one work-group per *item* (a run of consecutive halos whose
// current blocks fit the LDS hash table; larger halos go through per-halo tables in
// global memory, k_big_*).  Phase 1 streams the item's current blocks (ids, AoS x,
// AoS v) once, computes the frame in registers, writes r̂ and inserts (halo, id) ->
// position into an LDS cuckoo table.  Phase 2a streams the progenitor blocks' IDs
// and state words, probes the table and decides the strict sign test; phase 2b
// stages the item's current r̂ into the LDS the table occupied, streams the
// progenitor r̂, applies the arccos angle update and compacts apsis records in
// previous-block order with wave ballots.  Every input byte is read from HBM once;
// no sort, no per-particle gather from L2.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (no FMA contraction:
// the reference's NumPy arithmetic rounds every product and sum).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <math.h>
#include <type_traits>

#include "orbit_hip.h"

// Units of the library built from this file (OA_TU): 0 = everything in one unit; the
// split build (_build.py, units compiled in parallel) = -1 (the C ABI and every kernel
// but the step launchers) + 1, 2, 3 (the step launchers of one dtype plan each: float32
// coordinates and r̂, float32 coordinates with float64 r̂, float64).
#ifndef OA_TU
#define OA_TU 0
#endif
void oa_internal_error(const char *msg);   // the oa_last_error() buffer (unit 0 / -1)

namespace {

#ifndef OA_WG
#define OA_WG 1024
#endif
#ifndef OA_UNR1
#define OA_UNR1 1           // phase 1: rows per wave trip (2: dynamic trips; A/B r02 wg: 1 is 0.7 % faster)
#endif
#ifndef OA_KROWS
#define OA_KROWS (12 * 1024 / OA_WG)   // phase 2: progenitor rows held per wave (n_pv <= KROWS * WG)
#endif
#ifndef OA_PF2
#define OA_PF2 5            // phase 2b: rows of previous r̂ loads in flight ahead (A/B r02: 2 +3.5 %, 4 = 3, 5 -0.4 %)
#endif
#ifndef OA_HMAX
#define OA_HMAX 32
#endif
// phase 2b stages an item's current r̂ through registers, STAGE_* rows per thread:
// lds_entries <= STAGE_* * WG (11776 float32 / 6144 float64 entries fill the LDS)
constexpr int STAGE_F32 = 12 * 1024 / OA_WG, STAGE_F64 = 6 * 1024 / OA_WG;
constexpr int WG = OA_WG;           // k_step work-group
constexpr int NWAVE = WG / 64;
constexpr int HMAX = OA_HMAX;       // halos per item
constexpr int UNR1 = OA_UNR1;       // phase-1 particles per thread per loop trip
constexpr int KROWS = OA_KROWS;
constexpr int PF2 = OA_PF2;
constexpr int BULK_CHUNK = 8192;    // numpy pairwise-sum buffer chunk
constexpr int STASH = 64;           // cuckoo stash entries per item
#ifndef OA_MAXEV
#define OA_MAXEV 48
#endif
#ifndef OA_PU
#define OA_PU 4             // k_part_join: previous entries per thread loaded up front
#endif
constexpr int MAX_EVICT = OA_MAXEV; // eviction-chain length before an entry is stashed
constexpr int NCAND = 3;            // cuckoo candidate slots per key
static_assert(WG % 64 == 0 && WG <= 1024, "work-group must be whole waves");
static_assert(HMAX < WG, "halo table is staged by one thread per halo");
// direct records: wave 0 writes one halo offset per lane (direct_tail) and resolves the
// look-back while waves 1.. write the state words (phase 3)
static_assert(HMAX <= 64, "an item's halos are one lane each of wave 0");
static_assert(WG > 64, "phase 3 of a direct-records step needs waves beside wave 0");

#if OA_TU <= 0
thread_local char g_err[512] = "";
#endif

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    oa_internal_error(buf);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(OA_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
    return OA_OK;
}

// ------------------------------------------------------------------ loads
// streamed-once inputs: non-temporal loads leave L2 to the lines that are re-read
template <typename T> __device__ __forceinline__ T lds_nt(const T *p) {
    return __builtin_nontemporal_load(p);
}

#ifndef OA_STAMPS
#define OA_STAMPS 0
#endif
#if OA_STAMPS && OA_TU != 0
// every unit of the split build would hold its own copy of the stamp buffers, and
// oa_debug_stamps (unit -1) would read an empty one: stamps builds are one unit
#error "OA_STAMPS needs the single-unit build (OA_TU=0, tools/variants.sh)"
#endif
#if OA_STAMPS
// diagnostic build only: per-work-group s_memrealtime (100 MHz) at the 8 phase
// boundaries plus, per wave, the ends of its phase-1, 2a and 2b loops (WSTAMP 0/1/2)
constexpr int STAMP_MAX_WG = 1 << 16, STAMP_NP = 9, STAMP_N = STAMP_NP + 3 * (OA_WG / 64) + 1;
__device__ uint64_t g_stamps[STAMP_MAX_WG * STAMP_N];
#define STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < STAMP_MAX_WG) \
    g_stamps[blockIdx.x * STAMP_N + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// the last word: a diagnostic value of the work-group (table walks)
#define DIAG(v) do { if (threadIdx.x == 0 && blockIdx.x < STAMP_MAX_WG) \
    g_stamps[blockIdx.x * STAMP_N + STAMP_N - 1] = (v); } while (0)
// large-halo partition kernels: 8 stamps per work-group of k_part_join, then 8 per
// work-group of k_part_scatter (start, its first sub-chunk's phases, end)
constexpr int PSTAMP_N = 8;
__device__ uint64_t g_pstamps[STAMP_MAX_WG * PSTAMP_N];
__device__ uint64_t g_sstamps[STAMP_MAX_WG * PSTAMP_N];
#define PSTAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < STAMP_MAX_WG) \
    g_pstamps[blockIdx.x * PSTAMP_N + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define SSTAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < STAMP_MAX_WG) \
    g_sstamps[blockIdx.x * PSTAMP_N + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define WSTAMP(k) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < STAMP_MAX_WG) \
    g_stamps[blockIdx.x * STAMP_N + STAMP_NP + 3 * (threadIdx.x >> 6) + (k)] = \
        __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PSTAMP(k) do { } while (0)
#define SSTAMP(k) do { } while (0)
#define STAMP(k) do { } while (0)
#define WSTAMP(k) do { } while (0)
#define DIAG(v) do { } while (0)
#endif

template <typename T> struct V3 { T x, y, z; };

template <typename T>
__device__ __forceinline__ V3<T> ld3(const T *p, int64_t i) {
    const T *q = p + 3 * i;
    return V3<T>{q[0], q[1], q[2]};
}
template <typename T>
__device__ __forceinline__ V3<T> ld3_nt(const T *p, int64_t i) {
    const T *q = p + 3 * i;
    return V3<T>{lds_nt(q), lds_nt(q + 1), lds_nt(q + 2)};
}

// Row dot product in the reference host's einsum order (probed):
// f64 sums (p0 + p2) + p1, f32 (p0 + p1) + p2; no FMA (-ffp-contract=off).
__device__ __forceinline__ double dot3(double a0, double a1, double a2,
                                       double b0, double b1, double b2) {
    double p0 = a0 * b0, p1 = a1 * b1, p2 = a2 * b2;
    return (p0 + p2) + p1;
}
__device__ __forceinline__ float dot3(float a0, float a1, float a2,
                                      float b0, float b1, float b2) {
    float p0 = a0 * b0, p1 = a1 * b1, p2 = a2 * b2;
    return (p0 + p1) + p2;
}

__device__ __forceinline__ double acos_td(double x) { return acos(x); }
// numpy's float32 arccos (SIMD) is not correctly rounded either: both differ from the
// exact value by ~1 ulp; parity for float16 angles is checked to within 1 f16 ulp.
__device__ __forceinline__ float acos_td(float x) { return acosf(x); }
// The on-the-fly driver returns the angle changes themselves (track_orbits_onthefly.py:
// 173-174): a float32 change is rounded from a float64 arccos, i.e. correctly rounded
// (but for ~1e-8 of values), so it is within numpy's own float32 arccos error (<= 2 ulp,
// measured) of the reference; acosf alone adds its error on top.  The batch path keeps
// acosf: its changes only feed float16 sums.
template <bool OTF, typename TD> __device__ __forceinline__ TD acos_change(TD x) {
    if constexpr (OTF && sizeof(TD) == 4) return (float)acos((double)x);
    else return acos_td(x);
}

__device__ __forceinline__ uint16_t f32_to_f16(float f) {
    _Float16 h = (_Float16)f;                     // v_cvt_f16_f32, round to nearest even
    return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float f16_to_f32(uint16_t b) {
    return (float)__builtin_bit_cast(_Float16, b);
}
// float64 -> float16 with ONE rounding (numpy astype(float16) of a float64):
// round to odd into float32 (24 >= 11 + 2 bits), then nearest-even to float16.
__device__ __forceinline__ uint16_t f64_to_f16(double d) {
    float f = (float)d;
    double back = (double)f;
    if (back != d && d == d) {
        uint32_t u = __float_as_uint(f);
        if (fabs(back) > fabs(d)) u -= 1u;        // step toward zero: truncation
        u |= 1u;                                  // sticky bit
        f = __uint_as_float(u);
    }
    return f32_to_f16(f);
}

// angles_ = f16(prev) + change in the change's dtype (calc_angles, :342-343), then
// .astype(float16) (:351)
__device__ __forceinline__ uint16_t angle_add(uint16_t prev, float ch) {
    return f32_to_f16(f16_to_f32(prev) + ch);
}
__device__ __forceinline__ uint16_t angle_add(uint16_t prev, double ch) {
    return f64_to_f16((double)f16_to_f32(prev) + ch);
}

// ------------------------------------------------------------------ hashing
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
// Three cuckoo candidate slots of a key (low 32 bits of the ID) in a table of n slots.
__device__ __forceinline__ void cuckoo_slots(uint32_t lo, uint32_t n, uint32_t s[NCAND]) {
    // two 32-bit multiplicative mixes; 16-bit fields scaled by 24-bit (full-rate) products
    const uint32_t a = lo ^ (lo >> 16);
    uint32_t h1 = a * 0x9E3779B1u, h2 = (a ^ 0x5BD1E995u) * 0x85EBCA6Bu;
    h1 ^= h1 >> 15;
    h2 ^= h2 >> 13;
    s[0] = __umul24(h1 >> 16, n) >> 16;
    s[1] = __umul24(h1 & 0xFFFFu, n) >> 16;
    s[2] = __umul24(h2 >> 16, n) >> 16;
}

template <int IDB> struct IdT;
template <> struct IdT<4> { typedef uint32_t T; };
template <> struct IdT<8> { typedef uint64_t T; };

template <int IDB>
__device__ __forceinline__ void id_split(typename IdT<IDB>::T id, uint32_t &lo, uint32_t &hi) {
    lo = (uint32_t)id;
    hi = IDB == 8 ? (uint32_t)((uint64_t)id >> 32) : 0u;
}

// ------------------------------------------------------------------ LDS layout
// A work-group barrier that waits for this wave's LDS traffic only: global loads in
// flight stay in flight across it (__syncthreads waits for them too)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

struct ItemHdr {
    int64_t prefix;                 // direct records: the item's first output record
    uint32_t nonuniform, hi0, pad0, overflow;
    uint32_t nh, nseg, n_span, n_pv;
    uint32_t chunk_total, nsl, nstash, npend;
    uint32_t ctr1, pad1, pad2, pad3;    // phase-1 trip counter, walk diagnostics, walk cursor
    uint64_t stash[STASH];          // cuckoo entries whose eviction chain ran out
    uint32_t lstart[HMAX + 1];      // local start of each item halo's current block
    uint32_t vstart[HMAX + 1];      // virtual start of each progenitor segment
    int32_t seg_halo[HMAX];         // segment -> item-local halo
    int32_t halo_cnt[HMAX];         // apsis records per item halo
    uint16_t rowoff[OA_KROWS * (OA_WG / 64)];   // item-local offset of each progenitor
    uint8_t rowcnt[OA_KROWS * (OA_WG / 64)];    //   row's apsis records, and their count;
                                    // phase 1 of a packed item: the halo of each current
                                    // row's first position (rowh)
    uint32_t hslot[HMAX];           // bit 0: joined (non-empty progenitor block);
                                    // bits 1-31: the halo's out_slot + 1 (0: none)
    uint32_t seg_cnt[HMAX];         // progenitor particles of each segment
    int64_t seg_prev_off[HMAX];
    double cb[HMAX][6];             // centre[3], bulk[3]
    float cf[HMAX][6];              // the same, rounded to float32
};
constexpr int64_t HDR_BYTES = (sizeof(ItemHdr) + 255) & ~int64_t(255);

// ------------------------------------------------------------------ direct records
// Decoupled look-back over items (oa_step_args.direct): item b publishes its record
// count as soon as phase 2a knows it, then sums the counts of the items before it back
// to the nearest published inclusive prefix, and publishes its own inclusive prefix.
// A word is one 8-byte granule {epoch, state, value} written by one sc1 store and
// polled with sc1 loads (MI355X_MICROARCH.md, inter-workgroup hand-off R2): no fence.
// An item waits only on lower-numbered items, which publish their counts without
// waiting on anyone, so the chain always resolves; the spin is still bounded (a
// status bit asks the host for a re-run without direct records).
constexpr uint64_t LB_AGG = 1ull << 46, LB_INC = 2ull << 46, LB_VAL = (1ull << 46) - 1ull;
// a poll is one L2 round trip (~1 us): 2^14 polls bound a wait at ~16 ms, ~400x the
// time an item takes; past it the step is re-run without direct records (the engine)
constexpr uint32_t LB_SPIN_MAX = 1u << 14;

__device__ __forceinline__ void lb_publish(uint64_t *w, uint64_t v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_poll(const uint64_t *w) {
    return __hip_atomic_load(const_cast<uint64_t *>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One whole wave: item b's exclusive prefix, summing the counts of the items before it
// back to the nearest published inclusive prefix, LBW words per lane per poll (a window
// of 64 * LBW items: the items of one dispatch round resolve in one round trip), and
// publishes the inclusive one.  `publish_count`: also publish the count first.
constexpr int LBW = 4;
__device__ int64_t item_lookback(const oa_step_args &a, uint32_t b, uint32_t count,
                                 bool publish_count = true) {
    const int lane = threadIdx.x & 63;
    const uint64_t tag = (uint64_t)(uint32_t)a.lb_epoch << 48;
    if (publish_count && lane == 0) lb_publish(&a.lookback[b], tag | LB_AGG | count);
    int64_t excl = 0, j0 = (int64_t)b - 1;
    uint32_t spins = 0;
    const uint32_t spin_max = a.lb_spin_max ? a.lb_spin_max : LB_SPIN_MAX;
    while (j0 >= 0) {
        uint64_t w[LBW];
#pragma unroll
        for (int q = 0; q < LBW; ++q) {
            const int64_t j = j0 - (lane * LBW + q);
            // before item 0: an inclusive prefix of 0
            w[q] = j >= 0 ? lb_poll(&a.lookback[j]) : (tag | LB_INC);
        }
        // this lane's first inclusive word, and whether every word up to it is published
        int qi = LBW;
        bool ready = true;
#pragma unroll
        for (int q = 0; q < LBW; ++q) {
            const bool r = (w[q] >> 48) == (tag >> 48) && (w[q] & (3ull << 46)) != 0ull;
            if (qi == LBW) {
                ready &= r;
                if (r && (w[q] & LB_INC)) qi = q;
            }
        }
        const uint64_t inc = __ballot(qi < LBW);
        const uint64_t notready = __ballot(!ready);
        // lanes 0 .. the nearest inclusive word's lane are needed
        const int f = inc ? __builtin_ctzll(inc) : 64;
        const uint64_t need = f == 64 ? ~0ull : ((2ull << f) - 1ull);
        if (notready & need) {
            if (++spins > spin_max) {
                if (lane == 0) atomicOr(a.status, OA_STATUS_LOOKBACK);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        int64_t v = 0;
#pragma unroll
        for (int q = 0; q < LBW; ++q)
            if (lane < f || (lane == f && q <= qi)) v += (int64_t)(w[q] & LB_VAL);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        excl += v;
        if (f < 64) break;
        j0 -= 64 * LBW;
    }
    {   // uniform (every lane holds the same sum): keep it in SGPRs
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)excl);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)excl >> 32));
        excl = (int64_t)(((uint64_t)hi << 32) | lo);
    }
    if (lane == 0) lb_publish(&a.lookback[b], tag | LB_INC | (uint64_t)(excl + count));
    return excl;
}

#ifndef OA_PENDDIV
#define OA_PENDDIV 9        // deferral list: lds_entries / OA_PENDDIV entries of 8 bytes
#endif
__host__ __device__ inline int64_t table_bytes(int entries, int slots) {
    int64_t b = (int64_t)slots * 8 + (int64_t)entries * 8 / OA_PENDDIV;
    return (b + 15) & ~int64_t(15);
}
// packed items: per progenitor row, segment << 8 | row within the segment (u16), in
// region A past both the table and the staged r̂, so it lives through phases 0-2b
constexpr int64_t PROW_BYTES = ((int64_t)OA_KROWS * (OA_WG / 64) * 2 + 15) & ~int64_t(15);

__device__ __forceinline__ uint32_t upper_find(const uint32_t *starts, uint32_t n, uint32_t x) {
    // largest k in [0, n) with starts[k] <= x  (starts non-decreasing, starts[0] = 0)
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

// ------------------------------------------------------------------ frame
// One snapshot's periodic box as recenter_coordinates (utils.py:24-33) applies it,
// derived on the host (make_wrap).
struct WrapK {
    double box[3];         // L per dimension (float64 values)
    float hi[3];           // smallest float32 with  dx >  L/2  (float32 dx plans)
    float lo[3];           // largest  float32 with  dx < -L/2
    float ab[3];           // min(hi, -lo): |dx| below it never wraps
    int32_t n_dims;        // 0: no periodic wrap
    int32_t f64;           // recenter arithmetic in float64 (wrap_f64)
};
// Per-launch constants derived on the host from oa_step_args (oa_step()).
struct FrameK {
    float h_f;             // RN32(H / (1 + z)): Hubble factor of the f32 sign filter
    WrapK w;               // the current snapshot's box
};

template <typename TD> struct WrapT;
template <> struct WrapT<float> {
    static __device__ __forceinline__ bool hi(float dx, const WrapK &w, int d) { return dx >= w.hi[d]; }
    static __device__ __forceinline__ bool lo(float dx, const WrapK &w, int d) { return dx <= w.lo[d]; }
};
template <> struct WrapT<double> {
    static __device__ __forceinline__ bool hi(double dx, const WrapK &w, int d) { return dx > w.box[d] / 2; }
    static __device__ __forceinline__ bool lo(double dx, const WrapK &w, int d) { return dx < -(w.box[d] / 2); }
};

template <typename TD>
__device__ __forceinline__ TD wrap_sub(TD dx, const WrapK &w, int d) {
    return w.f64 ? (TD)((double)dx - w.box[d]) : (TD)((float)dx - (float)w.box[d]);
}
template <typename TD>
__device__ __forceinline__ TD wrap_add(TD dx, const WrapK &w, int d) {
    return w.f64 ? (TD)((double)dx + w.box[d]) : (TD)((float)dx + (float)w.box[d]);
}

// dx = recenter_coordinates(x - centre) (track_orbits.py:256-259, utils.py:24-33): one
// strict wrap per dimension, in the promoted dtype of (dx, box); the float64 arithmetic
// runs only in waves where some particle crosses the box edge.  cf = the centre rounded
// to float32 (exact for a float32 dx plan).
template <typename TX, typename TD>
__device__ __forceinline__ void centre_dx(const V3<TX> &x, const double *cb, const float *cf,
                                          const WrapK &w, TD dx[3]) {
    if constexpr (sizeof(TD) == 4) {
        dx[0] = (float)x.x - cf[0]; dx[1] = (float)x.y - cf[1]; dx[2] = (float)x.z - cf[2];
    } else {
        dx[0] = (TD)x.x - cb[0]; dx[1] = (TD)x.y - cb[1]; dx[2] = (TD)x.z - cb[2];
    }
    if (w.n_dims > 0) {
        // one wave-level test for the common case (no particle beyond half a box)
        bool m = false;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (d < w.n_dims) {
                if constexpr (sizeof(TD) == 4) m = m | (fabsf(dx[d]) >= w.ab[d]);
                else m = m | WrapT<TD>::hi(dx[d], w, d) | WrapT<TD>::lo(dx[d], w, d);
            }
        }
        if (__any(m)) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                if (d < w.n_dims) {
                    if (WrapT<TD>::hi(dx[d], w, d)) dx[d] = wrap_sub(dx[d], w, d);
                    if (WrapT<TD>::lo(dx[d], w, d)) dx[d] = wrap_add(dx[d], w, d);
                }
            }
        }
    }
}

// rads = sqrt(dot(dx, dx)); r̂ = dx / rads, correctly rounded in TD.
template <typename TD>
__device__ __forceinline__ void unit_vector(const TD dx[3], TD r[3]) {
    if constexpr (std::is_same<TD, float>::value) {
        const float s = dot3(dx[0], dx[1], dx[2], dx[0], dx[1], dx[2]);
        // Fast path for waves whose s lies in [2^-96, 2^100] and whose nonzero
        // components are >= 2^-75 (so rr is normal and every quotient >= 2^-125 is a
        // normal float); any other wave takes sqrtf and the IEEE division.
        //  * rr = RN(sqrt(s)): v_sqrt_f32 (<= 1 ulp) and a residual test on each
        //    neighbour -- the compiler's IEEE expansion without the denormal scaling
        //    and special-value handling, which such an s never needs.
        //  * r̂ = RN(dx / rr) from ONE float64 reciprocal: with y = 1/rr to 2^-52
        //    (v_rcp_f64 + two Newton steps), q = dx * y is within 2^-51 (relative) of
        //    dx / rr, while a quotient of two floats is never closer than 2^-50 to a
        //    float32 rounding midpoint, so rounding q gives RN(dx / rr).
        bool fast = (s >= 0x1p-96f) & (s <= 0x1p100f);
#pragma unroll
        for (int d = 0; d < 3; ++d) fast = fast & ((dx[d] == 0.f) | (fabsf(dx[d]) >= 0x1p-75f));
        if (__all(fast)) {
            const float r0 = __builtin_amdgcn_sqrtf(s);
            const float rm = __uint_as_float(__float_as_uint(r0) - 1u);
            const float rp = __uint_as_float(__float_as_uint(r0) + 1u);
            float rr = __builtin_fmaf(-rm, r0, s) <= 0.f ? rm : r0;
            rr = __builtin_fmaf(-rp, r0, s) > 0.f ? rp : rr;
            const double b = (double)rr;
            double y = __builtin_amdgcn_rcp(b);
            double e = __builtin_fma(-b, y, 1.0);
            y = __builtin_fma(y, e, y);
            e = __builtin_fma(-b, y, 1.0);
            y = __builtin_fma(y, e, y);
#pragma unroll
            for (int d = 0; d < 3; ++d) r[d] = (TD)((double)dx[d] * y);
        } else {
            const float rr = sqrtf(s);
            r[0] = dx[0] / rr; r[1] = dx[1] / rr; r[2] = dx[2] / rr;
        }
    } else {
        const TD rr = sqrt(dot3(dx[0], dx[1], dx[2], dx[0], dx[1], dx[2]));
        r[0] = dx[0] / rr; r[1] = dx[1] / rr; r[2] = dx[2] / rr;
    }
}

// The reference's exact float64 v_r (track_orbits.py:275-288) from r̂ and dx.
template <typename TV, typename TD>
__device__ __forceinline__ double vr_exact(const TD dx[3], const TV vv[3], const double *cb,
                                        const TD r[3], const oa_step_args &a) {
    double w[3];
    for (int d = 0; d < 3; ++d) {
        double vb = a.vb_f64 ? (double)vv[d] - cb[3 + d]
                             : (double)((float)vv[d] - (float)cb[3 + d]);
        w[d] = vb + (a.H * (double)dx[d]) / a.one_plus_z;
    }
    return dot3(w[0], w[1], w[2], (double)r[0], (double)r[1], (double)r[2]);
}

// region_frame (track_orbits.py:247-290) for one particle; cb = centre[3], bulk[3];
// cf = the same six values rounded to float32 (exact for a float32 dx plan).
// r̂ is computed exactly in the dx dtype.  Only sign(v_r) is kept, so v_r is first
// evaluated in float32 with a rigorous error bound (|error| <= ~10 * 2^-24 *
// sum_i |r_i| (|vb_i| + |h_i|)); when |v_r| is within 2^-16 of that scale the wave
// falls back to the reference's float64 expression tree (vr_exact).
template <typename TX, typename TV, typename TD>
__device__ __forceinline__ uint32_t frame(const V3<TX> &x, const V3<TV> &v, const double *cb,
                                          const float *cf, const oa_step_args &a,
                                          const FrameK &k, TD r[3], double *vr_full = nullptr) {
    TD dx[3];
    centre_dx<TX, TD>(x, cb, cf, k.w, dx);
    // rads = sqrt(dot(dx, dx)); rhats = dx / rads   (:286-287), exact in dx's dtype
    unit_vector(dx, r);
    // sign filter: w = (v - bulk) + (H * dx) / (1 + z), v_r = dot(w, r̂)   (:275-288)
    const TV vv[3] = {v.x, v.y, v.z};
    // error scale: sum_i |vb_i| + |h_i| bounds sum_i |r_i| (|vb_i| + |h_i|) since
    // |r_i| <= 1 + 2^-23, and the 2^-16 threshold leaves a margin of 2^4 over the
    // float32 evaluation error
    float wf[3], sc = 0.f;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        float vb = a.vb_f64 ? (float)((double)vv[d] - cb[3 + d]) : (float)vv[d] - cf[3 + d];
        float hf = k.h_f * (float)dx[d];
        wf[d] = vb + hf;
        sc += fabsf(vb) + fabsf(hf);
    }
    const float vrf = (wf[0] * (float)r[0] + wf[1] * (float)r[1]) + wf[2] * (float)r[2];
    const bool sure = fabsf(vrf) > sc * 0x1p-16f;
    uint32_t sgn = vrf > 0.f ? 1u : 2u;
    if (vr_full) {                         // module-level region_frame: the value itself
        const double vr = vr_exact<TV, TD>(dx, vv, cb, r, a);
        *vr_full = vr;
        return vr > 0.0 ? 1u : (vr < 0.0 ? 2u : 0u);
    }
    if (__any(!sure)) {
        if (!sure) {
            const double vr = vr_exact<TV, TD>(dx, vv, cb, r, a);
            sgn = vr > 0.0 ? 1u : (vr < 0.0 ? 2u : 0u);
        }
    }
    return sgn;
}

// region_frame of the on-the-fly driver (track_orbits_onthefly.py:71-120) for one
// particle: dx = recenter(x - c) in the promoted dtype of (x, c, box), stored in the
// coordinate dtype TD (:82-91); w = v - bulk stored in the velocity dtype (:93-110);
// no Hubble term; v_r = dot(w, r̂) in promote(TV, TD) (:112-114), evaluated exactly.
template <typename TX, typename TV, typename TD>
__device__ __forceinline__ uint32_t frame_otf(const V3<TX> &x, const V3<TV> &v, const double *cb,
                                              const oa_step_args &a, const FrameK &k, TD r[3]) {
    const TX xs[3] = {x.x, x.y, x.z};
    TD dx[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        if (a.dx_f64) {
            double t = (double)xs[d] - cb[d];
            if (d < k.w.n_dims) {
                if (t > k.w.box[d] / 2) t = t - k.w.box[d];
                if (t < -(k.w.box[d] / 2)) t = t + k.w.box[d];
            }
            dx[d] = (TD)t;
        } else {
            float t = (float)xs[d] - (float)cb[d];
            if (d < k.w.n_dims) {
                if (t >= k.w.hi[d]) t = wrap_sub(t, k.w, d);
                if (t <= k.w.lo[d]) t = wrap_add(t, k.w, d);
            }
            dx[d] = (TD)t;
        }
    }
    unit_vector(dx, r);
    const TV vs[3] = {v.x, v.y, v.z};
    TV w[3];
#pragma unroll
    for (int d = 0; d < 3; ++d)
        w[d] = a.vb_f64 ? (TV)((double)vs[d] - cb[3 + d]) : (TV)((float)vs[d] - (float)cb[3 + d]);
    if (a.vr_f64) {
        const double vr = dot3((double)w[0], (double)w[1], (double)w[2],
                               (double)r[0], (double)r[1], (double)r[2]);
        return vr > 0.0 ? 1u : (vr < 0.0 ? 2u : 0u);
    }
    const float vr = dot3((float)w[0], (float)w[1], (float)w[2], (float)r[0], (float)r[1], (float)r[2]);
    return vr > 0.f ? 1u : (vr < 0.f ? 2u : 0u);
}

// ------------------------------------------------------------------ step kernel
// LDS image of one item after the ItemHdr (two overlays of region A in time):
//   phases 1-2a  slots[S] u64  3-way cuckoo table of the item's current particles that
//                              have a progenitor block:
//                              lo32(ID) | (sign2 << 16 | (pos+1) << 18) << 32, 0 = empty;
//                pend[E/4] u64 phase 1's deferred inserts (walked before phase 2a)
//   phases 2b-3  rc[3][E] TD   the item's current r̂ as three component arrays (SoA),
//                              staged from the rows phase 1 wrote; after phase 2b reads
//                              rc_x[c] of the matched particle c it overwrites that word
//                              with c's new float16 angle
//   always       sgn[E] u8     sign(v_r) of every current position (bits 0-1) and, from
//                              phase 2a on, bit 2 = matched (the particle has its angle
//                              in rc_x[c]); phase 3 turns it into the state word
// The table side (phase 2a) and the r̂ side (phase 2b) of the join never need LDS at
// the same time, so the current r̂ a previous particle pairs with is read from LDS, not
// gathered from L2: a gathered 12-byte r̂ moves a whole L2 line to the CU, and those
// lines were what bounded phase 2.
constexpr uint32_t POS_BITS = 14, POS_SHIFT = 18, MAX_POS = (1u << POS_BITS) - 2;

__device__ __forceinline__ uint64_t slot_pack(uint32_t lo, uint32_t meta, uint32_t pos) {
    return (uint64_t)lo | ((uint64_t)(meta | ((pos + 1) << POS_SHIFT)) << 32);
}
__device__ __forceinline__ uint32_t slot_pos(uint64_t v) {
    return (uint32_t)(v >> (32 + POS_SHIFT)) - 1u;
}
__device__ __forceinline__ uint32_t slot_meta(uint64_t v) {
    return (uint32_t)(v >> 32) & ((1u << POS_SHIFT) - 1u);
}

// Region A: max(table + deferral list, three r̂ component arrays), 16-B aligned.
__host__ __device__ inline int64_t prow_offset(int entries, int slots, int td_bytes) {
    const int64_t t = table_bytes(entries, slots);
    const int64_t r = ((int64_t)3 * td_bytes * entries + 15) & ~int64_t(15);
    return t > r ? t : r;
}
__host__ __device__ inline int64_t region_a_bytes(int entries, int slots, int td_bytes) {
    return prow_offset(entries, slots, td_bytes) + PROW_BYTES;
}
__host__ __device__ inline int64_t step_lds_bytes(int entries, int slots, int td_bytes) {
    return HDR_BYTES + region_a_bytes(entries, slots, td_bytes) + (((int64_t)entries + 15) & ~int64_t(15));
}

// ---- buffer resources --------------------------------------------------------------
// Row loops address memory through buffer resources built from uniform (SGPR) bases
// with 32-bit per-lane offsets: no 64-bit address arithmetic per access, and lanes past
// a resource's end read 0 / drop their stores, so partial rows need no clamping.
// The LLVM buffer intrinsics are bound directly (v4i32 resource form): this hipcc's
// __builtin_amdgcn_raw_buffer_load_b96 lowers to a 4-byte load, and b128 loads read
// through vector swizzles lose their upper half.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef i32x4 Rsrc;
__device__ int32_t rbl_i32(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ int64_t rbl_i64(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.i64");
__device__ f32x3 rbl_v3f32(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.v3f32");
__device__ f64x2 rbl_v2f64(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.v2f64");
__device__ double rbl_f64(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.f64");
__device__ void rbs_i32(int32_t, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.i32");
__device__ void rbs_v4i32(i32x4, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.v4i32");
__device__ void rbs_v3f32(f32x3, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.v3f32");
__device__ void rbs_v2f64(f64x2, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.v2f64");
__device__ void rbs_f64(double, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.f64");
constexpr int AUX_NT = 2;      // nt: streamed-once inputs and outputs

// raw buffer resource (stride 0): 48-bit base, num_records in bytes, 32-bit data format
__device__ __forceinline__ Rsrc make_rsrc(const void *p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    Rsrc r;
    r.x = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((int32_t)((uint32_t)(a >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int32_t)bytes);
    r.w = 0x00020000;
    return r;
}
template <typename T, int AUX> __device__ __forceinline__ T bld(Rsrc r, uint32_t o) {
    if constexpr (sizeof(T) == 4) return __builtin_bit_cast(T, rbl_i32(r, (int32_t)o, 0, AUX));
    else return __builtin_bit_cast(T, rbl_i64(r, (int32_t)o, 0, AUX));
}
template <typename T, int AUX> __device__ __forceinline__ V3<T> bld3(Rsrc r, uint32_t o) {
    if constexpr (sizeof(T) == 4) {
        const f32x3 v = rbl_v3f32(r, (int32_t)o, 0, AUX);
        return V3<T>{v.x, v.y, v.z};
    } else {
        const f64x2 v = rbl_v2f64(r, (int32_t)o, 0, AUX);
        const double w = rbl_f64(r, (int32_t)(o + 16u), 0, AUX);
        return V3<T>{v.x, v.y, w};
    }
}
template <int AUX> __device__ __forceinline__ void bst32(Rsrc r, uint32_t o, uint32_t v) {
    rbs_i32((int32_t)v, r, (int32_t)o, 0, AUX);
}
constexpr int AUX_R = AUX_NT;       // r̂ stores non-temporal (A/B r03: 1.540-1.548 vs 1.561-1.581 ms)
template <typename T> __device__ __forceinline__ void bst3(Rsrc r, uint32_t o, const T v[3]) {
    if constexpr (sizeof(T) == 4) {
        const f32x3 w = {v[0], v[1], v[2]};
        rbs_v3f32(w, r, (int32_t)o, 0, AUX_R);
    } else {
        const f64x2 w = {v[0], v[1]};
        rbs_v2f64(w, r, (int32_t)o, 0, AUX_R);
        rbs_f64(v[2], r, (int32_t)(o + 16u), 0, AUX_R);
    }
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni64(int64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Phase-2 packed link of one previous particle (a register per row, phases 2a -> 2b):
//   bits 0-13 current position c of the match, bit 14 matched, bit 15 apsis flag,
//   bits 16-31 the previous float16 angle
constexpr uint32_t PK_HIT = 1u << 14, PK_FLAG = 1u << 15;

// SINGLE: every item holds one halo (oa_step_args.items_single): the packed-item paths
// (per-row halo and segment lookups) are compiled out
template <typename TX, typename TV, typename TD, int IDB, bool COMPARE, bool OTF, bool SINGLE = false>
__global__ __launch_bounds__(WG) void k_step(const oa_step_args a, const FrameK fk) {
    typedef typename IdT<IDB>::T ID;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    ItemHdr &H = *reinterpret_cast<ItemHdr *>(smem);
    const uint32_t nslots_max = (uint32_t)a.lds_slots, E = (uint32_t)a.lds_entries;
    uint64_t *slots = reinterpret_cast<uint64_t *>(smem + HDR_BYTES);
    uint64_t *pend = slots + nslots_max;              // phase 1: deferred cuckoo inserts
    const uint32_t pend_cap = E / (uint32_t)OA_PENDDIV;
    TD *rcx = reinterpret_cast<TD *>(smem + HDR_BYTES);   // phases 2b-3 (over the table)
    TD *rcy = rcx + E, *rcz = rcy + E;
    uint8_t *sgn8 = reinterpret_cast<uint8_t *>(
        smem + HDR_BYTES + region_a_bytes((int)E, (int)nslots_max, (int)sizeof(TD)));
    uint16_t *prow = reinterpret_cast<uint16_t *>(
        smem + HDR_BYTES + prow_offset((int)E, (int)nslots_max, (int)sizeof(TD)));

    // the item (host-planned, oa_plan_items): scalar loads, uniform values
    const oa_item it = a.items[blockIdx.x];
    const int nh = SINGLE ? 1 : it.h1 - it.h0;
    const uint32_t nhu = (uint32_t)nh;
    const int64_t base = it.cur_off;
    const uint32_t n_span = (uint32_t)it.n_span, nslots = (uint32_t)it.n_slots;
    // the wave index is uniform: readfirstlane lets every trip / row quantity derived
    // from it live in SGPRs (scalar arithmetic, scalar branches)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const ID *ids = reinterpret_cast<const ID *>(a.ids);
    const ID *ids_prev = reinterpret_cast<const ID *>(a.ids_prev);
    TD *rhat_out = reinterpret_cast<TD *>(a.rhat_out);
    const TD *rhat_prev = reinterpret_cast<const TD *>(a.rhat_prev);
    constexpr uint32_t SX = 3 * sizeof(TX), SV = 3 * sizeof(TV), SD = 3 * sizeof(TD);
    STAMP(0);

    // ---- phase 0: the item's halo table into LDS, the LDS table cleared, the first
    // phase-1 trip in flight -- all overlapped: wave 0 loads the halo rows first, then
    // every wave issues its first trip's loads (a later counted vmcnt for the halo
    // rows leaves them in flight), clears its share of the table, and the only barrier
    // waits for LDS traffic alone.
    oa_halo hrow;
    if (wave == 0 && lane < nh) hrow = a.halos[it.h0 + lane];
    // reference high word for the 32-bit LDS keys: the item's first particle
    uint32_t hi0 = 0u;
    if (IDB == 8 && COMPARE && n_span > 0) hi0 = uni((uint32_t)((uint64_t)ids[base] >> 32));
    __builtin_amdgcn_sched_barrier(0);
    const Rsrc r_id = make_rsrc(ids + base, n_span * IDB);
    const Rsrc r_x = make_rsrc(reinterpret_cast<const TX *>(a.coords) + 3 * base, n_span * SX);
    const Rsrc r_v = make_rsrc(reinterpret_cast<const TV *>(a.vels) + 3 * base, n_span * SV);
    const Rsrc r_rh = make_rsrc(rhat_out + 3 * base, n_span * SD);
    const Rsrc r_mt = make_rsrc(a.meta_out + base, n_span * 4u);
    // Phase-1 rows go in trips of U1 consecutive rows; a wave takes at most NTRIP trips
    // (<= SU rows) and keeps each row's r̂ in registers (rr) until phase 2b writes it
    // into the LDS the table held -- no read-back of the rows it stored.
    constexpr int SU = sizeof(TD) == 4 ? STAGE_F32 : STAGE_F64;
    // float64 r̂ keeps its phase-1 stores (register budget)
    constexpr bool RD = COMPARE && sizeof(TD) == 4;
    // float64 inputs: one row per trip (register budget of 1024-thread work-groups)
    constexpr int U1 = (sizeof(TX) == 8 || sizeof(TV) == 8) ? 1 : UNR1;
    constexpr int NTRIP = SU / U1;
    static_assert(SU % U1 == 0, "rows per wave must be whole trips");
    const uint32_t nrow1 = (n_span + 63) / 64;
    const uint32_t ntr1 = (nrow1 + U1 - 1) / U1;     // trips of U1 consecutive rows
    // the wave's k-th trip: wave, wave + NWAVE, then trips from an LDS counter (read a
    // trip ahead), at most NTRIP of them, so the rows' r̂ fit the wave's registers
    // (float64 inputs, one row per trip: rows dealt statically, wave + NWAVE * k)
    constexpr bool DYN = U1 > 1;
    uint32_t tp[NTRIP];
#pragma unroll
    for (int k = 0; k < NTRIP; ++k) tp[k] = (uint32_t)(wave + NWAVE * k);
    uint32_t ntrips = NTRIP;
#define OA_LOAD1(IDA, XA, VA, T)                                                   \
    _Pragma("unroll") for (int u = 0; u < U1; ++u) {                             \
        const uint32_t li_ = ((T) * U1 + u) * 64 + lane;                           \
        IDA[u] = bld<ID, AUX_NT>(r_id, li_ * IDB);                                 \
        XA[u] = bld3<TX, AUX_NT>(r_x, li_ * SX);                                   \
        VA[u] = bld3<TV, AUX_NT>(r_v, li_ * SV);                                   \
    }
    // one trip of loads in flight ahead of the one computing (two: A/B r02 neutral)
    ID idv[U1], idn[U1];
    V3<TX> xv[U1], xn[U1];
    V3<TV> vv[U1], vn[U1];
    V3<TD> rr[SU];
    OA_LOAD1(idv, xv, vv, tp[0])
    __builtin_amdgcn_sched_barrier(0);
    if (COMPARE) {
        for (uint32_t w = tid; w < nslots; w += WG) slots[w] = 0ull;
        // early walks read appended entries: an unwritten one is still 0
        for (uint32_t w = tid; w < pend_cap; w += WG) pend[w] = 0ull;
    }
    if (wave == 0) {
        // progenitor segments: every halo with a non-empty progenitor block, in halo
        // order, each starting on a 64-position row of the padded progenitor space
        // (lane scans over the item's <= HMAX halos)
        const bool in = lane < nh;
        const bool hp = COMPARE && in && hrow.prev_cnt > 0;
        const uint32_t pv = hp ? (((uint32_t)hrow.prev_cnt + 63u) & ~63u) : 0u;
        uint32_t vi = pv, si = hp ? 1u : 0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(vi, o), z = __shfl_up(si, o);
            if (lane >= o) { vi += y; si += z; }
        }
        if (in) {
            H.lstart[lane] = (uint32_t)(hrow.cur_off - base);
            // joined halos: those with a non-empty progenitor block (an empty one
            // matches nothing: its particles keep angle 0)
            // with the output slot, so the item's end needs no reload of the halo row
            H.hslot[lane] = ((uint32_t)(hrow.out_slot + 1) << 1) | (hp ? 1u : 0u);
            H.halo_cnt[lane] = 0;
            for (int d = 0; d < 3; ++d) { H.cb[lane][d] = hrow.centre[d]; H.cb[lane][3 + d] = hrow.bulk[d]; }
            for (int d = 0; d < 3; ++d) { H.cf[lane][d] = (float)hrow.centre[d]; H.cf[lane][3 + d] = (float)hrow.bulk[d]; }
            if (hp) {
                const uint32_t sg = si - 1u;
                H.seg_halo[sg] = lane; H.seg_prev_off[sg] = hrow.prev_off;
                H.vstart[sg] = vi - pv; H.seg_cnt[sg] = (uint32_t)hrow.prev_cnt;
            }
        }
        const uint32_t n_pv = (uint32_t)__shfl(vi, 63), nseg = (uint32_t)__shfl(si, 63);
        if (!SINGLE && nh > 1) {
            // per-row tables, so no row searches the halo or segment starts later: the
            // halo of each current row's first position, and each progenitor row's
            // segment and row within it (a lane per halo, its own rows)
            const uint32_t c0 = in ? (uint32_t)(hrow.cur_off - base) : n_span;
            uint32_t c1 = __shfl_down(c0, 1);
            if (lane == nh - 1) c1 = n_span;
            constexpr uint32_t NR = (uint32_t)(KROWS * NWAVE);
            if (in)
                for (uint32_t r = (c0 + 63u) >> 6; (r << 6) < c1 && r < NR; ++r) H.rowcnt[r] = (uint8_t)lane;
            if (hp) {
                const uint32_t r0 = (vi - pv) >> 6, sg = si - 1u;
                for (uint32_t r = 0; r < (pv >> 6) && r0 + r < NR; ++r) prow[r0 + r] = (uint16_t)((sg << 8) | r);
            }
        }
        if (lane == 0) {
            H.lstart[nh] = n_span;
            H.vstart[nseg] = n_pv; H.nseg = nseg; H.n_pv = n_pv;
            H.nonuniform = 0; H.overflow = 0; H.chunk_total = 0; H.nstash = 0; H.npend = 0;
            H.pad1 = 0; H.pad2 = 0;
            H.ctr1 = 2 * NWAVE;             // phase 1: the first two trips of every wave are static
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    STAMP(1);

    // ---- phase 1: frame of every current particle, LDS insert ---------------
    // software-pipelined: trip t+1's loads are in flight while trip t computes
#pragma unroll
    for (int kp = 0; kp < NTRIP; ++kp) {
        if (tp[kp] >= ntr1) { ntrips = kp; break; }         // trip numbers only grow
        const uint32_t tcur = DYN ? tp[kp] : (uint32_t)(wave + NWAVE * kp);
        uint32_t f = 0;
        if (DYN && kp + 2 < NTRIP && lane == 0) f = atomicAdd(&H.ctr1, 1u);   // trip kp + 2
        if (kp + 1 < NTRIP) OA_LOAD1(idn, xn, vn, (DYN ? tp[(kp + 1) % NTRIP] : (uint32_t)(wave + NWAVE * (kp + 1))))
        uint64_t val[U1];
        uint32_t csu[U1][NCAND];
        bool ins[U1];
#pragma unroll
        for (int u = 0; u < U1; ++u) {
            ins[u] = false;
            const uint32_t r0 = (tcur * U1 + u) * 64;        // uniform
            if (r0 >= n_span) continue;
            const uint32_t li = r0 + lane;
            const bool ok = li < n_span;
            // the row's halo (uniform search); rows that cross into later halos of a
            // packed item step each lane forward
            uint32_t hl = 0;
            if (!SINGLE && nhu > 1) {
                hl = uni((uint32_t)H.rowcnt[r0 >> 6]);               // rowh (phase 0)
                if (r0 + 63u >= H.lstart[hl + 1])
                    while (hl + 1 < nhu && li >= H.lstart[hl + 1]) ++hl;
            }
            TD r[3];
            uint32_t sgn;
            if (!COMPARE && !OTF && a.vr_out) {
                double vr;
                sgn = frame<TX, TV, TD>(xv[u], vv[u], H.cb[hl], H.cf[hl], a, fk, r, &vr);
                if (ok) a.vr_out[base + li] = vr;
            } else {
                sgn = OTF ? frame_otf<TX, TV, TD>(xv[u], vv[u], H.cb[hl], a, fk, r)
                          : frame<TX, TV, TD>(xv[u], vv[u], H.cb[hl], H.cf[hl], a, fk, r);
            }
            // compare steps store r̂ from registers in phase 2b (RDEFER): phase 1 then
            // issues loads only and ends without waiting on stores
            if (!RD) bst3<TD>(r_rh, li * SD, r);
            rr[kp * U1 + u] = V3<TD>{r[0], r[1], r[2]};
            if constexpr (!COMPARE) {
                uint32_t ang = 0;
                if (a.angles_in && ok) ang = a.angles_in[base + li];
                bst32<AUX_NT>(r_mt, li * 4u, ang | (sgn << 16));
                continue;
            } else {
                // every state word is written by phase 3, from this sign
                if (ok) sgn8[li] = (uint8_t)sgn;
                if (!ok || !(H.hslot[hl] & 1u)) continue;
                uint32_t lo, hi;
                id_split<IDB>(idv[u], lo, hi);
                if (IDB == 8 && hi != hi0) H.nonuniform = 1u;     // benign race: all write 1
                val[u] = slot_pack(lo, sgn << 16, li);
                cuckoo_slots(lo, nslots, csu[u]);
                ins[u] = true;
            }
        }
        if (COMPARE) {
            // first try: claim an EMPTY candidate with a CAS (at load <= 1/2 one of the
            // three almost always is), so eviction chains stay rare
            uint64_t cv[U1][NCAND];
#pragma unroll
            for (int u = 0; u < U1; ++u)
                if (ins[u]) {
#pragma unroll
                    for (int j = 0; j < NCAND; ++j) cv[u][j] = slots[csu[u][j]];
                }
#pragma unroll
            for (int u = 0; u < U1; ++u) {
                if (!ins[u]) continue;
                uint32_t t = 0xFFFFFFFFu;
#pragma unroll
                for (int j = NCAND - 1; j >= 0; --j) t = cv[u][j] == 0ull ? csu[u][j] : t;
                if (t == 0xFFFFFFFFu) continue;
                const uint64_t o = atomicCAS(reinterpret_cast<unsigned long long *>(&slots[t]),
                                             0ull, (unsigned long long)val[u]);
                if (o == 0ull) ins[u] = false;
            }
            // an entry whose three candidates are taken is deferred: the walks run after
            // the loop, spread over the whole work-group
#pragma unroll
            for (int u = 0; u < U1; ++u) {
                if (!ins[u]) continue;
                const uint32_t e = atomicAdd(&H.npend, 1u);
                if (e < pend_cap) pend[e] = val[u];
                else H.overflow = 2u;
            }
        }
#pragma unroll
        for (int u = 0; u < U1; ++u) {
            idv[u] = idn[u]; xv[u] = xn[u]; vv[u] = vn[u];
        }
        if (DYN && kp + 2 < NTRIP) tp[(kp + 2) % NTRIP] = __builtin_amdgcn_readfirstlane(f);
    }
#undef OA_LOAD1
    WSTAMP(0);
    STAMP(8);
    if constexpr (!COMPARE) return;

    // ---- phase 2: the join, in two halves -------------------------------------
    // Rows are 64 virtual positions; progenitor segment s occupies
    // [vstart[s], vstart[s] + seg_cnt[s]) and starts on a row, so a row lies in one
    // segment: its halo, block offset and resources are uniform.  Rows are dealt
    // statically: wave w takes rows w, w + NWAVE, ... (<= KROWS of them, the host
    // planner caps n_pv), and keeps each row's IDs and packed link in registers from
    // phase 2a to phase 2b.
    const uint32_t n_pv = uni(H.n_pv), nseg = SINGLE ? min(uni(H.nseg), 1u) : uni(H.nseg);
    const uint32_t nrow = (n_pv + 63) / 64;
    // r̂ of every row this wave computed, from registers (RDEFER); rows past the
    // item fall outside r_rh and are dropped
    auto store_rhat = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < SU; ++k) {
            if (DYN && (uint32_t)(k / U1) >= ntrips) break;
            const uint32_t li = DYN ? (tp[k / U1] * U1 + k % U1) * 64 + lane
                                    : (uint32_t)(wave + NWAVE * k) * 64 + lane;
            const TD w[3] = {rr[k].x, rr[k].y, rr[k].z};
            bst3<TD>(r_rh, li * SD, w);
        }
    };
    // direct records (oa_step_args.direct), wave 0 at the item's end: every halo of the
    // item with an output slot gets its offset (the item's prefix + the records of its
    // earlier halos, in halo order = slot order), and the last item writes the total
    auto direct_tail = [&](int64_t P, uint32_t total) __attribute__((always_inline)) {
        const int32_t c = lane < nh ? H.halo_cnt[lane] : 0;
        int32_t incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const uint32_t os = lane < nh ? H.hslot[lane] >> 1 : 0u;
        if (os) a.offsets_out[os - 1u] = P + (incl - c);
        if (lane == 0 && blockIdx.x == gridDim.x - 1) {
            a.offsets_out[a.n_slots] = P + total;
            *a.total_out = P + total;
        }
    };
    if (n_pv == 0) {                                 // nothing to join: state words only
        if (RD) store_rhat();
        __syncthreads();
        for (uint32_t li = tid; li < n_span; li += WG)
            bst32<AUX_NT>(r_mt, li * 4u, (uint32_t)(sgn8[li] & 3u) << 16);
        if (tid == 0) a.item_count[blockIdx.x] = 0;
        if (a.direct && wave == 0) direct_tail(item_lookback(a, blockIdx.x, 0u), 0u);
        return;
    }
    const uint32_t cnt0 = uni(H.seg_cnt[0]), hal0 = uni((uint32_t)H.seg_halo[0]);
    const int64_t off0 = uni64(H.seg_prev_off[0]);
    // a row's segment data: valid lanes nv, item-local halo hs, first previous index kb
    auto row_of = [&](uint32_t r, uint32_t &nv, uint32_t &hs, int64_t &kb) __attribute__((always_inline)) {
        const uint32_t r0 = r * 64u;
        uint32_t ro = r0, cnt = cnt0;
        hs = hal0;
        int64_t off = off0;
        if (nseg > 1) {
            // the row's segment from the phase-0 table (rows past the item: none)
            const uint32_t e = r < nrow ? uni((uint32_t)prow[r]) : 0u, s = e >> 8;
            ro = r < nrow ? (e & 0xFFu) * 64u : cnt0;
            cnt = uni(H.seg_cnt[s]);
            hs = uni((uint32_t)H.seg_halo[s]);
            off = uni64(H.seg_prev_off[s]);
        }
        nv = (r < nrow && ro < cnt) ? min(cnt - ro, 64u) : 0u;
        kb = off + ro;
    };
    // Every row's 2a loads (IDs, state words) go out before the walks and the barrier:
    // up to 2 * KROWS loads in flight per wave hide the HBM latency behind them.
    ID pid[KROWS];
    uint32_t pk[KROWS];
    V3<TD> prh[KROWS];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < KROWS; ++k) {
        pid[k] = 0;
        pk[k] = 0u;
        uint32_t nv, hs;
        int64_t kb;
        row_of(wave + NWAVE * k, nv, hs, kb);
        pid[k] = bld<ID, AUX_NT>(make_rsrc(ids_prev + kb, nv * IDB), lane * IDB);
        pk[k] = bld<uint32_t, AUX_NT>(make_rsrc(a.meta_prev + kb, nv * 4u), lane * 4u);
    }
    __builtin_amdgcn_sched_barrier(0);
    // one deferred insert's eviction walk (atomic exchanges: safe beside the first-try
    // CAS inserts of waves still in phase 1, and beside other walks)
    auto walk = [&](uint64_t v) __attribute__((always_inline)) {
        uint32_t cs[NCAND];
        cuckoo_slots((uint32_t)v, nslots, cs);
        uint32_t t = cs[0];
        for (int it_ = 0;; ++it_) {
            const uint64_t old = atomicExch(reinterpret_cast<unsigned long long *>(&slots[t]),
                                            (unsigned long long)v);
            if (old == 0ull) {
                if (OA_STAMPS) atomicMax(&H.pad1, (uint32_t)it_ + 1u);
                break;
            }
            if (it_ == MAX_EVICT) {
                if (OA_STAMPS) atomicMax(&H.pad1, 1000u);
                const uint32_t k = atomicAdd(&H.nstash, 1u);
                if (k < (uint32_t)STASH) H.stash[k] = old;
                else H.overflow = 2u;
                break;
            }
            cuckoo_slots((uint32_t)old, nslots, cs);
            // the displaced key moves to its candidate after the one it held
            uint32_t nx = cs[0];
#pragma unroll
            for (int j = NCAND - 2; j >= 0; --j) nx = cs[j] == t ? cs[j + 1] : nx;
            t = nx;
            v = old;
        }
    };
    {
        // a wave done with phase 1 walks the deferred inserts appended so far, claimed
        // in runs of 64 from a cursor, while later waves still stream; the barrier
        // below leaves the rest to the whole work-group
        volatile uint32_t *vnp = &H.npend, *vcur = &H.pad2;
        volatile uint64_t *vpend = pend;
        for (;;) {
            uint32_t c = 0, c2 = 0;
            if (lane == 0) {
                const uint32_t n = min(*vnp, pend_cap);
                c = *vcur;
                while (c < n) {
                    const uint32_t want = min(c + 64u, n);
                    const uint32_t old = atomicCAS(&H.pad2, c, want);
                    if (old == c) { c2 = want; break; }
                    c = old;
                }
            }
            c = __builtin_amdgcn_readlane(c, 0);
            c2 = __builtin_amdgcn_readlane(c2, 0);
            if (c2 <= c) break;
            const uint32_t e = c + (uint32_t)lane;
            if (e < c2) {
                uint64_t v;
                do { v = vpend[e]; } while (v == 0ull);     // reserved, not yet written
                walk(v);
            }
        }
    }
    // barrier on LDS traffic only: the loads above and phase 1's r̂ stores stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    STAMP(2);
    {
        const uint32_t np = min(H.npend, pend_cap);
        for (uint32_t e = H.pad2 + tid; e < np; e += WG) walk(pend[e]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    STAMP(3);
    DIAG((uint64_t)H.npend | ((uint64_t)H.pad1 << 20) | ((uint64_t)H.nstash << 40));
    if (H.overflow || nrow > (uint32_t)(KROWS * NWAVE)) {
        // the host re-plans this snapshot; the compaction that follows must see no
        // records from this item
        if (tid == 0) {
            atomicOr(a.status, H.overflow ? OA_STATUS_TABLE_OVERFLOW : OA_STATUS_PLAN);
            a.item_count[blockIdx.x] = 0;
        }
        // the later items' look-backs must still resolve (the step is re-run anyway)
        if (a.direct && wave == 0) item_lookback(a, blockIdx.x, 0u);
        return;
    }
    const bool nonuniform = IDB == 8 && uni(H.nonuniform) != 0;
    const uint32_t nstash = min(uni(H.nstash), (uint32_t)STASH);

    // ---- phase 2a: cuckoo lookup of every previous particle -----------------
    // Three candidate slots read together (one LDS round trip), the match selected
    // without branches; departed particles miss (setdiff1d / in1d, :300-304).  The
    // halo's position range tells copies of one ID in overlapping regions apart and
    // rejects empty slots.  The strict sign test (:311-314) needs only the two sign
    // fields, so the apsis flag is decided here.
#pragma unroll
    for (int k = 0; k < KROWS; ++k) {
        const uint32_t r = wave + NWAVE * k;
        uint32_t nv, hs;
        int64_t kb;
        row_of(r, nv, hs, kb);
        const uint32_t pmeta = pk[k];
        uint32_t lo, hi;
        id_split<IDB>(pid[k], lo, hi);
        const bool can = ((uint32_t)lane < nv) & (IDB != 8 || nonuniform || hi == hi0);
        uint32_t lmin = 0, lmax = n_span;                 // the halo's position span
        if (!SINGLE && nhu > 1) {
            lmin = uni(H.lstart[hs]);
            lmax = uni(H.lstart[hs + 1]) - lmin;
        }
        uint32_t cs[NCAND];
        cuckoo_slots(lo, nslots, cs);
        uint64_t cv[NCAND];
#pragma unroll
        for (int j = 0; j < NCAND; ++j) cv[j] = slots[cs[j]];
        auto m = [&](uint64_t v) { return ((uint32_t)v == lo) & (slot_pos(v) - lmin < lmax); };
        uint64_t hit = 0ull;
        if (IDB == 8 && nonuniform) {
            // rare: candidates whose low word matches are confirmed on the full ID
#pragma unroll
            for (int j = 0; j < NCAND; ++j)
                if (!hit && can && m(cv[j]) && ids[base + slot_pos(cv[j])] == pid[k]) hit = cv[j];
        } else {
            // (halo, low word) is unique in an item whose IDs share their high word
#pragma unroll
            for (int j = NCAND - 1; j >= 0; --j) hit = (can && m(cv[j])) ? cv[j] : hit;
        }
        if (nstash && can && !hit) {
            for (uint32_t e = 0; e < nstash; ++e) {
                const uint64_t v = H.stash[e];
                if (m(v) && (!(IDB == 8 && nonuniform) || ids[base + slot_pos(v)] == pid[k])) {
                    hit = v;
                    break;
                }
            }
        }
        uint32_t p = 0;
        if (hit) {
            const uint32_t c = slot_pos(hit), sc = slot_meta(hit) >> 16, sp = pmeta >> 16;
            const bool cond = a.mode == OA_MODE_PERICENTRIC ? (sp == 2u && sc == 1u)
                                                            : (sp == 1u && sc == 2u);
            p = c | PK_HIT | (cond ? PK_FLAG : 0u) | (pmeta << 16);
            sgn8[c] = (uint8_t)(sc | 4u);
        }
        pk[k] = p;
        // records per row: the apsis flags are known here, so phase 2b writes each
        // item's records contiguously (item-local offsets scanned below)
        const uint32_t fc = (uint32_t)__popcll(__ballot((p & PK_FLAG) != 0u));
        if (lane == 0 && r < nrow) H.rowcnt[r] = (uint8_t)fc;
        if (OTF && r < nrow && (uint32_t)lane < nv) a.matched_prev[kb + lane] = hit ? 1 : 0;
    }
    WSTAMP(1);
    STAMP(4);

    // ---- phase 2b: angles from the current r̂ staged in LDS, apsis records ------
    // The first PF2 rows' previous r̂ loads go out before the barrier (their HBM
    // latency behind the staging), which waits for LDS traffic only.
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < PF2 && k < KROWS; ++k) {
        uint32_t nv, hs;
        int64_t kb;
        row_of(wave + NWAVE * k, nv, hs, kb);
        prh[k] = bld3<TD, AUX_NT>(make_rsrc(rhat_prev + 3 * kb, nv * SD), lane * SD);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();          // every lookup done: the table is dead
    __builtin_amdgcn_sched_barrier(0);
    if (wave == 0) {
        // item-local record offsets of the rows (exclusive scan, <= KROWS * NWAVE rows)
        uint32_t carry = 0;
        for (uint32_t c0 = 0; c0 < nrow; c0 += 64) {
            const uint32_t r = c0 + lane;
            const uint32_t v = r < nrow ? (uint32_t)H.rowcnt[r] : 0u;
            uint32_t incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (r < nrow) H.rowoff[r] = (uint16_t)(carry + incl - v);
            carry += (uint32_t)__shfl(incl, 63);
        }
        if (lane == 0) H.chunk_total = carry;
        // direct records: the item's count is published now; its prefix is resolved
        // after phase 2b, beside phase 3, and the records are stored after that
        if (a.direct && lane == 0)
            lb_publish(&a.lookback[blockIdx.x],
                       ((uint64_t)(uint32_t)a.lb_epoch << 48) | LB_AGG | carry);
    }
    // the item's current r̂, from the registers phase 1 left it in
#pragma unroll
    for (int k = 0; k < SU; ++k) {
        if (DYN && (uint32_t)(k / U1) >= ntrips) break;
        const uint32_t li = DYN ? (tp[k / U1] * U1 + k % U1) * 64 + lane
                                : (uint32_t)(wave + NWAVE * k) * 64 + lane;
        if (li < n_span) { rcx[li] = rr[k].x; rcy[li] = rr[k].y; rcz[li] = rr[k].z; }
    }
    if (RD) store_rhat();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    STAMP(5);

    const uint64_t lanemask_lt = (1ull << lane) - 1ull;
    // records go to the item's scratch range now, or (direct) from registers to the
    // output once the item's prefix is known (after phase 3)
    const bool direct = a.direct != 0;
    ID *scr_ids = reinterpret_cast<ID *>(a.scratch_ids);
    uint32_t *rcw = reinterpret_cast<uint32_t *>(rcx);        // new angles over rc_x
    constexpr uint32_t RCW = sizeof(TD) / 4;
#pragma unroll
    for (int k = 0; k < KROWS; ++k) {
        if (k + PF2 < KROWS) {
            uint32_t nv, hs;
            int64_t kb;
            row_of(wave + NWAVE * (k + PF2), nv, hs, kb);
            prh[k + PF2] = bld3<TD, AUX_NT>(make_rsrc(rhat_prev + 3 * kb, nv * SD), lane * SD);
        }
        const uint32_t r = wave + NWAVE * k;
        if (r >= nrow) continue;
        uint32_t nv, hs;
        int64_t kb;
        row_of(r, nv, hs, kb);
        const uint32_t p = pk[k];
        bool flag = false;
        uint16_t a16 = 0;
        if (p & PK_HIT) {
            const uint32_t c = p & (PK_HIT - 1u);
            // angle change = arccos(dot(r̂_prev, r̂_match)), no clamp (:324-325)
            const TD dt = dot3(prh[k].x, prh[k].y, prh[k].z, rcx[c], rcy[c], rcz[c]);
            const TD change = acos_change<OTF>(dt);
            // calc_angles (:342-349): f16 + change, rounded once; reset at an apsis
            const uint16_t acc = angle_add((uint16_t)(p >> 16), change);
            flag = (p & PK_FLAG) != 0u;
            a16 = acc;
            rcw[RCW * c] = flag ? 0u : (uint32_t)acc;
            if (OTF) {
                // on-the-fly outputs (track_orbits_onthefly.py:145-174): the angle
                // change of every matched particle, and which current ones matched
                static_cast<TD *>(a.angle_out)[kb + lane] = change;
                a.matched_cur[base + c] = 1;
            }
        }
        // apsis records in previous-block order (:315-316): wave ballot + prefix
        // popcount place each row's records at the row's item-local offset, so an
        // item's records are contiguous and in order (k_gather_items copies them)
        const uint64_t mk = __ballot(flag);
        const uint32_t cnt = (uint32_t)__popcll(mk);
        if (direct) {
            if (p & PK_HIT) pk[k] = (p & 0xFFFFu) | ((uint32_t)a16 << 16);   // kept for later
        } else if (flag) {
            const int64_t sb = it.scratch_off + uni(H.rowoff[r]);
            const uint32_t q = (uint32_t)__popcll(mk & lanemask_lt);
            __builtin_nontemporal_store(pid[k], &scr_ids[sb + q]);
            __builtin_nontemporal_store(a16, &a.scratch_ang[sb + q]);
            if (a.scratch_pos) a.scratch_pos[sb + q] = (int32_t)(kb + lane);
        }
        if (lane == 0 && cnt) atomicAdd(&H.halo_cnt[hs], (int)cnt);
    }
    WSTAMP(2);
    STAMP(6);
    // phase 3 reads LDS alone: the records' global stores stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    // ---- phase 3: every state word of the item, in position order ---------------
    // matched: the new angle phase 2b left in rc_x; entered or in a halo without a
    // progenitor block: angle 0 (calc_angles :348-349).  Nothing in this launch reads
    // them again, so the stores are non-temporal.
    // (four consecutive positions per thread: one 16-byte store)
    // direct records: wave 0 resolves the item's prefix meanwhile (the look-back's
    // round trips overlap the other waves' stores)
    if (direct && wave == 0) {
        const int64_t P = item_lookback(a, blockIdx.x, uni(H.chunk_total), false);
        if (lane == 0) H.prefix = P;
    }
    const uint32_t t3 = direct ? (uint32_t)tid - 64u : (uint32_t)tid;
    const uint32_t nt3 = direct ? (uint32_t)(WG - 64) : (uint32_t)WG;
    const uint32_t n4 = (direct && wave == 0) ? 0u : n_span & ~3u;
    for (uint32_t l4 = t3 * 4u; l4 < n4; l4 += nt3 * 4u) {
        const uint32_t s4 = *reinterpret_cast<const uint32_t *>(sgn8 + l4);
        i32x4 w;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t sq = (s4 >> (8 * q)) & 0xFFu;
            const uint32_t ang = (sq & 4u) ? (rcw[RCW * (l4 + q)] & 0xFFFFu) : 0u;
            w[q] = (int32_t)(ang | ((sq & 3u) << 16));
        }
        rbs_v4i32(w, r_mt, (int32_t)(l4 * 4u), 0, AUX_NT);
    }
    for (uint32_t li = (n_span & ~3u) + t3; li < n_span && !(direct && wave == 0); li += nt3) {
        const uint32_t s = sgn8[li];
        const uint32_t ang = (s & 4u) ? (rcw[RCW * li] & 0xFFFFu) : 0u;
        bst32<AUX_NT>(r_mt, li * 4u, ang | ((s & 3u) << 16));
    }
    if (direct) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();             // H.prefix
        __builtin_amdgcn_sched_barrier(0);
        const int64_t rec0 = uni64(H.prefix);
        ID *out_ids = reinterpret_cast<ID *>(a.out_ids);
#pragma unroll
        for (int k = 0; k < KROWS; ++k) {
            const uint32_t r = wave + NWAVE * k;
            if (r >= nrow) continue;
            uint32_t nv, hs;
            int64_t kb;
            row_of(r, nv, hs, kb);
            const uint32_t p = pk[k];
            const bool flag = (p & (PK_HIT | PK_FLAG)) == (PK_HIT | PK_FLAG);
            const uint64_t mk = __ballot(flag);
            if (flag) {
                const int64_t sb = rec0 + uni(H.rowoff[r]) + __popcll(mk & lanemask_lt);
                __builtin_nontemporal_store(pid[k], &out_ids[sb]);
                __builtin_nontemporal_store((uint16_t)(p >> 16), &a.out_ang[sb]);
                if (a.out_pos) a.out_pos[sb] = (int32_t)(kb + lane);
            }
        }
        if (wave == 0) direct_tail(rec0, uni(H.chunk_total));
    } else if (tid < nh) {
        const uint32_t os = H.hslot[tid] >> 1;
        if (os) a.halo_count[os - 1u] = H.halo_cnt[tid];
    }
    if (tid == 0) a.item_count[blockIdx.x] = (int32_t)H.chunk_total;
    STAMP(7);
}

// ------------------------------------------------------------------ compaction
// previous-block positions per record chunk of a partitioned halo (k_part_join's RCHUNK)
constexpr int RCHUNK_GATHER = 4096;
__global__ __launch_bounds__(1024) void k_scan_slots(const int32_t *cnt, int32_t n,
                                                     int64_t *off, int64_t *total) {
    // exclusive scan of the per-halo record counts (one work-group).  Thread t owns the
    // contiguous run [t*c, t*c + c): its loads are independent and go out together (a
    // blocked scan has no serial chain of global loads), the run totals are scanned
    // across the work-group, and the second read of the run hits the cache.
    __shared__ int64_t wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c = (n + 1023) / 1024;
    const int s0 = min(n, tid * c), s1 = min(n, s0 + c);
    int64_t tot = 0;
#pragma unroll 8
    for (int i = s0; i < s1; ++i) tot += cnt[i];
    int64_t incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int64_t run = incl - tot;
    for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll 8
    for (int i = s0; i < s1; ++i) { off[i] = run; run += cnt[i]; }
    if (tid == 1023) { off[n] = run; *total = run; }
}

// Packed (k_step) items hold their records contiguously: a coalesced copy.  Global
// items of the global-table path (k_big_join) keep theirs in 64-position segments,
// packed at each segment's base: segments in chunks of 256 get a block-wide exclusive scan of their
// record counts (LDS), then the chunk's records are copied flat -- thread t moves
// records t, t + 256, ... (consecutive records of consecutive rows: coalesced), each
// finding its row by a binary search over the scanned offsets.
template <int IDB>
__device__ __forceinline__ void gather_segments(const oa_compact_args &a, const oa_item &it,
                                                int64_t dst, int64_t s_lo, int64_t s_hi,
                                                uint32_t *wsum, uint32_t *roff) {
    typedef typename IdT<IDB>::T ID;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const ID *src = reinterpret_cast<const ID *>(a.scratch_ids);
    ID *out = reinterpret_cast<ID *>(a.out_ids) + dst;
    uint16_t *oang = a.out_ang + dst;
    const uint8_t *sc = a.seg_count + (it.scratch_off >> 6);
    int64_t carry = 0;
    for (int64_t c0 = s_lo; c0 < s_hi; c0 += 256) {
        const int64_t sg = c0 + tid;
        const uint32_t cnt = sg < s_hi ? sc[sg] : 0u;
        uint32_t incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < 4; ++w) { if (w < wave) pre += wsum[w]; tot += wsum[w]; }
        roff[tid] = pre + incl - cnt;
        if (tid == 255) roff[256] = tot;
        __syncthreads();
        const uint32_t rows = (uint32_t)(s_hi - c0 < 256 ? s_hi - c0 : 256);
        for (uint32_t j = tid; j < tot; j += 256) {
            const uint32_t r = upper_find(roff, rows, j);      // roff[r] <= j < roff[r + 1]
            const int64_t from = it.scratch_off + ((c0 + r) << 6) + (j - roff[r]);
            out[carry + j] = src[from];
            oang[carry + j] = a.scratch_ang[from];
            if (a.out_pos) a.out_pos[dst + carry + j] = a.scratch_pos[from];
        }
        carry += tot;
        __syncthreads();
    }
}

template <int IDB>
__global__ __launch_bounds__(256) void k_gather_items(const oa_compact_args a) {
    typedef typename IdT<IDB>::T ID;
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t roff[257];
    const oa_item it = a.items[blockIdx.x];
    // an item holds at most one record per (padded) progenitor position
    const int32_t n = min((int64_t)a.item_count[blockIdx.x], it.n_pv);
    const int64_t slot = it.slot0;               // planned on the host: no halo walk
    if (n <= 0 || slot < 0) return;
    const int tid = threadIdx.x;
    const int64_t dst = a.offsets_out[slot];
    if ((int32_t)blockIdx.x < a.n_packed) {
        // k_step items: the records are already contiguous and in order
        const ID *src = reinterpret_cast<const ID *>(a.scratch_ids);
        ID *out = reinterpret_cast<ID *>(a.out_ids) + dst;
        uint16_t *oang = a.out_ang + dst;
        const int64_t s0 = it.scratch_off;
        for (int32_t j = tid; j < n; j += 256) {
            out[j] = src[s0 + j];
            oang[j] = a.scratch_ang[s0 + j];
            if (a.out_pos) a.out_pos[dst + j] = a.scratch_pos[s0 + j];
        }
        return;
    }
    if (a.gchunks) return;                       // k_gather_chunks moves these
    gather_segments<IDB>(a, it, dst, 0, (it.n_pv + 63) >> 6, wsum, roff);
}

// Global items, one work-group per previous-block chunk (gchunks rows: item, start,
// count; start a multiple of 64): the chunk's output offset is the item's plus the
// records of the item's segments before it (a block reduction over those segment
// counts, L2 hits), then its own segments as above.  A large halo's records move with
// as many work-groups as it has chunks instead of one.
template <int IDB>
__global__ __launch_bounds__(256) void k_gather_chunks(const oa_compact_args a) {
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t roff[257];
    __shared__ uint32_t red[4];
    const int64_t *ch = a.gchunks + 3 * (int64_t)blockIdx.x;
    const int64_t gi = ch[0], start = ch[1], cnt = ch[2];
    const oa_item it = a.items[gi];
    const int64_t slot = it.slot0;
    if (slot < 0 || a.item_count[gi] <= 0 || cnt <= 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t s_lo = start >> 6, s_hi = (start + cnt + 63) >> 6;
    const uint8_t *sc = a.seg_count + (it.scratch_off >> 6);
    uint32_t before = 0;
    for (int64_t sg = tid; sg < s_lo; sg += 256) before += sc[sg];
    for (int o = 32; o > 0; o >>= 1) before += __shfl_down(before, o);
    if (lane == 0) red[wave] = before;
    __syncthreads();
    const int64_t dst = a.offsets_out[slot] + (int64_t)(red[0] + red[1] + red[2] + red[3]);
    gather_segments<IDB>(a, it, dst, s_lo, s_hi, wsum, roff);
}

// Partitioned large halos (k_part_join): one work-group per previous-block chunk (gchunks
// rows, RCHUNK positions each); its records sit unordered at the chunk's scratch base,
// each with its position in the chunk (scratch_rk).  Positions are distinct, so a record's
// rank in previous-block order is the number of set bits below its own in a bitmap of the
// chunk's record positions; the chunk's output offset is the item's plus the records of
// the item's earlier chunks.
template <int IDB>
__global__ __launch_bounds__(256) void k_gather_recs(const oa_compact_args a) {
    typedef typename IdT<IDB>::T ID;
    constexpr int NW = RCHUNK_GATHER / 32;
    __shared__ uint32_t bm[NW], wpre[NW], red[4];
    const int64_t row = blockIdx.x;
    const int64_t *ch = a.gchunks + 3 * row;
    const int64_t gi = ch[0], start = ch[1], cnt = ch[2];
    const oa_item it = a.items[gi];
    const int64_t slot = it.slot0;
    if (slot < 0 || cnt <= 0) return;                   // uniform
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t n = a.chunk_count[row];
    uint32_t before = 0;
    for (int64_t r = row - start / RCHUNK_GATHER + tid; r < row; r += 256) before += a.chunk_count[r];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) before += __shfl_down(before, o);
    if (lane == 0) red[wave] = before;
    for (int w = tid; w < NW; w += 256) bm[w] = 0u;
    __syncthreads();
    if (n == 0) return;                                 // uniform
    const int64_t s0 = it.scratch_off + start;
    for (uint32_t j = tid; j < n; j += 256) {
        const uint32_t rk = a.scratch_rk[s0 + j];
        atomicOr(&bm[rk >> 5], 1u << (rk & 31u));
    }
    __syncthreads();
    if (wave == 0) {                                    // exclusive popcount prefix of the words
        uint32_t c[NW / 64], t = 0;
#pragma unroll
        for (int q = 0; q < NW / 64; ++q) { c[q] = __popc(bm[lane * (NW / 64) + q]); t += c[q]; }
        uint32_t incl = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        uint32_t e = incl - t;
#pragma unroll
        for (int q = 0; q < NW / 64; ++q) { wpre[lane * (NW / 64) + q] = e; e += c[q]; }
    }
    __syncthreads();
    const int64_t dst = a.offsets_out[slot] + (int64_t)(red[0] + red[1] + red[2] + red[3]);
    const ID *src = reinterpret_cast<const ID *>(a.scratch_ids);
    ID *out = reinterpret_cast<ID *>(a.out_ids) + dst;
    uint16_t *oang = a.out_ang + dst;
    const int64_t pbase = a.out_pos ? a.halos[it.h0].prev_off + start : 0;
    for (uint32_t j = tid; j < n; j += 256) {
        const uint32_t rk = a.scratch_rk[s0 + j], w = rk >> 5;
        const uint32_t rank = wpre[w] + __popc(bm[w] & ((1u << (rk & 31u)) - 1u));
        out[rank] = src[s0 + j];
        oang[rank] = a.scratch_ang[s0 + j];
        if (a.out_pos) a.out_pos[dst + rank] = (int32_t)(pbase + rk);
    }
}

// ------------------------------------------------------------------ bulk velocity
template <typename T> __device__ T pw_leaf(const T *x, int n) {
    if (n < 8) {
        T r = (T)0;
        for (int i = 0; i < n; ++i) r = r + x[i];
        return r;
    }
    T r0 = x[0], r1 = x[1], r2 = x[2], r3 = x[3], r4 = x[4], r5 = x[5], r6 = x[6], r7 = x[7];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
        r0 = r0 + x[i + 0]; r1 = r1 + x[i + 1]; r2 = r2 + x[i + 2]; r3 = r3 + x[i + 3];
        r4 = r4 + x[i + 4]; r5 = r5 + x[i + 5]; r6 = r6 + x[i + 6]; r7 = r7 + x[i + 7];
    }
    T r = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) r = r + x[i];
    return r;
}

__device__ __forceinline__ int pw_half(int n) { int h = n / 2; return h - (h % 8); }

// numpy pairwise_sum: leaves <= 128 elements, split n -> (h, n - h), h = n/2 - (n/2)%8,
// evaluated with an explicit post-order stack (depth <= 12 for n <= 8192)
template <typename T> __device__ T pw_sum(const T *x, int n) {
    if (n <= 128) return pw_leaf(x, n);
    int so[24], sn[24], sp = 0;
    unsigned char ph[24];
    T sl[24];
    so[0] = 0; sn[0] = n; ph[0] = 0; sp = 1;
    T val = (T)0;
    while (sp > 0) {
        int t = sp - 1;
        if (ph[t] == 0 && sn[t] > 128) {             // descend into the left half
            ph[t] = 1;
            so[sp] = so[t]; sn[sp] = pw_half(sn[t]); ph[sp] = 0; ++sp;
            continue;
        }
        if (ph[t] == 0) { val = pw_leaf(x + so[t], sn[t]); --sp; }
        else if (ph[t] == 2) { val = sl[t] + val; --sp; }
        // deliver `val` to the parent
        while (sp > 0) {
            int p = sp - 1;
            if (ph[p] == 1) {
                sl[p] = val; ph[p] = 2;
                int hh = pw_half(sn[p]);
                so[sp] = so[p] + hh; sn[sp] = sn[p] - hh; ph[sp] = 0; ++sp;
                break;
            }
            val = sl[p] + val; --sp;                  // ph == 2: both halves done
        }
    }
    return val;
}

// One 64-lane work-group per halo.  Lanes 0..2 run the sequential axis-0 sum of
// (m*)v over rows staged in LDS; lane 0 runs numpy's pairwise sum of m per chunk.
template <typename TV, typename TM, bool MASS>
__global__ __launch_bounds__(64) void k_bulk(const TV *vels, const TM *masses, oa_halo *halos,
                                             const int32_t *list) {
    typedef typename std::conditional<(sizeof(TM) > sizeof(TV)) && MASS, TM, TV>::type TP;
    __shared__ TP rows[64][3];
    __shared__ TM mchunk[MASS ? BULK_CHUNK : 1];
    oa_halo &h = halos[list[blockIdx.x]];
    const int64_t off = h.cur_off, n = h.cur_cnt;
    const int lane = threadIdx.x;
    TP acc = (TP)0;
    for (int64_t c0 = 0; c0 < n; c0 += 64) {
        int64_t r = c0 + lane;
        if (r < n) {
            V3<TV> v = ld3(vels, off + r);
            if (MASS) {
                TP m = (TP)masses[off + r];
                rows[lane][0] = m * (TP)v.x; rows[lane][1] = m * (TP)v.y; rows[lane][2] = m * (TP)v.z;
            } else {
                rows[lane][0] = (TP)v.x; rows[lane][1] = (TP)v.y; rows[lane][2] = (TP)v.z;
            }
        }
        __syncthreads();
        if (lane < 3) {
            int64_t m = n - c0 < 64 ? n - c0 : 64;
            int j = 0;
            if (c0 == 0) { acc = rows[0][lane]; j = 1; }
            for (; j < m; ++j) acc = acc + rows[j][lane];
        }
        __syncthreads();
    }
    TP res;
    if (MASS) {
        TM tot = (TM)0;
        for (int64_t c0 = 0; c0 < n; c0 += BULK_CHUNK) {
            int len = (int)(n - c0 < BULK_CHUNK ? n - c0 : BULK_CHUNK);
            for (int i = lane; i < len; i += 64) mchunk[i] = masses[off + c0 + i];
            __syncthreads();
            if (lane == 0) tot = tot + pw_sum(mchunk, len);
            __syncthreads();
        }
        __shared__ TP msum;
        if (lane == 0) msum = (TP)tot;
        __syncthreads();
        res = acc / msum;
    } else {
        res = acc / (TP)n;
    }
    if (lane < 3) h.bulk[lane] = (double)res;
}

WrapK make_wrap(const double box[3], int32_t n_dims, int32_t f64) {
    WrapK w;
    w.n_dims = n_dims;
    w.f64 = f64;
    for (int d = 0; d < 3; ++d) {
        w.box[d] = box[d];
        // exact float32 thresholds of the strict tests dx > L/2 and dx < -L/2, where
        // L/2 is float64 (wrap_f64) or float32 arithmetic
        const double half = f64 ? box[d] / 2 : (double)((float)box[d] / 2.0f);
        float f = (float)half;
        w.hi[d] = (double)f > half ? f : nextafterf(f, INFINITY);
        float g = (float)(-half);
        w.lo[d] = (double)g < -half ? g : nextafterf(g, -INFINITY);
        w.ab[d] = fminf(w.hi[d], -w.lo[d]);
    }
    return w;
}

FrameK make_frame_k(const oa_step_args &a) {
    FrameK k;
    k.h_f = (float)(a.H / a.one_plus_z);
    k.w = make_wrap(a.box, a.n_box_dims, a.wrap_f64);
    return k;
}

template <typename K>
int set_lds(K kernel, int64_t bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return fail(OA_E_LAUNCH, "hipFuncSetAttribute: %s", hipGetErrorString(e));
    return OA_OK;
}

template <typename TX, typename TV, typename TD, int IDB, bool COMPARE, bool OTF>
int launch_big(const oa_step_args &a, hipStream_t st);

int cu_count() {
    // cached per device (the attribute query is per launch otherwise)
    static int cache[64] = {0};
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    if (dev >= 0 && dev < 64 && cache[dev] > 0) return cache[dev];
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1;
    if (n <= 0) n = 1;
    if (dev >= 0 && dev < 64) cache[dev] = n;
    return n;
}

template <typename TX, typename TV, typename TD, int IDB, bool COMPARE, bool OTF>
int launch_step_c(const oa_step_args &a, hipStream_t st) {
    if (a.n_items > 0) {
        // a frame-only launch needs no table: several work-groups share a CU
        const int64_t lds = COMPARE ? step_lds_bytes(a.lds_entries, a.lds_slots, (int)sizeof(TD))
                                    : HDR_BYTES;
        auto k = (COMPARE && !OTF && a.items_single) ? k_step<TX, TV, TD, IDB, COMPARE, OTF, true>
                                                     : k_step<TX, TV, TD, IDB, COMPARE, OTF, false>;
        if (int rc = set_lds(k, lds)) return rc;
        hipLaunchKernelGGL(k, dim3(a.n_items), dim3(WG), (size_t)lds, st, a, make_frame_k(a));
        if (int rc = check_launch("k_step")) return rc;
    }
    return launch_big<TX, TV, TD, IDB, COMPARE, OTF>(a, st);
}

template <typename TX, typename TV, typename TD, int IDB>
int launch_step(const oa_step_args &a, hipStream_t st) {
    if constexpr (std::is_same<TX, TD>::value) {    // on-the-fly: r̂ in the coordinate dtype
        if (a.onthefly)
            return a.compare ? launch_step_c<TX, TV, TD, IDB, true, true>(a, st)
                             : launch_step_c<TX, TV, TD, IDB, false, true>(a, st);
    }
    return a.compare ? launch_step_c<TX, TV, TD, IDB, true, false>(a, st)
                     : launch_step_c<TX, TV, TD, IDB, false, false>(a, st);
}

template <typename TX, typename TV, typename TD>
int launch_step_id(const oa_step_args &a, hipStream_t st) {
    return a.id_bytes == 8 ? launch_step<TX, TV, TD, 8>(a, st) : launch_step<TX, TV, TD, 4>(a, st);
}

template <typename TX, typename TD>
int launch_step_v(const oa_step_args &a, hipStream_t st) {
    return a.vel_f64 ? launch_step_id<TX, double, TD>(a, st) : launch_step_id<TX, float, TD>(a, st);
}

// ------------------------------------------------------------------ block helpers
// Module-level compare_radial_velocities / calc_angles (track_orbits.py:293-351) on
// arbitrary arrays: a global-memory open-addressing table of the current IDs (unique
// within a block, the myin1d precondition, utils.py:4-11), probed by the previous IDs.
__device__ __forceinline__ uint64_t id_hash64(uint64_t x) {
    x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; x *= 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 33);
}
template <int IDB>
__device__ __forceinline__ uint64_t load_id(const void *p, int64_t i) {
    return IDB == 8 ? static_cast<const uint64_t *>(p)[i]
                    : (uint64_t)static_cast<const uint32_t *>(p)[i];
}
template <int IDB>
__global__ __launch_bounds__(256) void k_match_insert(const void *ids, int64_t n, uint64_t *keys,
                                                      uint32_t *vals, uint64_t cap) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t id = load_id<IDB>(ids, i);
    uint64_t s = id_hash64(id) & (cap - 1);
    for (uint64_t t = 0; t < cap; ++t) {
        if (atomicCAS(&vals[s], 0u, (uint32_t)(i + 1)) == 0u) { keys[s] = id; return; }
        s = (s + 1) & (cap - 1);
    }
}
template <int IDB>
__global__ __launch_bounds__(256) void k_match_probe(const void *ids_prev, int64_t n_prev,
                                                     const uint64_t *keys, const uint32_t *vals,
                                                     uint64_t cap, int64_t *match) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n_prev) return;
    const uint64_t id = load_id<IDB>(ids_prev, i);
    uint64_t s = id_hash64(id) & (cap - 1);
    int64_t m = -1;
    for (uint64_t t = 0; t < cap; ++t) {
        const uint32_t v = vals[s];
        if (v == 0u) break;
        if (keys[s] == id) { m = (int64_t)v - 1; break; }
        s = (s + 1) & (cap - 1);
    }
    match[i] = m;
}
// per previous particle: matched flag, strict sign-flip flag (:311-314) and
// arccos(dot(r̂_prev, r̂_match)) in TD (:324-325)
template <typename TD>
__global__ __launch_bounds__(256) void k_compare_pairs(const int64_t *match, int64_t n_prev,
                                                       const double *vr, const double *vr_prev,
                                                       const TD *rhat, const TD *rhat_prev,
                                                       int32_t mode, uint8_t *flag, TD *change) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n_prev) return;
    const int64_t j = match[i];
    if (j < 0) { flag[i] = 0; return; }
    const double a = vr_prev[i], b = vr[j];
    const bool c = mode == OA_MODE_PERICENTRIC ? (a < 0.0 && b > 0.0) : (a > 0.0 && b < 0.0);
    flag[i] = c ? 1 : 0;
    const TD d = dot3(rhat_prev[3 * i], rhat_prev[3 * i + 1], rhat_prev[3 * i + 2],
                      rhat[3 * j], rhat[3 * j + 1], rhat[3 * j + 2]);
    change[i] = acos_td(d);
}
// f16 angles + TD changes, rounded straight to f16 (calc_angles :342-351)
template <typename TD>
__global__ __launch_bounds__(256) void k_angle_add(const uint16_t *prev, const TD *change,
                                                   int64_t n, uint16_t *out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) out[i] = angle_add(prev[i], change[i]);
}

// ------------------------------------------------------------------ large halos
// A halo whose block exceeds one work-group's LDS table is joined through a
// per-halo open-addressing table in global memory (L2 / Infinity Cache resident),
// so any number of work-groups can share it and every particle is streamed once:
//   k_big_frame  chunks of the halo's current block: frame, r̂ / meta stores, and
//                (compare) insert id -> position (device-scope CAS on the slot)
//   k_big_join   chunks of its previous block, 64-position segments per wave:
//                probe, gather the current r̂ + meta, flag, angle, state update,
//                apsis records packed per segment exactly as k_step does
// Chunks are (item, start, count) triples built by the host (engine.plan_items).
constexpr int BIG_WG = 256;

// large-halo table slot of a hash: range reduction onto any capacity (the host sizes
// tables to a ~0.7 load so they stay Infinity-Cache resident), linear probing
__device__ __forceinline__ uint64_t big_slot(uint64_t h, uint64_t cap) {
    return __umul64hi(h, cap);
}
__device__ __forceinline__ uint64_t big_next(uint64_t s, uint64_t cap) {
    return s + 1 == cap ? 0 : s + 1;
}

template <typename TX, typename TV, typename TD, int IDB, bool COMPARE, bool OTF>
__global__ __launch_bounds__(BIG_WG) void k_big_frame(const oa_step_args a, const FrameK fk) {
    typedef typename IdT<IDB>::T ID;
    const int64_t *ch = a.gchunk1 + 3 * blockIdx.x;
    const int64_t gi = ch[0], start = ch[1], cnt = ch[2];
    const oa_item it = a.items[gi];
    const oa_halo &h = a.halos[it.h0];
    double cb[6];
    float cf[6];
#pragma unroll
    for (int d = 0; d < 3; ++d) { cb[d] = h.centre[d]; cb[3 + d] = h.bulk[d]; }
#pragma unroll
    for (int d = 0; d < 6; ++d) cf[d] = (float)cb[d];
    const int64_t base = h.cur_off;
    const bool ins = COMPARE && h.prev_cnt >= 0;
    const ID *ids = static_cast<const ID *>(a.ids);
    const TX *xs = static_cast<const TX *>(a.coords);
    const TV *vs = static_cast<const TV *>(a.vels);
    TD *rhat_out = static_cast<TD *>(a.rhat_out);
    const int64_t gk = gi - a.n_items;             // global items follow the packed ones
    // table entries: 16 bytes {u64 id, u32 position + 1 (0 = empty), pad}: a probe
    // touches one cache line
    uint64_t *tab = a.gkeys + 2 * a.gtab[2 * gk];
    const uint64_t cap = (uint64_t)a.gtab[2 * gk + 1];
    for (int64_t p = start + threadIdx.x; p < start + cnt; p += BIG_WG) {
        const int64_t i = base + p;
        const ID id = lds_nt(&ids[i]);
        const V3<TX> x = ld3_nt(xs, i);
        const V3<TV> v = ld3_nt(vs, i);
        TD r[3];
        const uint32_t sgn = OTF ? frame_otf<TX, TV, TD>(x, v, cb, a, fk, r)
                                 : frame<TX, TV, TD>(x, v, cb, cf, a, fk, r);
        TD *ro = rhat_out + 3 * i;
        ro[0] = r[0]; ro[1] = r[1]; ro[2] = r[2];
        uint32_t ang = 0;
        if (!COMPARE && a.angles_in) ang = a.angles_in[i];
        a.meta_out[i] = ang | (sgn << 16);
        if (ins) {
            uint64_t sl = big_slot(id_hash64((uint64_t)id), cap);
            for (uint64_t t = 0; t < cap; ++t) {
                uint32_t *val = reinterpret_cast<uint32_t *>(tab + 2 * sl + 1);
                if (atomicCAS(val, 0u, (uint32_t)(p + 1)) == 0u) {
                    tab[2 * sl] = (uint64_t)id;
                    break;
                }
                sl = big_next(sl, cap);
            }
        }
    }
}

template <typename TD, int IDB, bool OTF>
__global__ __launch_bounds__(BIG_WG) void k_big_join(const oa_step_args a) {
    typedef typename IdT<IDB>::T ID;
    const int64_t *ch = a.gchunk2 + 3 * blockIdx.x;
    const int64_t gi = ch[0], start = ch[1], cnt = ch[2];
    const oa_item it = a.items[gi];
    const oa_halo &h = a.halos[it.h0];
    const int64_t cbase = h.cur_off, pbase = h.prev_off;
    const ID *ids_prev = static_cast<const ID *>(a.ids_prev);
    const TD *rhat_prev = static_cast<const TD *>(a.rhat_prev);
    const TD *rhat_out = static_cast<const TD *>(a.rhat_out);
    const int64_t gk = gi - a.n_items;
    const uint64_t *tab = a.gkeys + 2 * a.gtab[2 * gk];
    const uint64_t cap = (uint64_t)a.gtab[2 * gk + 1];
    ID *scr_ids = static_cast<ID *>(a.scratch_ids);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lanemask_lt = (1ull << lane) - 1ull;
    for (int64_t v0 = start; v0 < start + cnt; v0 += BIG_WG) {
        const int64_t p = v0 + threadIdx.x;
        const bool ok = p < start + cnt;
        bool flag = false, hit = false;
        uint16_t a16 = 0;
        ID pid = 0;
        if (ok) {
            const int64_t k = pbase + p;
            pid = lds_nt(&ids_prev[k]);
            const V3<TD> prh = ld3_nt(rhat_prev, k);
            const uint32_t pmeta = lds_nt(&a.meta_prev[k]);
            uint64_t sl = big_slot(id_hash64((uint64_t)pid), cap);
            int64_t j = -1;
            for (uint64_t t = 0; t < cap; ++t) {
                const uint4 e = *reinterpret_cast<const uint4 *>(tab + 2 * sl);
                if (e.z == 0u) break;
                if ((((uint64_t)e.y << 32) | e.x) == (uint64_t)pid) { j = (int64_t)e.z - 1; break; }
                sl = big_next(sl, cap);
            }
            if (j >= 0) {
                hit = true;
                const int64_t c = cbase + j;
                const TD *cr = rhat_out + 3 * c;
                const uint32_t cmeta = a.meta_out[c];
                const uint32_t sc = cmeta >> 16, sp = pmeta >> 16;
                // strict sign test (:311-314)
                flag = a.mode == OA_MODE_PERICENTRIC ? (sp == 2u && sc == 1u) : (sp == 1u && sc == 2u);
                // arccos(dot(r̂_prev, r̂_match)) (:324-325), f16 + change (:342-351)
                const TD dt = dot3(prh.x, prh.y, prh.z, cr[0], cr[1], cr[2]);
                const TD change = acos_change<OTF>(dt);
                const uint16_t acc = angle_add((uint16_t)(pmeta & 0xFFFFu), change);
                a16 = acc;
                a.meta_out[c] = (uint32_t)(flag ? 0u : acc) | (sc << 16);
                if (OTF) {
                    static_cast<TD *>(a.angle_out)[k] = change;
                    a.matched_cur[c] = 1;
                }
            }
            if (OTF) a.matched_prev[k] = hit ? 1 : 0;
        }
        // apsis records in previous-block order (:315-316), one 64-position segment
        // per wave, packed at the segment's scratch base as in k_step
        const uint64_t m = __ballot(flag);
        const int64_t segpos = v0 + wave * 64;
        if (segpos < start + cnt) {
            if (flag) {
                const int64_t pos = it.scratch_off + segpos + __popcll(m & lanemask_lt);
                scr_ids[pos] = pid;
                a.scratch_ang[pos] = a16;
                if (a.scratch_pos) a.scratch_pos[pos] = (int32_t)(pbase + p);
            }
            if (lane == 0) {
                const uint32_t c = (uint32_t)__popcll(m);
                a.seg_count[(it.scratch_off + segpos) >> 6] = (uint8_t)c;
                if (c) {
                    atomicAdd(&a.halo_count[h.out_slot], (int32_t)c);
                    atomicAdd(&a.item_count[gi], (int32_t)c);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ partitioned large halos
// The default large-halo path of compare steps.  A halo too large for one work-group's
// LDS table is cut into K partitions by a hash of the full ID, each small enough for an
// LDS cuckoo table, so the join is LDS-local like k_step's and every HBM stream is
// coalesced (the global-table path above pays a random HBM access per insert and probe).
// A halo's state lives between snapshots as a *bucket set* (per partition: key, position
// word, state word, r̂), so a step streams the previous state from its buckets:
//   k_part_scatter  chunks of the current blocks: the frame, each particle's entry
//                   {key, position | sign << 30, r̂} staged in LDS in partition order and
//                   copied to its bucket as contiguous runs (one device atomic per
//                   partition and chunk reserves the range); previous chunks only for
//                   halos without an inherited set
//   k_part_join     one work-group per partition: LDS cuckoo table of the current
//                   bucket, then every previous entry of the partition looked up; a match
//                   gathers the current r̂ from the bucket, writes the current state word
//                   and, for an apsis, appends the record {ID, angle, position in chunk}
//                   to its previous-block chunk (oa_compact's k_gather_recs orders them)
#ifndef OA_PART_E
#define OA_PART_E 4096
#endif
constexpr int PART_E = OA_PART_E;       // current entries of one partition, at most
constexpr int PART_S = PART_E + PART_E / 2;   // LDS table slots, at most
// 512 threads, <= 128 VGPRs and ~58 KB of LDS: two join work-groups per CU, so one's
// table build overlaps the other's streaming
constexpr int PART_KMAX = 4096;         // partitions of one halo (scatter's LDS counters)
#ifndef OA_PART_WG
#define OA_PART_WG 512
#endif
constexpr int PART_WG = OA_PART_WG;
constexpr int GPART_W = 16;             // int64 per gpart row (orbit_hip.h)
#ifndef OA_SCAT_PER
#define OA_SCAT_PER 4       // k_part_scatter: particles per thread per staged sub-chunk
#endif
constexpr int SCAT_WG = 256, SCAT_PER = OA_SCAT_PER, SCAT_NS = SCAT_WG * SCAT_PER;
static_assert(PART_E - 1 <= (int)MAX_POS, "partition entries must fit the slot position field");
static_assert(PART_KMAX <= 65536, "staged partition numbers are 16-bit");

// partition of an ID: the high bits of a 64-bit mix (the LDS table hashes the low
// word with unrelated multipliers, so a partition's keys still spread over its table).
// K is a power of two, so partition p of K is partitions [p*2^d, (p+1)*2^d) of K*2^d:
// a bucket set built with one K serves a join with another.
__device__ __forceinline__ uint32_t part_of(uint64_t id, uint32_t K) {
    return (uint32_t)__umul64hi(id_hash64(id ^ 0x2545F4914F6CDD1Dull), (uint64_t)K);
}

// LDS of one k_part_scatter work-group: per partition its sub-chunk count (scanned in
// place into the run's first staged index) and reserved bucket index, then the staged
// records {r̂, key (kb bytes), position word, state word, partition} of one sub-chunk
// in partition order, copied out as contiguous runs.
__host__ __device__ inline int64_t scat_lds_bytes(int kmax, int td_bytes, int kb) {
    const int64_t k = ((int64_t)kmax * 8 + 15) & ~int64_t(15);
    return 64 + k + (int64_t)SCAT_NS * (3 * td_bytes + kb + 4 + 4 + 2);
}

// exclusive scan of v[0, n) in place (n <= PART_KMAX), SCAT_WG threads, wtot[>= 4]
__device__ __forceinline__ void block_scan_excl(uint32_t *v, uint32_t n, uint32_t *wtot) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c = (n + SCAT_WG - 1) / SCAT_WG, b = tid * c;
    uint32_t s = 0;
    for (uint32_t i = 0; i < c; ++i) if (b + i < n) s += v[b + i];
    uint32_t incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wave] = incl;
    lds_barrier();
    uint32_t run = incl - s;
    for (int w = 0; w < wave; ++w) run += wtot[w];
    for (uint32_t i = 0; i < c; ++i)
        if (b + i < n) { const uint32_t x = v[b + i]; v[b + i] = run; run += x; }
    lds_barrier();
}

// CUR: current chunks (gchunk1), else previous chunks (gchunk2).  A bucket entry holds
// a particle's whole state -- ID, position in its block (| sign << 30 for current
// entries), state word, r̂ -- so the join streams it and a current bucket set is the
// next snapshot's previous one.  Previous chunks of halos whose previous state is
// already such a set (gpart[3] = 1, inherited) are skipped.
// KB: bucket key bytes (4: the IDs' low words, oa_step_args.part_key4)
template <typename TX, typename TV, typename TD, int IDB, bool CUR, int KB>
__device__ __forceinline__ void part_scatter(const oa_step_args &a, const FrameK &fk, char *lds,
                                             int64_t chunk) {
    typedef typename IdT<IDB>::T ID;
    typedef typename IdT<KB>::T KEY;
    const int64_t *ch = (CUR ? a.gchunk1 : (a.gchunk3 ? a.gchunk3 : a.gchunk2)) + 3 * chunk;
    const int64_t gi = ch[0], start = ch[1], cnt = ch[2];
    const oa_item it = a.items[gi];
    const oa_halo &h = a.halos[it.h0];
    const int64_t gk = gi - a.n_items;
    const int64_t *gp = a.gpart + GPART_W * gk;
    const uint32_t K = (uint32_t)gp[1];
    const bool part = h.prev_cnt > 0 && K > 0;
    if (!CUR && (!part || gp[3] != 0)) return;          // inherited previous set (uniform)
    const int tid = threadIdx.x;
    double cb[6];
    float cf[6];
    if (CUR) {
#pragma unroll
        for (int d = 0; d < 3; ++d) { cb[d] = h.centre[d]; cb[3 + d] = h.bulk[d]; }
#pragma unroll
        for (int d = 0; d < 6; ++d) cf[d] = (float)cb[d];
    }
    const ID *ids = static_cast<const ID *>(CUR ? a.ids : a.ids_prev);
    const TX *xs = static_cast<const TX *>(a.coords);
    const TV *vs = static_cast<const TV *>(a.vels);
    TD *rhat_out = static_cast<TD *>(a.rhat_out);
    const TD *rhat_prev = static_cast<const TD *>(a.rhat_prev);
    const int64_t base = CUR ? h.cur_off : h.prev_off;
    uint32_t *ctr = a.pcnt + (CUR ? gp[2] : gp[7]);
    const uint32_t bcap = CUR ? (uint32_t)a.part_e : (uint32_t)gp[6];
    const int64_t bb = CUR ? gp[0] : gp[4];
    KEY *bkey = static_cast<KEY *>(CUR ? a.pkey_cur : a.pkey_prev) + bb;
    bool badhi = false;                                 // part_key4: a foreign high word
    uint32_t *bpos = (CUR ? a.ppos_cur : a.ppos_prev) + bb;
    uint32_t *bmeta = (CUR ? a.pmeta_cur : a.pmeta_prev) + bb;
    TD *brh = static_cast<TD *>(CUR ? a.prh_cur : a.prh_prev) + 3 * bb;
    // LDS carve-up (scat_lds_bytes)
    uint32_t *wtot = reinterpret_cast<uint32_t *>(lds);
    uint32_t *lrun = wtot + 16;                         // [K] count -> first staged index
    uint32_t *gres = lrun + K;                          // [K] reserved bucket index
    char *stg = lds + 64 + (((int64_t)K * 8 + 15) & ~int64_t(15));
    TD *srh = reinterpret_cast<TD *>(stg);
    KEY *skey = reinterpret_cast<KEY *>(srh + 3 * SCAT_NS);
    uint32_t *spw = reinterpret_cast<uint32_t *>(skey + SCAT_NS);
    uint32_t *smeta = spw + SCAT_NS;
    uint16_t *spart = reinterpret_cast<uint16_t *>(smeta + SCAT_NS);
    for (int64_t s0 = start; s0 < start + cnt; s0 += SCAT_NS) {
        const int64_t n0 = min(start + cnt - s0, (int64_t)SCAT_NS);
        if (part) {
            for (uint32_t k = tid; k < K; k += SCAT_WG) lrun[k] = 0u;
            lds_barrier();
        }
        uint64_t key[SCAT_PER];
        uint32_t pw[SCAT_PER], pr[SCAT_PER], pm[SCAT_PER];
        V3<TD> rh[SCAT_PER];
        V3<TX> xq[SCAT_PER];
        V3<TV> vq[SCAT_PER];
        // every load of the sub-chunk first, then the arithmetic: buffer loads, so lanes
        // past the sub-chunk read 0 with no branch (a load under a lane test waits for
        // its data before the next one issues)
        const int64_t i0 = base + s0;
        const Rsrc rid = make_rsrc(ids + i0, (uint32_t)n0 * IDB);
        const Rsrc rx = make_rsrc(CUR ? (const void *)(xs + 3 * i0) : (const void *)(a.meta_prev + i0),
                                  CUR ? (uint32_t)n0 * 3 * sizeof(TX) : (uint32_t)n0 * 4);
        const Rsrc rv = make_rsrc(CUR ? (const void *)(vs + 3 * i0) : (const void *)(rhat_prev + 3 * i0),
                                  (uint32_t)n0 * 3 * (CUR ? sizeof(TV) : sizeof(TD)));
#pragma unroll
        for (int q = 0; q < SCAT_PER; ++q) {
            const uint32_t j = (uint32_t)q * SCAT_WG + tid;
            key[q] = (uint64_t)bld<ID, AUX_NT>(rid, j * IDB);
            if (CUR) {
                xq[q] = bld3<TX, AUX_NT>(rx, j * 3 * sizeof(TX));
                vq[q] = bld3<TV, AUX_NT>(rv, j * 3 * sizeof(TV));
            } else {
                pm[q] = bld<uint32_t, AUX_NT>(rx, j * 4);
                rh[q] = bld3<TD, AUX_NT>(rv, j * 3 * sizeof(TD));
            }
        }
        if (IDB == 8 && KB == 4 && part) {
#pragma unroll
            for (int q = 0; q < SCAT_PER; ++q)
                badhi |= (int64_t)q * SCAT_WG + tid < n0 && (uint32_t)(key[q] >> 32) != a.part_hi;
        }
#pragma unroll
        for (int q = 0; q < SCAT_PER; ++q) {
            pr[q] = 0xFFFFFFFFu;
            pw[q] = 0u;
            const int64_t j = (int64_t)q * SCAT_WG + tid;
            if (j >= n0) continue;
            const int64_t p = s0 + j;                   // position in the halo's block
            const int64_t i = base + p;
            if (CUR) {
                const V3<TX> x = xq[q];
                const V3<TV> v = vq[q];
                TD r[3];
                const uint32_t sgn = frame<TX, TV, TD>(x, v, cb, cf, a, fk, r);
                if (!part) {
                    // a halo without a progenitor: its state in position order (angle 0:
                    // calc_angles :348-349), as k_big_frame writes it
                    TD *ro = rhat_out + 3 * i;
                    ro[0] = r[0]; ro[1] = r[1]; ro[2] = r[2];
                    a.meta_out[i] = sgn << 16;
                    continue;
                }
                rh[q] = V3<TD>{r[0], r[1], r[2]};
                pm[q] = sgn << 16;                      // angle 0 until the join matches it
                pw[q] = (uint32_t)p | (sgn << 30);
            } else {
                pw[q] = (uint32_t)p;
            }
            const uint32_t pp = part_of(key[q], K);
            pr[q] = (pp << 16) | atomicAdd(&lrun[pp], 1u);
        }
        if (!part) continue;                            // uniform
        if (s0 == start) SSTAMP(1);
        lds_barrier();
        if (s0 == start) SSTAMP(2);
        // this sub-chunk's range of every bucket (one device atomic per partition hit),
        // then the runs' first staged indices
        // (up to SCAT_WG partitions the reservations stay in registers until the staging
        // is done: the atomics' round trip overlaps the scan and the staging writes)
        const bool kreg = K <= (uint32_t)SCAT_WG;
        uint32_t res = 0u;
        if (kreg) {
            const uint32_t c = tid < (int)K ? lrun[tid] : 0u;
            if (c) res = atomicAdd(&ctr[tid], c);
        } else {
            for (uint32_t k = tid; k < K; k += SCAT_WG) {
                const uint32_t c = lrun[k];
                gres[k] = c ? atomicAdd(&ctr[k], c) : 0u;
            }
        }
        block_scan_excl(lrun, K, wtot);
        if (s0 == start) SSTAMP(3);
#pragma unroll
        for (int q = 0; q < SCAT_PER; ++q) {
            if (pr[q] == 0xFFFFFFFFu) continue;
            const uint32_t pp = pr[q] >> 16, e = lrun[pp] + (pr[q] & 0xFFFFu);
            skey[e] = (KEY)key[q];
            srh[3 * e] = rh[q].x; srh[3 * e + 1] = rh[q].y; srh[3 * e + 2] = rh[q].z;
            spw[e] = pw[q];
            smeta[e] = pm[q];
            spart[e] = (uint16_t)pp;
        }
        if (kreg && tid < (int)K) gres[tid] = res;
        lds_barrier();
        if (s0 == start) SSTAMP(4);
        // copy-out: consecutive staged records of one partition go to consecutive bucket
        // entries, so a wave's stores are a few contiguous runs, not 64 scattered words
        // (the work-group's barriers wait for LDS traffic only: these stores stay in
        // flight into the next sub-chunk)
        for (int64_t s = tid; s < n0; s += SCAT_WG) {
            const uint32_t k = spart[s];
            const uint32_t e = gres[k] + (uint32_t)(s - lrun[k]);
            if (e < bcap) {                             // an overflow is reported by the join
                const int64_t o = (int64_t)k * bcap + e;
                TD *d = brh + 3 * o;
                // key, position and state words non-temporal; a current entry's state
                // word is the join's (k_part_join stages them)
                __builtin_nontemporal_store(skey[s], &bkey[o]);
                __builtin_nontemporal_store(spw[s], &bpos[o]);
                if (!CUR) __builtin_nontemporal_store(smeta[s], &bmeta[o]);
#ifdef OA_DIAG_PART_NORH
                if (!CUR)   // diagnostic: no current r̂ in the bucket (wrong angles)
#endif
                d[0] = srh[3 * s]; d[1] = srh[3 * s + 1]; d[2] = srh[3 * s + 2];
            }
        }
        lds_barrier();
        if (s0 == start) SSTAMP(5);
    }
    if (IDB == 8 && KB == 4 && __ballot(badhi) && (threadIdx.x & 63) == 0)
        atomicOr(a.status, OA_STATUS_PART_KEYS);
}

// Current and previous chunks interleaved in one grid (their latencies overlap):
// even work-groups take current chunks, odd ones previous chunks, then the longer
// list's remainder.
template <typename TX, typename TV, typename TD, int IDB, int KB>
__global__ __launch_bounds__(SCAT_WG) void k_part_scatter(const oa_step_args a, const FrameK fk) {
    extern __shared__ __attribute__((aligned(16))) char slds[];
    const int64_t b = blockIdx.x, n1 = a.n_gchunk1,
                  n2 = a.gchunk3 ? a.n_gchunk3 : a.n_gchunk2;
    const int64_t m = n1 < n2 ? n1 : n2;
    bool cur;
    int64_t c;
    if (b < 2 * m) { cur = (b & 1) == 0; c = b >> 1; }
    else { cur = n1 > n2; c = b - m; }
    SSTAMP(0);
    if (cur) part_scatter<TX, TV, TD, IDB, true, KB>(a, fk, slds, c);
    else part_scatter<TX, TV, TD, IDB, false, KB>(a, fk, slds, c);
    SSTAMP(7);
}

// k_part_join's apsis records staged in LDS before their slots are claimed (16 B each:
// ID, position in the halo's previous block, angle, rank in its chunk); a work-group
// with more records claims the rest one global atomic each
constexpr int PART_RB = 768;

// LDS of one k_part_join work-group for a partition capacity of e entries, s slots:
// the slots, then max(deferral list, the partition's state words), the stash, flags,
// the staged records (two work-groups per CU at 4096 entries in 6144 slots)
__host__ __device__ inline int64_t part_lds_bytes(int e, int sl) {
    const int64_t mid = (int64_t)e * 4 > (int64_t)(e / 4) * 8 ? (int64_t)e * 4 : (int64_t)(e / 4) * 8;
    return (int64_t)sl * 8 + mid + (int64_t)STASH * 8 + 16 + 16 + (int64_t)PART_RB * 16;
}

// The apsis records of a partitioned halo (k_part_join -> oa_compact): a record is
// appended to the chunk of RCHUNK previous-block positions holding its particle (the
// gchunk2 rows of the item, engine.GCHUNK), at the chunk's scratch base + a slot from
// the chunk's counter, with its position in the chunk (scratch_rk); k_gather_recs ranks
// a chunk's records by that position, so they leave in previous-block order (:315-316).
constexpr int RCHUNK_LOG2 = 12, RCHUNK = 1 << RCHUNK_LOG2;
static_assert(RCHUNK == RCHUNK_GATHER, "record chunks of the join and the gather");

// One work-group per current partition: LDS cuckoo table of its current bucket, then
// every entry of the previous partitions that hold its IDs (one, several or a share of
// one, as K and the previous set's K compare) looked up; a match gathers the current
// r̂ from its bucket entry and writes that entry's state word; an apsis appends its
// record to its previous-block chunk.  KB: bucket key bytes (4: low words, every ID's
// high word is part_hi).
template <typename TD, int IDB, int KB>
__global__ __launch_bounds__(PART_WG) void k_part_join(const oa_step_args a) {
    typedef typename IdT<IDB>::T ID;
    typedef typename IdT<KB>::T KEY;
    extern __shared__ __attribute__((aligned(16))) char psm[];
    const uint32_t PE = (uint32_t)a.part_e, PS = (uint32_t)a.part_slots;
    uint64_t *slots = reinterpret_cast<uint64_t *>(psm);               // [PS]
    uint64_t *pend = slots + PS;                                        // [PE / 4]
    // after the walks: the partition's state words, over the deferral list
    uint32_t *mlds = reinterpret_cast<uint32_t *>(pend);                // [PE]
    uint64_t *stash = pend + (PE * 4 > (PE / 4) * 8 ? PE / 2 : PE / 4); // [STASH]
    uint32_t *flags = reinterpret_cast<uint32_t *>(stash + STASH);      // npend, nstash, overflow, nonuniform
    uint32_t *nrec = flags + 4;                                         // records of the work-group
    uint64_t *rbuf = reinterpret_cast<uint64_t *>(flags + 8);           // [2 PART_RB] staged records
    const int tid = threadIdx.x;
    PSTAMP(0);
    // the work-group's descriptor row: its item's gpart row and the item and halo fields
    // it needs, in one row, read by one vector load (lane f: field f) and broadcast with
    // readlane -- scalar loads of the row were split around the padding-row test and
    // chained several round trips before the bucket loads
    int64_t gp[GPART_W];
    {
        const Rsrc rrow = make_rsrc(a.prow + GPART_W * (int64_t)blockIdx.x, GPART_W * 8u);
        const int64_t mine = bld<int64_t, 0>(rrow, (uint32_t)(tid & (GPART_W - 1)) * 8u);
        const uint32_t lo = (uint32_t)mine, hi = (uint32_t)((uint64_t)mine >> 32);
#pragma unroll
        for (int f = 0; f < 14; ++f)
            gp[f] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, f) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)lo, f));
    }
    const int64_t g = gp[10];
    if (g < 0) return;                                  // padding row
    const uint32_t pp = (uint32_t)gp[9];
    const int64_t gi = a.n_items + g;
    const uint32_t K = (uint32_t)gp[1];
    const int64_t cb = gp[0] + (int64_t)pp * PE;
    const bool inh = gp[3] != 0;
    const uint32_t Kp = (uint32_t)gp[5], pcap = (uint32_t)gp[6];
    const uint32_t *qcnt = (inh ? a.icnt : a.pcnt) + gp[7];
    const KEY *qk0 = static_cast<const KEY *>(inh ? a.ikey : a.pkey_prev) + gp[4];
    const uint32_t *qp0 = (inh ? a.ipos : a.ppos_prev) + gp[4];
    const uint32_t *qm0 = (inh ? a.imeta : a.pmeta_prev) + gp[4];
    const TD *qr0 = static_cast<const TD *>(inh ? a.irh : a.prh_prev) + 3 * gp[4];
    // the previous partitions holding this partition's IDs: K and Kp are powers of two
    const bool filt = Kp < K;
    const uint32_t q0 = filt ? (uint32_t)pp / (K / Kp) : (uint32_t)pp * (Kp / K);
    const uint32_t nq = filt ? 1u : Kp / K;
    const KEY *ck = static_cast<const KEY *>(a.pkey_cur) + cb;
    const uint32_t *cp = a.ppos_cur + cb;
    // Every load of the partition goes out first (both buckets are streamed once):
    // their HBM latency hides behind the table clear, the inserts and the walks.  The
    // loads are buffer loads bounded by the buckets' capacities, so they issue before
    // the counts arrive and back to back (a load under a lane test waits for its data
    // before the next one issues); entries past a count are masked where they are used.
    constexpr int CU = PART_E / PART_WG, PU = OA_PU;
    // the counts too, as uniform-address vector loads issued first: they are waited for
    // after the table clear, beside the first bucket data, not on a scalar round trip
    // before the clear (the table spans every slot, so its size needs no count)
    const uint32_t nc_v = bld<uint32_t, 0>(make_rsrc(a.pcnt + gp[2] + pp, 4u), 0u);
    const uint32_t np0_v = bld<uint32_t, 0>(make_rsrc(qcnt + q0, 4u), 0u);
    KEY ckey[CU];
    uint32_t cpw[CU];
    {
        const Rsrc rk = make_rsrc(ck, PE * KB), rp = make_rsrc(cp, PE * 4);
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const uint32_t i = (uint32_t)u * PART_WG + tid;
            ckey[u] = bld<KEY, 0>(rk, i * KB);
            cpw[u] = bld<uint32_t, 0>(rp, i * 4);
        }
    }
    const TD *crh0 = static_cast<const TD *>(a.prh_cur) + 3 * cb;
    KEY qkey[PU];
    uint32_t qpos[PU], qmeta[PU];
    V3<TD> qrh[PU];
    // entries [j0, j0 + PART_WG * PU) of previous partition q0 + q, lanes past np read 0
    auto load_prev = [&](uint32_t q, uint32_t np, uint32_t j0) __attribute__((always_inline)) {
        const int64_t qo = (int64_t)(q0 + q) * pcap;
        const Rsrc rk = make_rsrc(qk0 + qo, np * KB), rp = make_rsrc(qp0 + qo, np * 4);
        const Rsrc rm = make_rsrc(qm0 + qo, np * 4);
        const Rsrc rr = make_rsrc(qr0 + 3 * qo, np * 3 * (uint32_t)sizeof(TD));
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const uint32_t j = j0 + (uint32_t)u * PART_WG + tid;
            qkey[u] = bld<KEY, 0>(rk, j * KB);
            qpos[u] = bld<uint32_t, 0>(rp, j * 4);
            qmeta[u] = bld<uint32_t, 0>(rm, j * 4);
            qrh[u] = bld3<TD, 0>(rr, j * 3 * (uint32_t)sizeof(TD));
        }
    };
    load_prev(0u, pcap, 0u);                            // the capacity: the count is in flight
    const uint32_t nsl = PS;                            // load <= 0.67 (4096 in 6144)
    for (uint32_t w = tid; w < nsl; w += PART_WG) slots[w] = 0ull;
    if (tid < 8) flags[tid] = 0u;
    const uint32_t hi0 = KB == 8 ? (uint32_t)((uint64_t)ck[0] >> 32) : 0u;
    // barriers on LDS traffic only up to the lookups: the previous entries' loads stay
    // in flight behind the table build (each use waits for its own loads)
    lds_barrier();
    const uint32_t nc = uni(nc_v);
    bool over = nc > PE || uni(np0_v) > pcap;
    for (uint32_t q = 1; q < nq; ++q) over |= qcnt[q0 + q] > pcap;
    if (over) {                                         // uniform
        if (tid == 0) atomicOr(a.status, OA_STATUS_PART_OVERFLOW);
        return;
    }
    PSTAMP(1);
    // current bucket -> LDS table: lo32(ID) | (sign << 16 | (entry + 1) << 18) << 32
    const uint32_t pend_cap = PE / 4;
#pragma unroll
    for (int u = 0; u < CU; ++u) {
        const uint32_t i = (uint32_t)u * PART_WG + tid;
        if (i >= nc) continue;
        const uint64_t key = (uint64_t)ckey[u];
        if (KB == 8 && (uint32_t)(key >> 32) != hi0) flags[3] = 1u;   // benign race: all write 1
        const uint64_t val = slot_pack((uint32_t)key, (cpw[u] >> 30) << 16, i);
        uint32_t cs[NCAND];
        cuckoo_slots((uint32_t)key, nsl, cs);
        uint64_t cv[NCAND];
#pragma unroll
        for (int j = 0; j < NCAND; ++j) cv[j] = slots[cs[j]];
        uint32_t t = 0xFFFFFFFFu;
#pragma unroll
        for (int j = NCAND - 1; j >= 0; --j) t = cv[j] == 0ull ? cs[j] : t;
        if (t != 0xFFFFFFFFu &&
            atomicCAS(reinterpret_cast<unsigned long long *>(&slots[t]), 0ull,
                      (unsigned long long)val) == 0ull)
            continue;
        const uint32_t e = atomicAdd(&flags[0], 1u);
        if (e < pend_cap) pend[e] = val; else flags[2] = 1u;
    }
    lds_barrier();
    PSTAMP(2);
    {   // deferred eviction walks (as k_step's)
        const uint32_t npd = min(flags[0], pend_cap);
        for (uint32_t e = tid; e < npd; e += PART_WG) {
            uint64_t v = pend[e];
            uint32_t cs[NCAND];
            cuckoo_slots((uint32_t)v, nsl, cs);
            uint32_t t = cs[0];
            for (int s = 0;; ++s) {
                const uint64_t old = atomicExch(reinterpret_cast<unsigned long long *>(&slots[t]),
                                                (unsigned long long)v);
                if (old == 0ull) break;
                if (s == MAX_EVICT) {
                    const uint32_t k = atomicAdd(&flags[1], 1u);
                    if (k < (uint32_t)STASH) stash[k] = old; else flags[2] = 1u;
                    break;
                }
                cuckoo_slots((uint32_t)old, nsl, cs);
                uint32_t nx = cs[0];
#pragma unroll
                for (int j = NCAND - 2; j >= 0; --j) nx = cs[j] == t ? cs[j + 1] : nx;
                t = nx;
                v = old;
            }
        }
    }
    lds_barrier();
    PSTAMP(3);
    if (flags[2]) {
        if (tid == 0) atomicOr(a.status, OA_STATUS_PART_OVERFLOW);
        return;
    }
    // every current entry's state word starts as angle 0 | its sign (an entered
    // particle keeps it, calc_angles :348-349); a match overwrites it below
#pragma unroll
    for (int u = 0; u < CU; ++u) {
        const uint32_t i = (uint32_t)u * PART_WG + tid;
        if (i < nc) mlds[i] = (cpw[u] >> 30) << 16;
    }
    lds_barrier();
    const bool nonuniform = KB == 8 && flags[3] != 0u;
    const uint32_t nstash = min(flags[1], (uint32_t)STASH);
    uint32_t *cmeta = a.pmeta_cur + cb;
    // record chunks of this item: counters in pcnt from gp[8], slots at the item's
    // scratch base + chunk * RCHUNK
    uint32_t *rcnt = a.pcnt + gp[8];
    ID *scr_ids = static_cast<ID *>(a.scratch_ids);
    const uint64_t hiw = KB == 4 ? (uint64_t)a.part_hi << 32 : 0ull;
    // previous entries, PU per thread: lookups, then the gathers of the matched current
    // r̂ (the partition's own bucket entries), then the angle and state-word arithmetic
    const Rsrc rcr = make_rsrc(crh0, PE * 3 * (uint32_t)sizeof(TD));
    for (uint32_t q = 0; q < nq; ++q) {
        const uint32_t np = qcnt[q0 + q];
        for (uint32_t j0 = 0; j0 < np; j0 += (uint32_t)PART_WG * PU) {
            if (j0 || q) load_prev(q, np, j0);
            uint32_t hit[PU];
            V3<TD> crh[PU];                             // a miss reads past the buffer: 0
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                hit[u] = 0xFFFFFFFFu;
                do {
                    const uint32_t j = j0 + (uint32_t)u * PART_WG + tid;
                    const uint64_t key = (uint64_t)qkey[u] | hiw;
                    const uint32_t lo = (uint32_t)key;
                    if (j >= np || (KB == 8 && !nonuniform && (uint32_t)(key >> 32) != hi0)) break;
                    if (filt && part_of(key, K) != (uint32_t)pp) break;
                    uint32_t cs[NCAND];
                    cuckoo_slots(lo, nsl, cs);
                    uint64_t m = 0ull;
#pragma unroll
                    for (int c = 0; c < NCAND; ++c) {
                        const uint64_t v = slots[cs[c]];
                        if (!m && v && (uint32_t)v == lo && slot_pos(v) < nc &&
                            (!nonuniform || (uint64_t)ck[slot_pos(v)] == key))
                            m = v;
                    }
                    for (uint32_t e = 0; !m && e < nstash; ++e) {
                        const uint64_t v = stash[e];
                        if ((uint32_t)v == lo && (!nonuniform || (uint64_t)ck[slot_pos(v)] == key)) m = v;
                    }
                    if (m) hit[u] = slot_pos(m) | ((slot_meta(m) >> 16) << 30);
                } while (0);
                // the gather of the matched current r̂ issued right after its lookup, so
                // it is in flight through the next entries' lookups (1 % on configs[1])
                crh[u] = bld3<TD, 0>(rcr, hit[u] != 0xFFFFFFFFu
                                              ? (hit[u] & 0x3FFFFFFFu) * 3 * (uint32_t)sizeof(TD)
                                              : 0x7FFFFFF0u);
            }
#ifdef OA_DIAG_PART_NOGATHER
            // diagnostic: the matched current r̂ not used (wrong angles), as if no gather
#pragma unroll
            for (int u = 0; u < PU; ++u) crh[u] = qrh[u];
#endif
            uint16_t rang[PU];
            uint32_t rslot[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                rslot[u] = 0xFFFFFFFFu;                 // staged (or none)
                if (hit[u] == 0xFFFFFFFFu) continue;
                const uint32_t sc = hit[u] >> 30, sp = qmeta[u] >> 16;
                // strict sign test (:311-314), arccos of the r̂ dot product (:324-325),
                // f16 + change rounded once, reset at an apsis (:342-349)
                const bool flag = a.mode == OA_MODE_PERICENTRIC ? (sp == 2u && sc == 1u)
                                                                : (sp == 1u && sc == 2u);
                const TD dt = dot3(qrh[u].x, qrh[u].y, qrh[u].z, crh[u].x, crh[u].y, crh[u].z);
                const uint16_t acc = angle_add((uint16_t)(qmeta[u] & 0xFFFFu), acos_td(dt));
                mlds[hit[u] & 0x3FFFFFFFu] = (uint32_t)(flag ? 0u : acc) | (sc << 16);
                rang[u] = acc;
                // an inherited set's position words carry the sign in bits 30-31; the
                // record is staged in LDS (its slot is claimed per chunk below), or,
                // past the stage's capacity, claims its slot with a global atomic
                if (flag) {
                    const uint32_t p = qpos[u] & 0x3FFFFFFFu;
                    const uint32_t e = atomicAdd(nrec, 1u);
                    if (e < (uint32_t)PART_RB) {
                        rbuf[2 * e] = (uint64_t)qkey[u] | hiw;
                        rbuf[2 * e + 1] = (uint64_t)p | ((uint64_t)acc << 32);
                    } else {
                        rslot[u] = atomicAdd(&rcnt[p >> RCHUNK_LOG2], 1u);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                if (rslot[u] == 0xFFFFFFFFu) continue;
                const uint32_t p = qpos[u] & 0x3FFFFFFFu;
                const int64_t s = gp[11] + (int64_t)(p & ~(uint32_t)(RCHUNK - 1)) + rslot[u];
                scr_ids[s] = (ID)((uint64_t)qkey[u] | hiw);
                a.scratch_ang[s] = rang[u];
                a.scratch_rk[s] = (uint16_t)(p & (RCHUNK - 1));
            }
            if (j0 == 0 && q == 0) PSTAMP(4);
        }
    }
    // barriers on LDS traffic only from here: the state words' stores go out first and
    // stay in flight through the record claims (a full __syncthreads would wait for them)
    lds_barrier();
    PSTAMP(6);
    // the partition's state words leave as one coalesced run
    for (uint32_t i = tid; i < nc; i += PART_WG) cmeta[i] = mlds[i];
    // the staged records: ranks within their chunks from LDS counters over the dead
    // table, one global atomic per touched chunk for the chunk's slots, then the stores
    // (a halo with more chunks than the counters claims per record)
    const uint32_t nst = min(*nrec, (uint32_t)PART_RB);
    const uint32_t nch = (uint32_t)gp[12];
    uint32_t *lc = reinterpret_cast<uint32_t *>(slots);
    const bool lds_ranks = nch <= 2u * PS;
    if (nst) {
        if (lds_ranks)
            for (uint32_t c = tid; c < nch; c += PART_WG) lc[c] = 0u;
        lds_barrier();
        for (uint32_t e = tid; e < nst; e += PART_WG) {
            const uint32_t c = (uint32_t)rbuf[2 * e + 1] >> RCHUNK_LOG2;
            const uint32_t r = lds_ranks ? atomicAdd(&lc[c], 1u) : atomicAdd(&rcnt[c], 1u);
            rbuf[2 * e + 1] |= (uint64_t)r << 48;
        }
        lds_barrier();
        if (lds_ranks)
            for (uint32_t c = tid; c < nch; c += PART_WG) {
                const uint32_t n = lc[c];
                if (n) lc[c] = atomicAdd(&rcnt[c], n);
            }
        lds_barrier();
        for (uint32_t e = tid; e < nst; e += PART_WG) {
            const uint64_t w = rbuf[2 * e + 1];
            const uint32_t p = (uint32_t)w, c = p >> RCHUNK_LOG2;
            const uint32_t slot = (uint32_t)(w >> 48) + (lds_ranks ? lc[c] : 0u);
            const int64_t s = gp[11] + (int64_t)c * RCHUNK + slot;
            scr_ids[s] = (ID)rbuf[2 * e];
            a.scratch_ang[s] = (uint16_t)(w >> 32);
            a.scratch_rk[s] = (uint16_t)(p & (RCHUNK - 1));
        }
    }
    // the work-group's record count: one pair of device atomics (halo and item counts)
    if (tid == 0 && *nrec) {
        atomicAdd(&a.halo_count[gp[13]], (int32_t)*nrec);
        atomicAdd(&a.item_count[gi], (int32_t)*nrec);
    }
    PSTAMP(5);
}

// A bucket set back to position order (the state arrays of the snapshot it holds):
// one work-group per (halo row, partition) of plist; rows: base, K, counter index,
// block offset per halo.
template <typename TD>
__global__ __launch_bounds__(256) void k_part_unbucket(const oa_unbucket_args a) {
    const int32_t r = a.plist[2 * blockIdx.x], p = a.plist[2 * blockIdx.x + 1];
    if (r < 0) return;
    const int64_t *rw = a.rows + 4 * (int64_t)r;
    const uint32_t cap = (uint32_t)a.cap;
    uint32_t n = a.bcnt[rw[2] + p];
    n = n < cap ? n : cap;
    const int64_t o0 = rw[0] + (int64_t)p * cap, dst0 = rw[3];
    const TD *brh = static_cast<const TD *>(a.brh);
    TD *rh = static_cast<TD *>(a.rhat_out);
    for (uint32_t e = threadIdx.x; e < n; e += 256) {
        const int64_t o = o0 + e;
        const int64_t d = dst0 + (a.bpos[o] & 0x3FFFFFFFu);
        a.meta_out[d] = a.bmeta[o];
        rh[3 * d] = brh[3 * o]; rh[3 * d + 1] = brh[3 * o + 1]; rh[3 * d + 2] = brh[3 * o + 2];
    }
}

template <typename TX, typename TV, typename TD, int IDB, int KB>
int launch_part_k(const oa_step_args &a, hipStream_t st) {
    // previous chunks to scatter: those of halos without an inherited set (gchunk3)
    const int64_t n_scat = a.n_gchunk1 + (a.gchunk3 ? a.n_gchunk3 : a.n_gchunk2);
    if (n_scat > 0) {
        auto k = k_part_scatter<TX, TV, TD, IDB, KB>;
        const int64_t lds = scat_lds_bytes(a.part_kmax, (int)sizeof(TD), KB);
        if (int rc = set_lds(k, lds)) return rc;
        hipLaunchKernelGGL(k, dim3((unsigned)n_scat), dim3(SCAT_WG), (size_t)lds,
                           st, a, make_frame_k(a));
        if (int rc = check_launch("k_part_scatter")) return rc;
    }
    if (a.n_parts > 0) {
        auto k = k_part_join<TD, IDB, KB>;
        const int64_t lds = part_lds_bytes(a.part_e, a.part_slots);
        if (int rc = set_lds(k, lds)) return rc;
        hipLaunchKernelGGL(k, dim3((unsigned)a.n_parts), dim3(PART_WG), (size_t)lds, st, a);
        if (int rc = check_launch("k_part_join")) return rc;
    }
    return OA_OK;
}

template <typename TX, typename TV, typename TD, int IDB>
int launch_part(const oa_step_args &a, hipStream_t st) {
    if (hipMemsetAsync(a.pcnt, 0, (size_t)a.n_pcnt * 4, st) != hipSuccess)
        return fail(OA_E_LAUNCH, "oa_step: partition / record counters reset");
    // 4-byte IDs are their own low words
    if (IDB == 4 || a.part_key4) return launch_part_k<TX, TV, TD, IDB, 4>(a, st);
    return launch_part_k<TX, TV, TD, IDB, IDB>(a, st);
}

template <typename TX, typename TV, typename TD, int IDB, bool COMPARE, bool OTF>
int launch_big(const oa_step_args &a, hipStream_t st) {
    if constexpr (COMPARE && !OTF) {
        if (a.n_parts > 0) return launch_part<TX, TV, TD, IDB>(a, st);
    }
    if (a.n_gchunk1 > 0) {
        hipLaunchKernelGGL((k_big_frame<TX, TV, TD, IDB, COMPARE, OTF>), dim3((unsigned)a.n_gchunk1),
                           dim3(BIG_WG), 0, st, a, make_frame_k(a));
        if (int rc = check_launch("k_big_frame")) return rc;
    }
    if (COMPARE && a.n_gchunk2 > 0) {
        hipLaunchKernelGGL((k_big_join<TD, IDB, OTF>), dim3((unsigned)a.n_gchunk2), dim3(BIG_WG), 0,
                           st, a);
        if (int rc = check_launch("k_big_join")) return rc;
    }
    return OA_OK;
}

}  // namespace

// The step launchers of the three dtype plans (oa_step), one unit each in the split build.
int oa_step_plan_f32(const oa_step_args &a, hipStream_t st);    // float32 coordinates, r̂
int oa_step_plan_f32d(const oa_step_args &a, hipStream_t st);   // float32 coordinates, f64 r̂
int oa_step_plan_f64(const oa_step_args &a, hipStream_t st);    // float64 coordinates, r̂
#if OA_TU == 0 || OA_TU == 1
int oa_step_plan_f32(const oa_step_args &a, hipStream_t st) { return launch_step_v<float, float>(a, st); }
#endif
#if OA_TU == 0 || OA_TU == 2
int oa_step_plan_f32d(const oa_step_args &a, hipStream_t st) { return launch_step_v<float, double>(a, st); }
#endif
#if OA_TU == 0 || OA_TU == 3
int oa_step_plan_f64(const oa_step_args &a, hipStream_t st) { return launch_step_v<double, double>(a, st); }
#endif

#if OA_TU <= 0
// ------------------------------------------------------------------ sharded output
// One rank's apsis records to their final positions in the output every rank maps
// (sharding.ShardedEngine.fetch_async).  The destination is page-locked host memory:
// a rank's records of one halo are one run of consecutive positions, so a wave's stores
// cover consecutive bytes and cross PCIe as full lines.  Four records per thread, every
// load issued before the stores.
template <typename ID>
__global__ __launch_bounds__(256) void k_place_records(const ID *ids, const uint16_t *ang,
                                                       const int64_t *dst, int64_t n,
                                                       ID *out_ids, uint16_t *out_ang,
                                                       int64_t cap, int32_t *status) {
    constexpr int U = 4;
    const int64_t i0 = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    ID v[U];
    uint16_t g[U];
    int64_t d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * 256, ic = i < n ? i : n - 1;
        v[u] = ids ? __builtin_nontemporal_load(ids + ic) : (ID)0;
        g[u] = ang ? __builtin_nontemporal_load(ang + ic) : (uint16_t)0;
        d[u] = __builtin_nontemporal_load(dst + ic);
    }
    bool bad = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (i0 + u * 256 >= n) break;
        if (d[u] < 0 || d[u] >= cap) { bad = true; continue; }
        if (out_ids) out_ids[d[u]] = v[u];
        if (out_ang) out_ang[d[u]] = g[u];
    }
    if (bad && status) atomicAdd(status, 1);
}

// A step's status word and record count into page-locked host words (oa_post_status):
// the host's settle then waits only for this stream, not for a copy engine that may be
// busy with an earlier step's records.  Two lanes, two vector stores, then a
// system-scope fence.
__global__ __launch_bounds__(64) void k_post_status(const int32_t *status, const int64_t *total,
                                                    int32_t *h_status, int64_t *h_total) {
    const int t = threadIdx.x;
    if (t == 0) h_status[0] = status[0];
    else if (t == 1) h_total[0] = total[0];
    __threadfence_system();
}

// Bytes from a device-accessible address (a page-locked staging block, oa_host_register)
// into device memory by a kernel on `stream` (oa_copy_bytes): a step's host tables reach
// the device without a copy engine, whose queue may hold an earlier step's records D2H
// for milliseconds.  16-byte lanes, grid-stride; block 0 copies the tail bytes.
__global__ __launch_bounds__(256) void k_copy_bytes(const uint8_t *src, uint8_t *dst, int64_t n) {
    const int64_t n16 = n >> 4, stride = (int64_t)gridDim.x * 256;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) d4[i] = s4[i];
    if (blockIdx.x == 0)
        for (int64_t i = (n16 << 4) + threadIdx.x; i < n; i += 256) dst[i] = src[i];
}

// Error channel shared with the other units (orbit_post.hip, the step-plan units):
// nullptr clears the message, anything else becomes oa_last_error().
void oa_internal_error(const char *msg) {
    if (!msg) { g_err[0] = 0; return; }
    snprintf(g_err, sizeof(g_err), "%s", msg);
}

extern "C" {

int oa_abi_version(void) { return OA_ABI_VERSION; }

int32_t oa_build_info(int32_t which) {
    switch (which) {
        case 0: return WG;
        case 1: return HMAX;
        case 2: return UNR1;
        case 3: return KROWS;
        case 4: return PART_E;
        case 5: return PART_KMAX;
        case 6: return GPART_W;
        case 7: return RCHUNK;
        default: return -1;
    }
}

int64_t oa_struct_size(int32_t which) {
    switch (which) {
        case 0: return sizeof(oa_halo);
        case 1: return sizeof(oa_item);
        case 2: return sizeof(oa_step_args);
        case 3: return sizeof(oa_compact_args);
        case 4: return sizeof(oa_unbucket_args);
        default: return -1;
    }
}

const char *oa_last_error(void) { return g_err; }

int64_t oa_part_lds_bytes(int32_t entries, int32_t slots) {
    return part_lds_bytes(entries, slots);
}

int64_t oa_step_lds_bytes(int32_t entries, int32_t slots, int32_t dx_f64) {
    return step_lds_bytes(entries, slots, dx_f64 ? 8 : 4);
}

// Host-side item plan: greedy packing of consecutive halos, O(n_halos).
int64_t oa_plan_items(const int64_t *cur_off, const int64_t *cur_cnt, const int64_t *prev_cnt,
                      const int64_t *out_slot, int64_t n_halos, int64_t entries, int64_t slots,
                      int64_t hmax, int64_t max_pv, oa_item *items, int64_t cap,
                      int64_t *n_small, int64_t *scratch) {
    g_err[0] = 0;
    if (n_halos < 0 || entries < 0 || slots < 0 || hmax < 1 || max_pv < 0 || !n_small ||
        !scratch || (n_halos > 0 && (!cur_off || !cur_cnt || !prev_cnt || !items)))
        return fail(OA_E_ARG, "oa_plan_items: bad arguments");
    if (n_halos > INT32_MAX) return fail(OA_E_ARG, "oa_plan_items: more than 2^31 halos");
    auto pv = [&](int64_t j) { const int64_t p = prev_cnt[j] > 0 ? prev_cnt[j] : 0; return (p + 63) / 64 * 64; };
    auto big = [&](int64_t j) { return cur_cnt[j] > entries || pv(j) > max_pv; };
    auto slot0 = [&](int64_t h0, int64_t h1) -> int32_t {
        if (out_slot)
            for (int64_t j = h0; j < h1; ++j)
                if (out_slot[j] >= 0) return (int32_t)out_slot[j];
        return -1;
    };
    int64_t n = 0, sc = 0, ng = 0;
    for (int64_t j = 0; j < n_halos;) {                 // packed items
        if (cur_cnt[j] < 0) return fail(OA_E_ARG, "oa_plan_items: negative block size");
        if (big(j)) { ++j; ++ng; continue; }
        const int64_t h0 = j;
        int64_t tot = 0, ptot = 0, nj = 0;
        while (j < n_halos && j - h0 < hmax && !big(j) && tot + cur_cnt[j] <= entries &&
               ptot + pv(j) <= max_pv) {
            tot += cur_cnt[j];
            ptot += pv(j);
            if (prev_cnt[j] > 0) nj += cur_cnt[j];
            ++j;
        }
        if (n >= cap) return fail(OA_E_ARG, "oa_plan_items: more than cap items");
        const int64_t nsl = 2 * nj + 64 < slots ? 2 * nj + 64 : slots;   // load <= 1/2 if it fits
        items[n] = oa_item{(int32_t)h0, (int32_t)j, slot0(h0, j), (int32_t)tot, sc, ptot,
                           cur_off[h0], (int32_t)nsl, 0};
        sc += ptot;                                    // one 64-slot segment per row
        ++n;
    }
    *n_small = n;
    if (n + ng > cap) return fail(OA_E_ARG, "oa_plan_items: more than cap items");
    for (int64_t j = 0; j < n_halos; ++j) {             // global (large-halo) items
        if (!big(j)) continue;
        items[n++] = oa_item{(int32_t)j, (int32_t)(j + 1), slot0(j, j + 1), 0, sc, pv(j),
                             cur_off[j], 0, 0};
        sc += pv(j);
    }
    *scratch = sc;
    return n;
}

int oa_host_register(void *host, int64_t bytes, void **device_ptr) {
    g_err[0] = 0;
    if (!host || bytes <= 0 || !device_ptr) return fail(OA_E_ARG, "oa_host_register: bad arguments");
    hipError_t e = hipHostRegister(host, (size_t)bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) return fail(OA_E_DEVICE, "hipHostRegister: %s", hipGetErrorString(e));
    e = hipHostGetDevicePointer(device_ptr, host, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(host);
        return fail(OA_E_DEVICE, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
    }
    return OA_OK;
}

int oa_host_unregister(void *host) {
    g_err[0] = 0;
    if (!host) return fail(OA_E_ARG, "oa_host_unregister: null");
    const hipError_t e = hipHostUnregister(host);
    if (e != hipSuccess) return fail(OA_E_DEVICE, "hipHostUnregister: %s", hipGetErrorString(e));
    return OA_OK;
}

namespace {
struct HostFlag { int64_t *addr; int64_t value; };
void host_flag_cb(void *p) {
    HostFlag *f = static_cast<HostFlag *>(p);
    __atomic_store_n(f->addr, f->value, __ATOMIC_RELEASE);
    delete f;
}
}  // namespace

int oa_stream_set_flag(void *stream, int64_t *host_addr, int64_t value) {
    g_err[0] = 0;
    if (!host_addr) return fail(OA_E_ARG, "oa_stream_set_flag: null address");
    HostFlag *f = new HostFlag{host_addr, value};
    const hipError_t e = hipLaunchHostFunc(reinterpret_cast<hipStream_t>(stream), host_flag_cb, f);
    if (e != hipSuccess) {
        delete f;
        return fail(OA_E_LAUNCH, "hipLaunchHostFunc: %s", hipGetErrorString(e));
    }
    return OA_OK;
}

int oa_copy_bytes(const void *src, void *dst, int64_t bytes, void *stream) {
    g_err[0] = 0;
    if (bytes < 0 || (bytes > 0 && (!src || !dst)) ||
        (((uintptr_t)src | (uintptr_t)dst) & 15u))
        return fail(OA_E_ARG, "oa_copy_bytes: bad arguments (16-byte aligned pointers)");
    if (bytes == 0) return OA_OK;
    const int64_t n16 = bytes >> 4;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n16 + 255) / 256, 512));
    hipLaunchKernelGGL(k_copy_bytes, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       static_cast<const uint8_t *>(src), static_cast<uint8_t *>(dst), bytes);
    return check_launch("k_copy_bytes");
}

int oa_post_status(const int32_t *status, const int64_t *total, int32_t *host_status,
                   int64_t *host_total, void *stream) {
    g_err[0] = 0;
    if (!status || !total || !host_status || !host_total)
        return fail(OA_E_ARG, "oa_post_status: null pointer");
    hipLaunchKernelGGL(k_post_status, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                       status, total, host_status, host_total);
    return check_launch("k_post_status");
}

int oa_place_records(const void *ids, const uint16_t *ang, const int64_t *dst, int64_t n,
                     int32_t id_bytes, void *out_ids, uint16_t *out_ang, int64_t cap,
                     int32_t *status, void *stream) {
    g_err[0] = 0;
    if (n <= 0) return OA_OK;
    if (!dst || cap < 0 || (id_bytes != 4 && id_bytes != 8) || (!ids != !out_ids) ||
        (!ang != !out_ang) || (!ids && !ang))
        return fail(OA_E_ARG, "oa_place_records: bad arguments");
    const unsigned grid = (unsigned)((n + 1023) / 1024);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (id_bytes == 8)
        hipLaunchKernelGGL(k_place_records<uint64_t>, dim3(grid), dim3(256), 0, st,
                           static_cast<const uint64_t *>(ids), ang, dst, n,
                           static_cast<uint64_t *>(out_ids), out_ang, cap, status);
    else
        hipLaunchKernelGGL(k_place_records<uint32_t>, dim3(grid), dim3(256), 0, st,
                           static_cast<const uint32_t *>(ids), ang, dst, n,
                           static_cast<uint32_t *>(out_ids), out_ang, cap, status);
    return check_launch("k_place_records");
}

int oa_build_halos(const int64_t *cur_off, const int64_t *cur_cnt, const int64_t *prev_off,
                   const int64_t *prev_cnt, const int64_t *out_slot, const double *centre,
                   const double *bulk, int64_t n, oa_halo *halos) {
    g_err[0] = 0;
    if (n < 0 || (n > 0 && (!cur_off || !cur_cnt || !prev_off || !prev_cnt || !out_slot ||
                            !centre || !halos)))
        return fail(OA_E_ARG, "oa_build_halos: bad arguments");
    for (int64_t j = 0; j < n; ++j) {
        oa_halo &h = halos[j];
        h.cur_off = cur_off[j];
        h.cur_cnt = cur_cnt[j];
        h.prev_off = prev_off[j];
        h.prev_cnt = prev_cnt[j];
        for (int d = 0; d < 3; ++d) {
            h.centre[d] = centre[3 * j + d];
            h.bulk[d] = bulk ? bulk[3 * j + d] : 0.0;
        }
        h.out_slot = out_slot[j];
        h.reserved = 0;
    }
    return OA_OK;
}

// Diagnostic builds (-DOA_STAMPS=1): copy the per-work-group phase stamps of the last
// oa_step launch (s_memrealtime, 100 MHz) to host memory; returns count or -1.
int64_t oa_debug_stamps(uint64_t *host, int64_t n) {
#if OA_STAMPS
    int64_t m = n < (int64_t)STAMP_MAX_WG * STAMP_N ? n : (int64_t)STAMP_MAX_WG * STAMP_N;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), m * sizeof(uint64_t)) != hipSuccess)
        return -1;
    return m;
#else
    (void)host; (void)n;
    return -1;
#endif
}

// Diagnostic builds: stamps of the large-halo partition kernels of the last oa_step
// (which = 0: k_part_join, 8 per work-group; 1: k_part_scatter, 2 per work-group).
int64_t oa_debug_part_stamps(int32_t which, uint64_t *host, int64_t n) {
#if OA_STAMPS
    const int64_t cap = (int64_t)STAMP_MAX_WG * PSTAMP_N;
    const int64_t m = n < cap ? n : cap;
    hipError_t e = which ? hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sstamps), m * sizeof(uint64_t))
                         : hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pstamps), m * sizeof(uint64_t));
    return e == hipSuccess ? m : -1;
#else
    (void)which; (void)host; (void)n;
    return -1;
#endif
}

int64_t oa_max_lds_bytes(void) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 65536;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
        return 65536;
    return v;
}

int oa_step(const oa_step_args *args, void *stream) {
    g_err[0] = 0;
    if (!args) return fail(OA_E_ARG, "oa_step: null args");
    const oa_step_args &a = *args;
    if (a.id_bytes != 4 && a.id_bytes != 8) return fail(OA_E_ARG, "id_bytes must be 4 or 8");
    if (!a.dx_f64 && a.coord_f64) return fail(OA_E_ARG, "dx dtype narrower than coordinates");
    if (!a.vb_f64 && a.vel_f64) return fail(OA_E_ARG, "v-bulk dtype narrower than velocities");
    if (a.wrap_f64 == 0 && a.dx_f64) return fail(OA_E_ARG, "float32 wrap with float64 dx");
    if (a.n_box_dims < 0 || a.n_box_dims > 3) return fail(OA_E_ARG, "n_box_dims out of range");
    if (a.mode != OA_MODE_PERICENTRIC && a.mode != OA_MODE_APOCENTRIC)
        return fail(OA_E_ARG, "bad mode");
    if (a.n_items > 0 && (a.lds_entries <= 0 || a.lds_entries > (int)MAX_POS + 1 ||
                          a.lds_entries > (a.dx_f64 || a.onthefly && a.coord_f64 ? STAGE_F64 : STAGE_F32) * WG ||
                          a.lds_slots <= a.lds_entries))
        return fail(OA_E_ARG, "bad lds_entries/lds_slots (entries <= %d (r̂ dtype) < slots)",
                    (a.dx_f64 ? STAGE_F64 : STAGE_F32) * WG);
    if (a.n_items + a.n_global_items > 0 &&
        (!a.halos || !a.ids || !a.coords || !a.vels || !a.rhat_out || !a.meta_out))
        return fail(OA_E_ARG, "null input/output pointer");
    if (a.compare && (!a.ids_prev || !a.rhat_prev || !a.meta_prev || !a.halo_count || !a.status ||
                      (a.n_items > 0 && (!a.scratch_ids || !a.scratch_ang || !a.item_count ||
                                         !a.seg_count))))
        return fail(OA_E_ARG, "null previous-state / scratch pointer");
    if (a.compare && a.scratch_pos && a.n_prev >= (int64_t)INT32_MAX)
        return fail(OA_E_ARG, "scratch_pos: previous state of 2^31 rows or more");
    if (a.onthefly && a.compare && (!a.angle_out || !a.matched_prev || !a.matched_cur))
        return fail(OA_E_ARG, "null on-the-fly output pointer");
    if (a.n_gchunk1 > 0 && (!a.gchunk1 || !a.gtab ||
                            (a.compare && !(a.n_parts > 0 && !a.onthefly) && !a.gkeys)))
        return fail(OA_E_ARG, "null large-halo table pointer");
    if (a.compare && a.n_gchunk2 > 0 && !a.gchunk2)
        return fail(OA_E_ARG, "null large-halo chunk pointer");
    const bool part = a.compare && !a.onthefly && a.n_parts > 0;
    if (part && (!a.prow || !a.gpart || !a.pkey_cur || !a.ppos_cur || !a.pmeta_cur ||
                 !a.prh_cur || !a.pcnt || !a.scratch_rk || a.n_pcnt < 1 ||
                 (a.id_bytes == 4 && a.part_hi != 0) ||
                 (a.n_gchunk2 > 0 && (!a.pkey_prev || !a.ppos_prev || !a.pmeta_prev ||
                                      !a.prh_prev)) || a.part_kmax < 1 ||
                 a.part_e < 64 || a.part_e > PART_E || a.part_e % 64 ||
                 a.part_slots <= a.part_e || a.part_slots > PART_S ||
                 a.part_kmax > PART_KMAX))
        return fail(OA_E_ARG, "bad large-halo partition arguments");
    if (a.onthefly && a.n_parts > 0)
        return fail(OA_E_ARG, "the partitioned large-halo path is not for on-the-fly steps");
    if (a.direct && (!a.compare || a.onthefly || a.n_global_items > 0 || !a.lookback ||
                     !a.offsets_out || !a.out_ids || !a.out_ang || !a.total_out ||
                     a.lb_epoch < 1 || a.lb_epoch > 0xFFFF || a.n_slots < 0))
        return fail(OA_E_ARG, "direct records: a packed-only compare step with look-back "
                              "words, epoch in [1, 65535] and output pointers");
    if (a.direct && a.n_items == 0) {
        // no item writes the (empty) output: offsets = [0], total = 0
        if (hipMemsetAsync(a.offsets_out, 0, 8, reinterpret_cast<hipStream_t>(stream)) != hipSuccess ||
            hipMemsetAsync(a.total_out, 0, 8, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
            return fail(OA_E_LAUNCH, "oa_step: empty direct output");
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (a.compare && a.n_global_items > 0) {
        if ((!part && hipMemsetAsync(a.gkeys, 0, (size_t)a.gtab_total * 16, st) != hipSuccess) ||
            hipMemsetAsync(a.item_count + a.n_items, 0, (size_t)a.n_global_items * 4, st) != hipSuccess)
            return fail(OA_E_LAUNCH, "oa_step: large-halo table reset");
    }
    if (a.onthefly) return a.coord_f64 ? oa_step_plan_f64(a, st) : oa_step_plan_f32(a, st);
    if (a.dx_f64) return a.coord_f64 ? oa_step_plan_f64(a, st) : oa_step_plan_f32d(a, st);
    return oa_step_plan_f32(a, st);
}

int oa_part_unbucket(const oa_unbucket_args *args, void *stream) {
    g_err[0] = 0;
    if (!args) return fail(OA_E_ARG, "oa_part_unbucket: null args");
    const oa_unbucket_args &a = *args;
    if (a.n_parts <= 0) return OA_OK;
    if (!a.bpos || !a.bmeta || !a.brh || !a.bcnt || !a.rows || !a.plist || !a.rhat_out ||
        !a.meta_out || a.cap < 1)
        return fail(OA_E_ARG, "oa_part_unbucket: null pointer / bad capacity");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (a.td_f64) hipLaunchKernelGGL(k_part_unbucket<double>, dim3((unsigned)a.n_parts), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_part_unbucket<float>, dim3((unsigned)a.n_parts), dim3(256), 0, st, a);
    return check_launch("k_part_unbucket");
}

int oa_compact(const oa_compact_args *args, void *stream) {
    g_err[0] = 0;
    if (!args) return fail(OA_E_ARG, "oa_compact: null args");
    const oa_compact_args &a = *args;
    if (a.id_bytes != 4 && a.id_bytes != 8) return fail(OA_E_ARG, "id_bytes must be 4 or 8");
    if (!a.offsets_out || !a.total_out || (a.n_slots > 0 && !a.halo_count))
        return fail(OA_E_ARG, "null output pointer");
    if (!a.out_pos != !a.scratch_pos) return fail(OA_E_ARG, "out_pos needs scratch_pos");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_scan_slots, dim3(1), dim3(1024), 0, st, a.halo_count, a.n_slots,
                       a.offsets_out, a.total_out);
    if (int rc = check_launch("k_scan_slots")) return rc;
    if (a.n_gchunks < 0 || (a.n_gchunks > 0 && !a.gchunks))
        return fail(OA_E_ARG, "oa_compact: n_gchunks without gchunks");
    const int32_t n_direct = a.gchunks ? a.n_packed : a.n_items;   // per-item launches
    if (n_direct > 0) {
        if (a.id_bytes == 8) hipLaunchKernelGGL(k_gather_items<8>, dim3(n_direct), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_gather_items<4>, dim3(n_direct), dim3(256), 0, st, a);
        if (int rc = check_launch("k_gather_items")) return rc;
    }
    if (a.chunk_count && (!a.gchunks || !a.scratch_rk))
        return fail(OA_E_ARG, "oa_compact: chunk_count needs gchunks and scratch_rk");
    if (a.gchunks && a.n_gchunks > 0 && a.chunk_count) {
        if (a.id_bytes == 8) hipLaunchKernelGGL(k_gather_recs<8>, dim3(a.n_gchunks), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_gather_recs<4>, dim3(a.n_gchunks), dim3(256), 0, st, a);
        if (int rc = check_launch("k_gather_recs")) return rc;
    } else if (a.gchunks && a.n_gchunks > 0) {
        if (a.id_bytes == 8) hipLaunchKernelGGL(k_gather_chunks<8>, dim3(a.n_gchunks), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_gather_chunks<4>, dim3(a.n_gchunks), dim3(256), 0, st, a);
        if (int rc = check_launch("k_gather_chunks")) return rc;
    }
    return OA_OK;
}

int oa_bulk_velocity(const void *vels, int32_t vel_f64, const void *masses, int32_t mass_f64,
                     oa_halo *halos, const int32_t *halo_list, int32_t n_list, void *stream) {
    g_err[0] = 0;
    if (n_list <= 0) return OA_OK;
    if (!vels || !halos || !halo_list) return fail(OA_E_ARG, "oa_bulk_velocity: null pointer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 g(n_list), b(64);
    if (!masses) {
        if (vel_f64) hipLaunchKernelGGL((k_bulk<double, double, false>), g, b, 0, st,
                                        (const double *)vels, (const double *)nullptr, halos, halo_list);
        else hipLaunchKernelGGL((k_bulk<float, float, false>), g, b, 0, st,
                                (const float *)vels, (const float *)nullptr, halos, halo_list);
    } else if (vel_f64 && mass_f64) {
        hipLaunchKernelGGL((k_bulk<double, double, true>), g, b, 0, st,
                           (const double *)vels, (const double *)masses, halos, halo_list);
    } else if (vel_f64) {
        hipLaunchKernelGGL((k_bulk<double, float, true>), g, b, 0, st,
                           (const double *)vels, (const float *)masses, halos, halo_list);
    } else if (mass_f64) {
        hipLaunchKernelGGL((k_bulk<float, double, true>), g, b, 0, st,
                           (const float *)vels, (const double *)masses, halos, halo_list);
    } else {
        hipLaunchKernelGGL((k_bulk<float, float, true>), g, b, 0, st,
                           (const float *)vels, (const float *)masses, halos, halo_list);
    }
    return check_launch("k_bulk");
}

int64_t oa_match_workspace_bytes(int64_t n_cur) {
    uint64_t cap = 64;
    while (cap < 2 * (uint64_t)(n_cur > 0 ? n_cur : 1)) cap <<= 1;
    return (int64_t)(cap * (8 + 4));
}

int oa_match_ids(const void *ids_cur, int64_t n_cur, const void *ids_prev, int64_t n_prev,
                 int32_t id_bytes, void *workspace, int64_t *match_out, void *stream) {
    g_err[0] = 0;
    if (id_bytes != 4 && id_bytes != 8) return fail(OA_E_ARG, "id_bytes must be 4 or 8");
    if (n_cur < 0 || n_prev < 0 || n_cur >= (int64_t)0xFFFFFFFF)
        return fail(OA_E_ARG, "oa_match_ids: bad sizes");
    if (n_prev > 0 && (!ids_prev || !match_out || !workspace || (n_cur > 0 && !ids_cur)))
        return fail(OA_E_ARG, "oa_match_ids: null pointer");
    if (n_prev == 0) return OA_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    uint64_t cap = 64;
    while (cap < 2 * (uint64_t)(n_cur > 0 ? n_cur : 1)) cap <<= 1;
    uint64_t *keys = static_cast<uint64_t *>(workspace);
    uint32_t *vals = reinterpret_cast<uint32_t *>(keys + cap);
    if (hipMemsetAsync(vals, 0, cap * 4, st) != hipSuccess)
        return fail(OA_E_LAUNCH, "oa_match_ids: memset");
    if (n_cur > 0) {
        dim3 g((unsigned)((n_cur + 255) / 256));
        if (id_bytes == 8) hipLaunchKernelGGL(k_match_insert<8>, g, dim3(256), 0, st, ids_cur, n_cur, keys, vals, cap);
        else hipLaunchKernelGGL(k_match_insert<4>, g, dim3(256), 0, st, ids_cur, n_cur, keys, vals, cap);
        if (int rc = check_launch("k_match_insert")) return rc;
    }
    dim3 g((unsigned)((n_prev + 255) / 256));
    if (id_bytes == 8) hipLaunchKernelGGL(k_match_probe<8>, g, dim3(256), 0, st, ids_prev, n_prev, keys, vals, cap, match_out);
    else hipLaunchKernelGGL(k_match_probe<4>, g, dim3(256), 0, st, ids_prev, n_prev, keys, vals, cap, match_out);
    return check_launch("k_match_probe");
}

int oa_compare_pairs(const int64_t *match, int64_t n_prev, const double *vr, const double *vr_prev,
                     const void *rhat, const void *rhat_prev, int32_t td_f64, int32_t mode,
                     uint8_t *flag_out, void *change_out, void *stream) {
    g_err[0] = 0;
    if (mode != OA_MODE_PERICENTRIC && mode != OA_MODE_APOCENTRIC) return fail(OA_E_ARG, "bad mode");
    if (n_prev <= 0) return OA_OK;
    if (!match || !vr_prev || !rhat_prev || !flag_out || !change_out)
        return fail(OA_E_ARG, "oa_compare_pairs: null pointer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 g((unsigned)((n_prev + 255) / 256));
    if (td_f64)
        hipLaunchKernelGGL(k_compare_pairs<double>, g, dim3(256), 0, st, match, n_prev, vr, vr_prev,
                           static_cast<const double *>(rhat), static_cast<const double *>(rhat_prev),
                           mode, flag_out, static_cast<double *>(change_out));
    else
        hipLaunchKernelGGL(k_compare_pairs<float>, g, dim3(256), 0, st, match, n_prev, vr, vr_prev,
                           static_cast<const float *>(rhat), static_cast<const float *>(rhat_prev),
                           mode, flag_out, static_cast<float *>(change_out));
    return check_launch("k_compare_pairs");
}

int oa_angle_add(const uint16_t *angles_prev, const void *change, int64_t n, int32_t td_f64,
                 uint16_t *out, void *stream) {
    g_err[0] = 0;
    if (n <= 0) return OA_OK;
    if (!angles_prev || !change || !out) return fail(OA_E_ARG, "oa_angle_add: null pointer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 g((unsigned)((n + 255) / 256));
    if (td_f64)
        hipLaunchKernelGGL(k_angle_add<double>, g, dim3(256), 0, st, angles_prev,
                           static_cast<const double *>(change), n, out);
    else
        hipLaunchKernelGGL(k_angle_add<float>, g, dim3(256), 0, st, angles_prev,
                           static_cast<const float *>(change), n, out);
    return check_launch("k_angle_add");
}

}  // extern "C"
#endif  // OA_TU <= 0
