// orbit_hip.hip — MI355X (gfx950 / CDNA4) kernels for the per-snapshot orbit-tagging
// hot path of s-balu/nbody-orbit-analysis, behind the C ABI of include/orbit_hip.h.
//
// Reference path (paths under /root/reference/orbitanalysis/):
//   region_frame               track_orbits.py:247-290    -> k_step phase 1
//   compare_radial_velocities  track_orbits.py:293-327    -> k_step phase 2
//   calc_angles                track_orbits.py:330-351    -> k_step phase 2
//   result assembly            track_orbits.py:199-227    -> k_scan_slots, k_gather_*
//   bulk velocity (sum/mean)   track_orbits.py:262-284    -> k_bulk
//
// Design: one work-group per *item* (a run of consecutive halos whose
// current blocks fit the LDS hash table, or one hash bucket of a halo too large for
// it).  Phase 1 streams the item's current blocks (ids, AoS x, AoS v) once,
// computes the frame in registers, writes the particle record {r̂, meta} and inserts
// (halo, id) -> local index into an LDS open-addressing table.  Phase 2 streams the
// progenitor blocks (ids, records), probes the table, gathers the just-written
// current record from L2, applies the strict sign test and the arccos angle update
// and compacts apsis records in previous-block order with wave ballots.  Every
// input byte is read from HBM once; no sort, no global hash table.
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

namespace {

constexpr int WG = 1024;            // k_step work-group (16 waves)
constexpr int NWAVE = WG / 64;
constexpr int HMAX = 128;           // halos per item
constexpr int UNR = 2;              // particles per thread per loop trip
constexpr int BULK_CHUNK = 8192;    // numpy pairwise-sum buffer chunk

thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(OA_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
    return OA_OK;
}

// ------------------------------------------------------------------ records
template <typename TD> struct Rec;
template <> struct __attribute__((aligned(16))) Rec<float> { float r[3]; uint32_t meta; };
template <> struct __attribute__((aligned(16))) Rec<double> { double r[3]; uint32_t meta, pad; };

template <typename T> struct V3 { T x, y, z; };

template <typename T>
__device__ __forceinline__ V3<T> ld3(const T *p, int64_t i) {
    const T *q = p + 3 * i;
    return V3<T>{q[0], q[1], q[2]};
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
// numpy's float32 arccos is not correctly rounded (SIMD); the closest portable
// choice is the correctly rounded one: float64 acos rounded to float32.
__device__ __forceinline__ float acos_td(float x) { return (float)acos((double)x); }

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
__device__ __forceinline__ uint32_t slot_of(uint32_t lo, uint32_t hl, uint32_t nslots) {
    uint32_t h = fmix32(lo ^ (hl * 0x9E3779B9u) ^ 0xA511E9B3u);
    return (uint32_t)(((uint64_t)h * nslots) >> 32);
}
__device__ __forceinline__ uint32_t bucket_of(uint32_t lo, uint32_t hi, uint32_t nb) {
    uint32_t h = fmix32(lo * 0x9E3779B1u + hi * 0x85EBCA77u + 0x27D4EB2Fu);
    return (uint32_t)(((uint64_t)h * nb) >> 32);
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
struct ItemHdr {
    int64_t cur_base;
    uint32_t nonuniform, hi0, nent, overflow;
    uint32_t nh, nseg, n_span, n_pv;
    uint32_t chunk_total, pad0, pad1, pad2;
    uint32_t wave_cnt[UNR * NWAVE];
    uint32_t wave_pre[UNR * NWAVE];
    uint32_t lstart[HMAX + 1];      // local start of each item halo's current block
    uint32_t vstart[HMAX + 1];      // virtual start of each progenitor segment
    int32_t seg_halo[HMAX];         // segment -> item-local halo
    int32_t halo_cnt[HMAX];         // apsis records per item halo
    int32_t has_prev[HMAX];
    int64_t seg_prev_off[HMAX];
    double cb[HMAX][6];             // centre[3], bulk[3]
};
constexpr int64_t HDR_BYTES = (sizeof(ItemHdr) + 255) & ~int64_t(255);

__host__ __device__ inline int64_t table_bytes(int entries, int slots, bool bucketed) {
    int64_t b = (int64_t)entries * 4 + (bucketed ? (int64_t)entries * 4 : 0) +
                (int64_t)((slots + 1) / 2) * 4;
    return (b + 15) & ~int64_t(15);
}

__device__ __forceinline__ uint32_t upper_find(const uint32_t *starts, uint32_t n, uint32_t x) {
    // largest k in [0, n) with starts[k] <= x  (starts non-decreasing, starts[0] = 0)
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void lds_insert(uint32_t *slotw, uint32_t nslots, uint32_t s,
                                           uint32_t val) {
    for (;;) {
        uint32_t wi = s >> 1, sh = (s & 1u) << 4;
        uint32_t cur = __hip_atomic_load(&slotw[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (;;) {
            if ((cur >> sh) & 0xFFFFu) break;       // occupied: next slot
            uint32_t prev = atomicCAS(&slotw[wi], cur, cur | (val << sh));
            if (prev == cur) return;
            cur = prev;
        }
        s = (s + 1 == nslots) ? 0u : s + 1;
    }
}

// ------------------------------------------------------------------ frame
// region_frame (track_orbits.py:247-290) for one particle; cb = centre[3], bulk[3].
template <typename TX, typename TV, typename TD>
__device__ __forceinline__ uint32_t frame(const V3<TX> &x, const V3<TV> &v, const double *cb,
                                          const oa_step_args &a, TD r[3]) {
    TD dx[3] = {(TD)x.x - (TD)cb[0], (TD)x.y - (TD)cb[1], (TD)x.z - (TD)cb[2]};
    // recenter_coordinates (utils.py:24-33): one strict wrap per dimension, in the
    // promoted dtype of (dx, box), cast back to dx's dtype
    for (int d = 0; d < 3; ++d) {
        if (d >= a.n_box_dims) break;
        if (a.wrap_f64) {
            double L = a.box[d], half = L / 2;
            double t = (double)dx[d];
            if (t > half) dx[d] = (TD)(t - L);
            t = (double)dx[d];
            if (t < -half) dx[d] = (TD)(t + L);
        } else {
            float L = (float)a.box[d], half = L / 2;
            float t = (float)dx[d];
            if (t > half) dx[d] = (TD)(t - L);
            t = (float)dx[d];
            if (t < -half) dx[d] = (TD)(t + L);
        }
    }
    // w = (v - bulk) + (H * dx) / (1 + z)   (:275-276, :283-284); H is a float64 scalar
    const TV vv[3] = {v.x, v.y, v.z};
    double w[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        double vb = a.vb_f64 ? (double)vv[d] - cb[3 + d]
                             : (double)((float)vv[d] - (float)cb[3 + d]);
        w[d] = vb + (a.H * (double)dx[d]) / a.one_plus_z;
    }
    // rads = sqrt(dot(dx, dx)); rhats = dx / rads; v_r = dot(w, rhats)   (:286-288)
    TD rr = sqrt(dot3(dx[0], dx[1], dx[2], dx[0], dx[1], dx[2]));
    r[0] = dx[0] / rr; r[1] = dx[1] / rr; r[2] = dx[2] / rr;
    double vr = dot3(w[0], w[1], w[2], (double)r[0], (double)r[1], (double)r[2]);
    return vr > 0.0 ? 1u : (vr < 0.0 ? 2u : 0u);
}

// ------------------------------------------------------------------ step kernel
template <typename TX, typename TV, typename TD, int IDB, bool BUCKETED>
__global__ __launch_bounds__(WG) void k_step(const oa_step_args a) {
    typedef typename IdT<IDB>::T ID;
    typedef Rec<TD> R;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    ItemHdr &H = *reinterpret_cast<ItemHdr *>(smem);
    const int nent_max = BUCKETED ? a.big_entries : a.lds_entries;
    const uint32_t nslots = (uint32_t)(BUCKETED ? a.big_slots : a.lds_slots);
    uint32_t *ids_lo = reinterpret_cast<uint32_t *>(smem + HDR_BYTES);
    uint32_t *lidx = BUCKETED ? ids_lo + nent_max : nullptr;
    uint32_t *slotw = (BUCKETED ? lidx : ids_lo) + nent_max;

    const oa_item it = (BUCKETED ? a.big_items : a.items)[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const ID *ids = reinterpret_cast<const ID *>(a.ids);
    const ID *ids_prev = reinterpret_cast<const ID *>(a.ids_prev);
    const TX *coords = reinterpret_cast<const TX *>(a.coords);
    const TV *vels = reinterpret_cast<const TV *>(a.vels);
    R *rec_out = reinterpret_cast<R *>(a.rec_out);
    const R *rec_prev = reinterpret_cast<const R *>(a.rec_prev);
    const bool compare = a.compare != 0;
    const uint32_t q = (uint32_t)it.bucket, nb = (uint32_t)it.nbuckets;

    // ---- phase 0: stage the item's halo table in LDS -------------------------
    const int nh = it.h1 - it.h0;
    if (tid < nh) {
        const oa_halo &h = a.halos[it.h0 + tid];
        const oa_halo &h0 = a.halos[it.h0];
        H.lstart[tid] = (uint32_t)(h.cur_off - h0.cur_off);
        H.has_prev[tid] = compare && h.prev_cnt >= 0;
        H.halo_cnt[tid] = 0;
        for (int d = 0; d < 3; ++d) { H.cb[tid][d] = h.centre[d]; H.cb[tid][3 + d] = h.bulk[d]; }
        if (tid == nh - 1) {
            H.lstart[nh] = (uint32_t)(h.cur_off + h.cur_cnt - h0.cur_off);
            H.n_span = H.lstart[nh];
            H.cur_base = h0.cur_off;
        }
    }
    if (tid == 0) {
        H.nonuniform = 0; H.nent = 0; H.overflow = 0; H.nh = nh;
        // progenitor segments in halo order (serial: nh <= HMAX)
        uint32_t ns = 0, vp = 0;
        for (int k = 0; k < nh; ++k) {
            const oa_halo &h = a.halos[it.h0 + k];
            if (compare && h.prev_cnt > 0) {
                H.seg_halo[ns] = k; H.seg_prev_off[ns] = h.prev_off; H.vstart[ns] = vp;
                vp += (uint32_t)h.prev_cnt; ++ns;
            }
        }
        H.vstart[ns] = vp; H.nseg = ns; H.n_pv = vp;
        // reference high word for the 32-bit LDS keys: the item's first particle
        const oa_halo &h0 = a.halos[it.h0], &hl1 = a.halos[it.h1 - 1];
        H.hi0 = 0;
        if (IDB == 8 && hl1.cur_off + hl1.cur_cnt > h0.cur_off)
            H.hi0 = (uint32_t)((uint64_t)ids[h0.cur_off] >> 32);
    }
    if (compare) {
        for (uint32_t w = tid; w < (nslots + 1) / 2; w += WG) slotw[w] = 0u;
    }
    __syncthreads();

    const int64_t base = H.cur_base;
    const uint32_t n_span = H.n_span;
    const uint32_t hi0 = H.hi0;

    // ---- phase 1: frame of every current particle, LDS insert ---------------
    for (uint32_t l0 = 0; l0 < n_span; l0 += WG * UNR) {
        ID idv[UNR];
        V3<TX> xv[UNR];
        V3<TV> vv[UNR];
        bool ok[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            uint32_t li = l0 + u * WG + tid;
            ok[u] = li < n_span;
            if (ok[u]) {
                int64_t i = base + li;
                idv[u] = ids[i];
                xv[u] = ld3(coords, i);
                vv[u] = ld3(vels, i);
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (!ok[u]) continue;
            uint32_t li = l0 + u * WG + tid;
            uint32_t lo, hi;
            id_split<IDB>(idv[u], lo, hi);
            if (BUCKETED && bucket_of(lo, hi, nb) != q) continue;
            uint32_t hl = (BUCKETED || H.nh == 1) ? 0u : upper_find(H.lstart, H.nh, li);
            TD r[3];
            uint32_t sgn = frame<TX, TV, TD>(xv[u], vv[u], H.cb[hl], a, r);
            uint32_t ang = 0;
            if (!compare && a.angles_in) ang = a.angles_in[base + li];
            R rec;
            rec.r[0] = r[0]; rec.r[1] = r[1]; rec.r[2] = r[2];
            rec.meta = ang | (sgn << 16);
            if constexpr (sizeof(R) == 32) rec.pad = 0;
            rec_out[base + li] = rec;
            if (H.has_prev[hl]) {
                if (IDB == 8 && hi != hi0) H.nonuniform = 1u;     // benign race: all write 1
                uint32_t e = li;
                if (BUCKETED) {
                    e = atomicAdd(&H.nent, 1u);
                    if (e >= (uint32_t)nent_max) { H.overflow = 1u; continue; }
                    lidx[e] = li;
                }
                ids_lo[e] = lo;
                lds_insert(slotw, nslots, slot_of(lo, hl, nslots), e + 1);
            }
        }
    }
    if (!compare) return;
    __syncthreads();
    if (H.overflow) {
        if (tid == 0) atomicOr(a.status, OA_STATUS_BUCKET_OVERFLOW);
        return;
    }

    // ---- phase 2: stream progenitor blocks, join, flag, angle, emit ---------
    const uint32_t n_pv = H.n_pv, nseg = H.nseg;
    const bool nonuniform = IDB == 8 && H.nonuniform != 0;
    const uint64_t lanemask_lt = (1ull << lane) - 1ull;
    uint32_t running = 0;
    ID *scr_ids = reinterpret_cast<ID *>(a.scratch_ids);

    for (uint32_t v0 = 0; v0 < n_pv; v0 += WG * UNR) {
        ID pid[UNR];
        R prec[UNR];
        int64_t kpos[UNR];
        uint32_t hlv[UNR];
        bool ok[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            uint32_t vp = v0 + u * WG + tid;
            ok[u] = vp < n_pv;
            if (ok[u]) {
                uint32_t sg = nseg == 1 ? 0u : upper_find(H.vstart, nseg, vp);
                hlv[u] = (uint32_t)H.seg_halo[sg];
                kpos[u] = H.seg_prev_off[sg] + (vp - H.vstart[sg]);
                pid[u] = ids_prev[kpos[u]];
                prec[u] = rec_prev[kpos[u]];
            }
        }
        bool flag[UNR];
        uint16_t a16[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            flag[u] = false;
            a16[u] = 0;
            if (!ok[u]) continue;
            uint32_t lo, hi;
            id_split<IDB>(pid[u], lo, hi);
            if (BUCKETED && bucket_of(lo, hi, nb) != q) { ok[u] = false; continue; }
            const uint32_t hl = hlv[u];
            // probe (hl, id): departed particles miss (setdiff1d/in1d, :300-304)
            int32_t e = -1;
            if (!(IDB == 8 && !nonuniform && hi != hi0)) {
                const uint32_t lmin = BUCKETED ? 0u : H.lstart[hl];
                const uint32_t lmax = BUCKETED ? 0xFFFFFFFFu : H.lstart[hl + 1];
                uint32_t s = slot_of(lo, hl, nslots);
                for (;;) {
                    uint32_t f = (slotw[s >> 1] >> ((s & 1u) << 4)) & 0xFFFFu;
                    if (!f) break;
                    uint32_t c = f - 1;
                    if (ids_lo[c] == lo && c >= lmin && c < lmax) {
                        if (!nonuniform) { e = (int32_t)c; break; }
                        uint32_t lc = BUCKETED ? lidx[c] : c;
                        if (ids[base + lc] == pid[u]) { e = (int32_t)c; break; }
                    }
                    s = (s + 1 == nslots) ? 0u : s + 1;
                }
            }
            if (e < 0) { a16[u] = 0xFFFFu; continue; }
            const uint32_t li = BUCKETED ? lidx[e] : (uint32_t)e;
            const R cur = rec_out[base + li];
            const uint32_t sc = cur.meta >> 16, sp = prec[u].meta >> 16;
            // strict sign test (:311-314): zeros and NaNs never flag
            const bool cond = a.mode == OA_MODE_PERICENTRIC ? (sp == 2u && sc == 1u)
                                                            : (sp == 1u && sc == 2u);
            // angle change = arccos(dot(r̂_prev, r̂_match)), no clamp (:324-325)
            TD dt = dot3(prec[u].r[0], prec[u].r[1], prec[u].r[2], cur.r[0], cur.r[1], cur.r[2]);
            uint16_t acc = angle_add((uint16_t)(prec[u].meta & 0xFFFFu), acos_td(dt));
            // calc_angles (:342-349): apsis angle emitted, then reset to 0
            *reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(&rec_out[base + li]) +
                                          offsetof(R, meta)) = cond ? (uint16_t)0 : acc;
            flag[u] = cond;
            a16[u] = acc;
        }
        if (BUCKETED) {
            // dense per-previous-position code; order restored by k_gather_dense
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                if (ok[u]) {
                    uint16_t code = flag[u] ? a16[u] : (uint16_t)0xFFFFu;
                    if (flag[u] && code == 0xFFFFu) code = 0x7E00u;   // keep the sentinel free
                    a.dense_code[kpos[u]] = code;
                }
                uint64_t m = __ballot(flag[u]);
                if (lane == 0 && m) {
                    const oa_halo &h = a.halos[it.h0];
                    atomicAdd(&a.halo_count[h.out_slot], (int32_t)__popcll(m));
                }
            }
            continue;
        }
        // ordered stream compaction (previous-block order, :315-316) via wave ballots
        uint64_t masks[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            masks[u] = __ballot(flag[u]);
            if (lane == 0) H.wave_cnt[u * NWAVE + wave] = (uint32_t)__popcll(masks[u]);
        }
        __syncthreads();
        if (wave == 0) {
            uint32_t x = lane < UNR * NWAVE ? H.wave_cnt[lane] : 0u, incl = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (lane < UNR * NWAVE) H.wave_pre[lane] = incl - x;
            if (lane == 63) H.chunk_total = incl;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (flag[u]) {
                uint32_t pos = running + H.wave_pre[u * NWAVE + wave] +
                               (uint32_t)__popcll(masks[u] & lanemask_lt);
                scr_ids[it.scratch_off + pos] = pid[u];
                a.scratch_ang[it.scratch_off + pos] = a16[u];
                atomicAdd(&H.halo_cnt[hlv[u]], 1);
            }
        }
        running += H.chunk_total;
        __syncthreads();
    }
    if (BUCKETED) return;
    __syncthreads();
    if (tid < nh) {
        const oa_halo &h = a.halos[it.h0 + tid];
        if (h.out_slot >= 0) a.halo_count[h.out_slot] = H.halo_cnt[tid];
    }
    if (tid == 0) a.item_count[blockIdx.x] = (int32_t)running;
}

// ------------------------------------------------------------------ compaction
__global__ __launch_bounds__(1024) void k_scan_slots(const int32_t *cnt, int32_t n,
                                                     int64_t *off, int64_t *total) {
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int b = 0; b < n; b += 1024) {
        int i = b + tid;
        int64_t x = i < n ? cnt[i] : 0, incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            int64_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        int64_t wpre = 0;
        for (int w = 0; w < wave; ++w) wpre += wsum[w];
        if (i < n) off[i] = carry + wpre + incl - x;
        __syncthreads();
        if (tid == 0) { int64_t s = 0; for (int w = 0; w < 16; ++w) s += wsum[w]; carry += s; }
        __syncthreads();
    }
    if (tid == 0) { off[n] = carry; *total = carry; }
}

template <int IDB>
__global__ __launch_bounds__(256) void k_gather_items(const oa_compact_args a) {
    typedef typename IdT<IDB>::T ID;
    const oa_item it = a.items[blockIdx.x];
    const int32_t n = a.item_count[blockIdx.x];
    if (n <= 0) return;
    int64_t slot = -1;
    for (int h = it.h0; h < it.h1 && slot < 0; ++h) slot = a.halos[h].out_slot;
    if (slot < 0) return;
    const int64_t dst = a.offsets_out[slot];
    const ID *src = reinterpret_cast<const ID *>(a.scratch_ids) + it.scratch_off;
    ID *out = reinterpret_cast<ID *>(a.out_ids) + dst;
    const uint16_t *sa = a.scratch_ang + it.scratch_off;
    uint16_t *oa = a.out_ang + dst;
    for (int i = threadIdx.x; i < n; i += 256) { out[i] = src[i]; oa[i] = sa[i]; }
}

template <int IDB>
__global__ __launch_bounds__(1024) void k_gather_dense(const oa_compact_args a) {
    typedef typename IdT<IDB>::T ID;
    __shared__ uint32_t wcnt[16];
    const oa_item it = a.big_items[blockIdx.x];
    if (it.bucket != 0) return;
    const oa_halo h = a.halos[it.h0];
    if (h.out_slot < 0 || h.prev_cnt <= 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lanemask_lt = (1ull << lane) - 1ull;
    const ID *ids_prev = reinterpret_cast<const ID *>(a.ids_prev);
    ID *out = reinterpret_cast<ID *>(a.out_ids) + a.offsets_out[h.out_slot];
    uint16_t *oa = a.out_ang + a.offsets_out[h.out_slot];
    int64_t running = 0;
    for (int64_t b = 0; b < h.prev_cnt; b += 1024) {
        int64_t k = b + tid;
        uint16_t code = k < h.prev_cnt ? a.dense_code[h.prev_off + k] : (uint16_t)0xFFFFu;
        bool f = code != 0xFFFFu;
        uint64_t m = __ballot(f);
        if (lane == 0) wcnt[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < 16; ++w) { uint32_t c = wcnt[w]; if (w < wave) pre += c; tot += c; }
        if (f) {
            int64_t pos = running + pre + __popcll(m & lanemask_lt);
            out[pos] = ids_prev[h.prev_off + k];
            oa[pos] = code;
        }
        running += tot;
        __syncthreads();
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

template <typename K>
int set_lds(K kernel, int64_t bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return fail(OA_E_LAUNCH, "hipFuncSetAttribute: %s", hipGetErrorString(e));
    return OA_OK;
}

template <typename TX, typename TV, typename TD, int IDB>
int launch_step(const oa_step_args &a, hipStream_t st) {
    if (a.n_items > 0) {
        int64_t lds = HDR_BYTES + table_bytes(a.lds_entries, a.lds_slots, false);
        auto k = k_step<TX, TV, TD, IDB, false>;
        if (int rc = set_lds(k, lds)) return rc;
        hipLaunchKernelGGL(k, dim3(a.n_items), dim3(WG), (size_t)lds, st, a);
        if (int rc = check_launch("k_step")) return rc;
    }
    if (a.n_big_items > 0) {
        int64_t lds = HDR_BYTES + table_bytes(a.big_entries, a.big_slots, true);
        auto k = k_step<TX, TV, TD, IDB, true>;
        if (int rc = set_lds(k, lds)) return rc;
        hipLaunchKernelGGL(k, dim3(a.n_big_items), dim3(WG), (size_t)lds, st, a);
        if (int rc = check_launch("k_step(bucketed)")) return rc;
    }
    return OA_OK;
}

template <typename TX, typename TV, typename TD>
int launch_step_id(const oa_step_args &a, hipStream_t st) {
    return a.id_bytes == 8 ? launch_step<TX, TV, TD, 8>(a, st) : launch_step<TX, TV, TD, 4>(a, st);
}

template <typename TX, typename TD>
int launch_step_v(const oa_step_args &a, hipStream_t st) {
    return a.vel_f64 ? launch_step_id<TX, double, TD>(a, st) : launch_step_id<TX, float, TD>(a, st);
}

}  // namespace

extern "C" {

int oa_abi_version(void) { return OA_ABI_VERSION; }

int64_t oa_struct_size(int32_t which) {
    switch (which) {
        case 0: return sizeof(oa_halo);
        case 1: return sizeof(oa_item);
        case 2: return sizeof(oa_step_args);
        case 3: return sizeof(oa_compact_args);
        default: return -1;
    }
}

const char *oa_last_error(void) { return g_err; }

int64_t oa_step_lds_bytes(int32_t entries, int32_t slots, int32_t bucketed) {
    return HDR_BYTES + table_bytes(entries, slots, bucketed != 0);
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
    if (a.n_items > 0 && (a.lds_entries <= 0 || a.lds_entries > 65534 ||
                          a.lds_slots <= a.lds_entries))
        return fail(OA_E_ARG, "bad lds_entries/lds_slots");
    if (a.n_big_items > 0 && (a.big_entries <= 0 || a.big_entries > 65534 ||
                              a.big_slots <= a.big_entries))
        return fail(OA_E_ARG, "bad big_entries/big_slots");
    if (a.n_items + a.n_big_items > 0 && (!a.halos || !a.ids || !a.coords || !a.vels || !a.rec_out))
        return fail(OA_E_ARG, "null input/output pointer");
    if (a.compare && (!a.ids_prev || !a.rec_prev || !a.halo_count || !a.status ||
                      (a.n_items > 0 && (!a.scratch_ids || !a.scratch_ang || !a.item_count)) ||
                      (a.n_big_items > 0 && !a.dense_code)))
        return fail(OA_E_ARG, "null previous-state / scratch pointer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (a.dx_f64) {
        return a.coord_f64 ? launch_step_v<double, double>(a, st)
                           : launch_step_v<float, double>(a, st);
    }
    return launch_step_v<float, float>(a, st);
}

int oa_compact(const oa_compact_args *args, void *stream) {
    g_err[0] = 0;
    if (!args) return fail(OA_E_ARG, "oa_compact: null args");
    const oa_compact_args &a = *args;
    if (a.id_bytes != 4 && a.id_bytes != 8) return fail(OA_E_ARG, "id_bytes must be 4 or 8");
    if (!a.offsets_out || !a.total_out || (a.n_slots > 0 && !a.halo_count))
        return fail(OA_E_ARG, "null output pointer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_scan_slots, dim3(1), dim3(1024), 0, st, a.halo_count, a.n_slots,
                       a.offsets_out, a.total_out);
    if (int rc = check_launch("k_scan_slots")) return rc;
    if (a.n_items > 0) {
        if (a.id_bytes == 8) hipLaunchKernelGGL(k_gather_items<8>, dim3(a.n_items), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_gather_items<4>, dim3(a.n_items), dim3(256), 0, st, a);
        if (int rc = check_launch("k_gather_items")) return rc;
    }
    if (a.n_big_items > 0) {
        if (a.id_bytes == 8) hipLaunchKernelGGL(k_gather_dense<8>, dim3(a.n_big_items), dim3(1024), 0, st, a);
        else hipLaunchKernelGGL(k_gather_dense<4>, dim3(a.n_big_items), dim3(1024), 0, st, a);
        if (int rc = check_launch("k_gather_dense")) return rc;
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

}  // extern "C"
