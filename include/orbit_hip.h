/*
 * orbit_hip.h — C ABI of liborbit_hip.so, the MI355X (gfx950) implementation of the
 * per-snapshot orbit-tagging hot path of s-balu/nbody-orbit-analysis.
 *
 * The reference is pure Python/NumPy and has no FFI; every entry point below
 * replaces a NumPy code path of the reference, cited per function
 * (paths relative to /root/reference/orbitanalysis/).  Bindings: INTEGRATION.md.
 *
 * Conventions
 *   - all array arguments are DEVICE pointers (HIP global memory) unless noted;
 *   - sizes are element counts; `stream` is a hipStream_t (NULL = default stream);
 *   - functions enqueue work on `stream` and return immediately; they never
 *     allocate, free or synchronise, so they are graph-capturable;
 *   - return 0 on success, a negative OA_E* code on bad arguments or a launch
 *     error; oa_last_error() returns the message of the last failure (thread-local);
 *   - no exception ever crosses the ABI.
 *
 * Numerics contract: the frame follows the reference's
 * NumPy expression tree and dtype promotion, with the reference host's einsum
 * summation order (f64 (p0+p2)+p1, f32 (p0+p1)+p2), no FMA contraction,
 * correctly rounded sqrt/div, float16 rounded directly from float64.
 */
#ifndef ORBIT_HIP_H
#define ORBIT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OA_ABI_VERSION 19

#define OA_OK 0
#define OA_E_ARG (-1)       /* invalid argument / unsupported dtype plan */
#define OA_E_LAUNCH (-2)    /* HIP launch error */
#define OA_E_DEVICE (-3)    /* no HIP device */

/* Run-time flags reported by the step kernel in `status` (bit mask). */
#define OA_STATUS_TABLE_OVERFLOW 2u   /* the LDS cuckoo table could not place every
                                         entry (stash full): re-plan smaller items */
#define OA_STATUS_PLAN 4u             /* an item exceeds the kernel's limits (more than
                                         oa_build_info(3) * work-group progenitor
                                         positions): the plan did not come from
                                         oa_plan_items                               */
#define OA_STATUS_PART_OVERFLOW 8u    /* a large-halo hash partition outgrew its bucket
                                         or LDS table: re-run the snapshot on the
                                         global-table path (n_parts = 0)             */
#define OA_STATUS_PART_KEYS 32u       /* part_key4: a large-halo ID's high word differs
                                         from part_hi: re-run on the global-table path
                                         and keep 8-byte bucket keys                 */
#define OA_STATUS_LOOKBACK 16u        /* direct records: an item's look-back found no
                                         predecessor prefix within its spin budget
                                         (records invalid): re-run with direct = 0   */

#define OA_MODE_PERICENTRIC 0
#define OA_MODE_APOCENTRIC 1

/* One current-snapshot halo (region block).  96 bytes, device array. */
typedef struct oa_halo {
    int64_t cur_off, cur_cnt;   /* block [cur_off, cur_off+cur_cnt) of the current arrays
                                   (region_offsets, track_orbits.py:129-132)            */
    int64_t prev_off, prev_cnt; /* progenitor block in the previous snapshot's arrays;
                                   prev_cnt < 0: the halo has no progenitor
                                   (track_orbits.py:162-165)                             */
    double centre[3];           /* region_positions[j], exact value of its dtype         */
    double bulk[3];             /* bulk velocity: catalogue value or oa_bulk_velocity()  */
    int64_t out_slot;           /* index among halos with a progenitor (apsis offsets),
                                   -1 if none                                            */
    int64_t reserved;
} oa_halo;

/* One work-group's share of a snapshot.  48 bytes, device array, built on the host by
 * oa_plan_items.
 * Packed items (k_step): halos [h0,h1) whose current blocks total <= lds_entries.
 * Global items (large halos, items[n_items ..]): the single halo h0 = h1 - 1.   */
typedef struct oa_item {
    int32_t h0, h1;
    int32_t slot0;              /* first output slot (oa_halo.out_slot) among [h0,h1),
                                   or -1                                               */
    int32_t n_span;             /* current particles of halos [h0,h1)                  */
    int64_t scratch_off;        /* first apsis-scratch slot of this item (a multiple
                                   of 64; one slot per padded progenitor position)    */
    int64_t n_pv;               /* padded progenitor positions of the item (each block
                                   with prev_cnt > 0 rounded up to 64)                */
    int64_t cur_off;            /* halos[h0].cur_off: the item's first current row     */
    int32_t n_slots;            /* LDS cuckoo slots of a packed item's table:
                                   min(2 * (current particles with a progenitor) + 64,
                                   the slots budget); 0 for global items             */
    int32_t reserved;
} oa_item;

/* Arguments of oa_step (one snapshot of the batch driver's inner loop). */
typedef struct oa_step_args {
    /* current snapshot, as returned by load_snapshot_data (track_orbits.py:121) */
    const void *ids;            /* (n_cur,) int32/int64 (id_bytes)                 */
    const void *coords;         /* (n_cur,3) row-major, f32 or f64 (coord_f64)     */
    const void *vels;           /* (n_cur,3) row-major, f32 or f64 (vel_f64)       */
    int64_t n_cur;
    /* previous snapshot state (outputs of the previous oa_step) */
    const void *ids_prev;       /* (n_prev,) same dtype as ids                     */
    const void *rhat_prev;      /* (n_prev,3) r̂ of the previous snapshot (dx dtype)  */
    const uint32_t *meta_prev;  /* (n_prev,) meta words, see meta_out                */
    int64_t n_prev;
    /* outputs: the particle state the next snapshot reads */
    void *rhat_out;             /* (n_cur,3) unit radial vectors, dx dtype           */
    uint32_t *meta_out;         /* (n_cur,) f16 angle bits | sign(v_r) << 16
                                   (sign: 1 = v_r > 0, 2 = v_r < 0, 0 = neither)    */
    const uint16_t *angles_in;  /* optional (n_cur,) f16 bits used as angles when
                                   compare == 0 (checkpoint resume), NULL -> 0     */
    /* tables: packed items [0, n_items), then n_global_items global items */
    const oa_halo *halos;
    int32_t n_halos;
    const oa_item *items;
    int32_t n_items;
    /* per-snapshot scalars (hubble_parameter, utils.py:36-39) */
    double H, one_plus_z;
    double box[3];
    int32_t n_box_dims;         /* 0: no periodic wrap */
    /* dtype plan: 1 = float64, 0 = float32 */
    int32_t coord_f64, vel_f64, dx_f64, vb_f64, wrap_f64;
    int32_t id_bytes;           /* 4 or 8 */
    int32_t mode;               /* OA_MODE_* */
    int32_t compare;            /* 0: frame only (first processed snapshot)       */
    int32_t lds_entries;        /* hash-table entries per work-group (items)      */
    int32_t lds_slots;          /* open-addressing slots per work-group (> entries) */
    /* apsis scratch */
    void *scratch_ids;          /* apsis records, one 64-slot segment per 64
                                   progenitor positions, packed per segment          */
    uint16_t *scratch_ang;
    uint8_t *seg_count;         /* records per segment ([scratch slots / 64])        */
    int32_t *halo_count;        /* [n_slots] apsis count per halo with a progenitor;
                                   must be zero on entry                             */
    int32_t *item_count;        /* [n_items + n_global_items] */
    uint32_t *status;           /* device word, OA_STATUS_* bits; zero on entry       */
    /* on-the-fly driver (track_orbits_onthefly.py:71-205); onthefly = 0: unused.
     * Frame semantics of that driver: dx stored in the coordinate dtype (r̂ too),
     * w = v - bulk stored in the velocity dtype, no Hubble term, v_r in
     * promote(velocity, coordinate) dtype (vr_f64). */
    int32_t onthefly;
    int32_t vr_f64;
    void *angle_out;            /* (n_prev,) coordinate dtype: arccos(r̂_prev . r̂_match)
                                   of every matched previous particle (:173-174)      */
    uint8_t *matched_prev;      /* (n_prev,) 1 = matched, 0 = departed (:145-148)     */
    uint8_t *matched_cur;       /* (n_cur,) set to 1 when matched; zero on entry
                                   (0 = entered, :168)                                */
    double *vr_out;             /* optional (n_cur,) float64 radial velocities of a
                                   frame-only batch launch (the module-level
                                   region_frame, track_orbits.py:247-290); NULL = off */
    /* large halos (blocks beyond one work-group's LDS table): items[n_items ..
     * n_items + n_global_items) are single-halo items joined through per-halo
     * open-addressing tables in global memory (any number of work-groups per halo) */
    int32_t n_global_items;
    int32_t n_gchunk1, n_gchunk2;
    const int64_t *gchunk1;     /* (item, start, count) chunks of current blocks      */
    const int64_t *gchunk2;     /* (item, start, count) chunks of previous blocks,
                                   start a multiple of 64                             */
    const int64_t *gtab;        /* per global item: (slot offset, capacity = 2^k)     */
    uint64_t *gkeys;            /* table entries, 16 B each: {u64 id, u32 position + 1
                                   (0 = empty), u32 pad}; zeroed by oa_step          */
    uint32_t *gvals;            /* unused (NULL)                                      */
    int64_t gtab_total;         /* slots over all global items                        */
    /* optional (NULL = off): per apsis record, the index of its particle in the
     * previous-state arrays (ids_prev / rhat_prev rows, < 2^31), stored beside
     * scratch_ids; the sharded driver maps it to the particle's position in the global
     * previous block, which orders the merged records (sharding.py) */
    int32_t *scratch_pos;
    /* Partitioned large halos (compare steps, not on-the-fly; n_parts = 0: the
     * global-table path above).  Each global item's IDs are cut into K hash partitions
     * (K a power of two, partition = mulhi64(mix64(ID), K)) so one partition's current
     * particles fit an LDS table of oa_build_info(4) entries.  A *bucket set* holds one
     * snapshot's state of those halos by partition: per entry the ID (its low word
     * only with part_key4), the position in the halo's block (| sign(v_r) << 30 in a
     * current set), the state word and r̂.  The current set of one step is the previous
     * set of the next (inherited), so the previous state is streamed from its buckets,
     * never scattered again:
     *   k_part_scatter  frame of the current chunks (gchunk1) into the current set
     *                   (LDS-staged: each partition's entries leave as one run); the
     *                   previous chunks (gchunk2) of halos without an inherited set
     *                   into a fresh previous set, from the position-order state
     *   k_part_join     one work-group per prow row (LDS: oa_part_lds_bytes): LDS table
     *                   of a current bucket, lookups of the previous bucket(s) holding
     *                   its IDs, the state word of every matched current entry; each
     *                   apsis record is appended to its previous-block chunk (gchunk2
     *                   row: 4096 positions, oa_build_info(7)) in the item's scratch
     *                   range with its position in the chunk (scratch_rk)
     *   oa_compact      ranks each chunk's records by position (k_gather_recs)
     * The position-order rhat_out / meta_out of these halos are NOT written
     * (oa_part_unbucket restores them from the set when a caller needs them).      */
    int32_t n_parts;            /* rows of prow (padding rows included)               */
    int32_t part_kmax;          /* largest K of any global item                       */
    int32_t part_e;             /* current bucket capacity = LDS table entries of one
                                   partition (multiple of 64, <= oa_build_info(4))    */
    int32_t part_slots;         /* its cuckoo slots (part_e < slots <= 1.5 build max) */
    const int64_t *prow;        /* [n_parts] join work-group descriptors, 16 int64:
                                   [0..8] the gpart row of its global item g, [9] the
                                   partition, [10] g (-1: an idle padding row), [11]
                                   the item's scratch_off, [12] its record chunks
                                   (ceil(previous block / oa_build_info(7))), [13] the
                                   halo's out_slot (one row: a work-group's first
                                   loads need no second, dependent one)              */
    const int64_t *gpart;       /* per global item, oa_build_info(6) = 16 int64:
                                   [0] current set base (entries; partition p at
                                   base + p * part_e), [1] K, [2] index of its first
                                   counter in pcnt, [3] previous set: 0 fresh (the
                                   *_prev arrays, counters in pcnt), 1 inherited (the
                                   i* arrays, counters in icnt), [4] previous set base,
                                   [5] its K (a power of two), [6] its entries per
                                   partition, [7] index of its first counter,
                                   [8] index in pcnt of the record counter of its
                                   first previous-block chunk (one per gchunk2 row of
                                   the item, in order), [9..15] 0                     */
    void *pkey_cur;             /* current set: IDs (uint64; uint32 low words with
                                   part_key4)                                         */
    uint32_t *ppos_cur;         /*   position in the halo's block | sign(v_r) << 30   */
    uint32_t *pmeta_cur;        /*   state word (f16 angle | sign << 16)              */
    void *prh_cur;              /*   r̂ (3 values of the r̂ dtype)                      */
    void *pkey_prev;            /* fresh previous set: IDs (as pkey_cur)              */
    uint32_t *ppos_prev;        /*   position in the halo's previous block            */
    uint32_t *pmeta_prev;       /*   its previous state word                          */
    void *prh_prev;             /*   its previous r̂ (3 values of the r̂ dtype)         */
    const void *ikey;           /* inherited previous set (the previous step's current
                                   set, keys of the same width; any of these may be
                                   NULL when none is used)                            */
    const uint32_t *ipos;
    const uint32_t *imeta;
    const void *irh;
    const uint32_t *icnt;       /*   its fill counters                                */
    uint32_t *pcnt;             /* [n_pcnt] fill counters of the current set and of the
                                   fresh previous set, then the record counters of the
                                   previous-block chunks; zeroed by oa_step           */
    int64_t n_pcnt;
    uint16_t *scratch_rk;       /* per apsis record of a partitioned halo: its position
                                   in its 4096-position chunk (beside scratch_ids)    */
    int32_t part_key4;          /* 1: bucket keys are the IDs' low words; every
                                   large-halo ID's high word must equal part_hi, else
                                   OA_STATUS_PART_KEYS (4-byte IDs: always 1)         */
    uint32_t part_hi;
    const int64_t *gchunk3;     /* the previous chunks k_part_scatter reads: those of
                                   halos with a fresh previous set (NULL: gchunk2)    */
    int32_t n_gchunk3;
    int32_t items_single;       /* 1: every packed item holds one halo (the launch takes
                                   k_step's one-halo specialisation); 0: any item plan */
    /* Direct records (replaces oa_compact for a compare step with packed items only,
     * not on-the-fly): k_step writes every apsis record at its final output offset
     * and the per-halo offsets (track_orbits.py:199-227), each item finding its
     * record prefix by a decoupled look-back over the items before it.            */
    int32_t direct;             /* 1: on (n_global_items must be 0); 0: scratch +
                                   oa_compact                                        */
    uint64_t *lookback;         /* [n_items] item prefix words: lb_epoch << 48 | state
                                   << 46 | records (state 1: the item's own count,
                                   2: inclusive prefix); words of other epochs read as
                                   unpublished, so the buffer is zeroed only once and
                                   again before an epoch repeats                      */
    int32_t lb_epoch;           /* 1..65535 */
    int32_t n_slots;            /* halos with a progenitor (out_slot range)           */
    int64_t *offsets_out;       /* [n_slots + 1] apsis region offsets                 */
    void *out_ids;              /* capacity >= records (<= n_prev), ID dtype           */
    uint16_t *out_ang;          /* float16 bits                                        */
    int32_t *out_pos;           /* optional: each record's previous-state row (the
                                   oa_compact_args.out_pos of a scratch_pos step)     */
    int64_t *total_out;         /* device scalar: number of records                    */
    uint32_t lb_spin_max;       /* direct records: polls of an unpublished look-back word
                                   before OA_STATUS_LOOKBACK (0: the default, 2^14; a
                                   test sets 1 to exercise the re-run without direct)  */
    int32_t reserved_abi16;
} oa_step_args;

/* Arguments of oa_part_unbucket: a bucket set's entries back to position order. */
typedef struct oa_unbucket_args {
    const uint32_t *bpos;       /* the set's position words (position | sign << 30)   */
    const uint32_t *bmeta;      /* its state words                                    */
    const void *brh;            /* its r̂ (3 values of the r̂ dtype per entry)          */
    const uint32_t *bcnt;       /* its fill counters                                  */
    const int64_t *rows;        /* per listed halo, 4 int64: set base, K, first counter
                                   index, block offset of the halo in the state arrays */
    const int32_t *plist;       /* [n_parts] (row, partition) pairs; row -1: padding   */
    int32_t n_parts;
    int32_t cap;                /* entries per partition of the set (part_e)          */
    void *rhat_out;             /* the snapshot's position-order state arrays        */
    uint32_t *meta_out;
    int32_t td_f64;             /* r̂ dtype: 1 float64, 0 float32                      */
    int32_t reserved;
} oa_unbucket_args;

/* Arguments of oa_compact: gather the per-item apsis records into the reference's
 * output layout (track_orbits.py:212-227 -> save_to_file :379-381). */
typedef struct oa_compact_args {
    const oa_halo *halos;
    int32_t n_halos;
    const oa_item *items;
    int32_t n_items;
    const void *ids_prev;
    int32_t id_bytes;
    const void *scratch_ids;
    const uint16_t *scratch_ang;
    const uint8_t *seg_count;
    const int32_t *halo_count;
    const int32_t *item_count;
    int32_t n_slots;
    int64_t *offsets_out;       /* [n_slots+1] apsis region offsets (cumsum([0]+lens)) */
    void *out_ids;              /* capacity >= total (<= n_prev) */
    uint16_t *out_ang;
    int64_t *total_out;         /* device scalar: number of apsis records */
    const int32_t *scratch_pos; /* optional: oa_step_args.scratch_pos of the step        */
    int32_t *out_pos;           /* optional: the records' previous-state indices, in
                                   output order (with scratch_pos)                     */
    int32_t n_packed;           /* items[0, n_packed) are k_step items (records
                                   contiguous from scratch_off), the rest global items
                                   (records in 64-position segments)                  */
    int32_t n_gchunks;
    const int64_t *gchunks;     /* optional: oa_step_args.gchunk2 of the step (the global
                                   items' previous-block chunks); their records are then
                                   gathered one work-group per chunk instead of one per
                                   item (NULL: per item)                                */
    const uint32_t *chunk_count;/* partitioned steps (with gchunks): the record count of
                                   each gchunk2 row (oa_step_args.pcnt + gpart[8] of its
                                   item's first row ...); the records of a chunk sit
                                   unordered at its scratch base and are ranked by
                                   scratch_rk.  NULL: 64-position segments (seg_count) */
    const uint16_t *scratch_rk;
} oa_compact_args;

/* ABI version (OA_ABI_VERSION) — lets the host reject a stale library. */
int oa_abi_version(void);

/* sizeof() of the ABI structs (0 oa_halo, 1 oa_item, 2 oa_step_args,
 * 3 oa_compact_args, 4 oa_unbucket_args) so a binding can verify its layout; -1
 * otherwise. */
int64_t oa_struct_size(int32_t which);

/* Compile-time configuration: 0 work-group size, 1 max halos per item,
 * 2 phase-1 unroll, 3 progenitor rows (64 positions) per wave of an item, 4 current
 * entries per large-halo partition (k_part_join's LDS table), 5 largest K per halo
 * (k_part_scatter's LDS counters), 6 int64 per gpart row, 7 previous-block positions
 * per large-halo chunk (gchunk2 rows; the record chunks of k_part_join); -1 otherwise. */
int32_t oa_build_info(int32_t which);

/* LDS bytes of one k_part_join work-group for a partition of `entries` current
 * entries in a table of `slots` slots (oa_step_args.part_e / part_slots). */
int64_t oa_part_lds_bytes(int32_t entries, int32_t slots);

/* Message of the last failing call on this thread ("" if none). */
const char *oa_last_error(void);

/* Bulk velocity of each listed halo block, with NumPy's reduction orders:
 *   masses == NULL : mean(v, axis=0)          (track_orbits.py:279-280)
 *   masses != NULL : sum(m[:,None]*v, axis=0) / sum(m)   (:269-272)
 * axis-0 sums are sequential; sum(m) is NumPy's pairwise sum over 8192-element
 * chunks.  Writes halos[list[k]].bulk (exact value of the result dtype). */
int oa_bulk_velocity(const void *vels, int32_t vel_f64, const void *masses, int32_t mass_f64,
                     oa_halo *halos, const int32_t *halo_list, int32_t n_list, void *stream);

/* Fused per-snapshot kernel: region_frame (track_orbits.py:247-290) for every
 * particle of every halo, then — when compare != 0 — the ID join against the
 * progenitor block, the strict sign-flip test, the arccos angle change and the
 * float16 angle bookkeeping of compare_radial_velocities + calc_angles
 * (:293-351), emitting apsis records in previous-block order. */
int oa_step(const oa_step_args *args, void *stream);

/* Dynamic LDS bytes a join work-group needs for the given table sizes and r̂ dtype
 * (dx_f64: 1 = float64): max(8 * slots + 2 * entries, 3 * entries * sizeof(r̂)) +
 * entries + the item header. */
int64_t oa_step_lds_bytes(int32_t entries, int32_t slots, int32_t dx_f64);

/* HOST function (no device needed): the work-group plan of one snapshot.
 * Replaces the per-halo dispatch of track_orbits.py:147-194 (the `track(j)` closure
 * mapped over halos): consecutive halos whose current blocks fit one LDS table
 * (<= entries particles, <= hmax halos, <= max_pv padded progenitor positions) are
 * packed greedily into items (k_step); a halo beyond any of those limits becomes a
 * single-halo global item (k_big_*), listed after every packed item.
 *   cur_off[n_halos], cur_cnt[n_halos] (the current blocks), prev_cnt[n_halos]
 *   (< 0: no progenitor), out_slot[n_halos] (-1: none) are host arrays; `slots` is
 *   the LDS table budget (oa_step_args.lds_slots); items[cap] receives the plan.
 * Returns the number of items written (packed + global), or a negative OA_E*;
 * *n_small = packed items, *scratch = apsis-scratch slots (one per padded
 * progenitor position). */
int64_t oa_plan_items(const int64_t *cur_off, const int64_t *cur_cnt, const int64_t *prev_cnt,
                      const int64_t *out_slot, int64_t n_halos, int64_t entries, int64_t slots,
                      int64_t hmax, int64_t max_pv, oa_item *items, int64_t cap,
                      int64_t *n_small, int64_t *scratch);

/* HOST function (no device needed): the halo table of one snapshot (oa_halo rows) from
 * its columns -- block starts and sizes (region_offsets, track_orbits.py:129-132), the
 * progenitor blocks (prev_off / prev_cnt, -1: none, :162-165), output slots, centres
 * (region_positions) and catalogue bulk velocities (NULL: zero, computed later by
 * oa_bulk_velocity).  All arrays are host arrays of n rows; centre / bulk are (n, 3)
 * float64.  Returns 0 or OA_E_ARG. */
int oa_build_halos(const int64_t *cur_off, const int64_t *cur_cnt, const int64_t *prev_off,
                   const int64_t *prev_cnt, const int64_t *out_slot, const double *centre,
                   const double *bulk, int64_t n, oa_halo *halos);

/* Diagnostic builds only (-DOA_STAMPS=1): copy the per-work-group phase timestamps
 * (s_memrealtime, 100 MHz; 6 per work-group) of the last oa_step to host memory.
 * Returns the number of values copied, -1 in normal builds. */
int64_t oa_debug_stamps(uint64_t *host, int64_t n);

/* Diagnostic builds only: stamps of the large-halo partition kernels of the last
 * oa_step (which = 0: k_part_join, 8 per work-group; 1: k_part_scatter, 2 per
 * work-group).  Returns the number of values copied, -1 in normal builds. */
int64_t oa_debug_part_stamps(int32_t which, uint64_t *host, int64_t n);

/* Largest dynamic LDS allocation a work-group may use on this device (bytes). */
int64_t oa_max_lds_bytes(void);

/* Restore the position-order state (r̂, state word) of the listed halos from a bucket
 * set (oa_step_args' partitioned large halos): for a checkpoint of the angles
 * (track_orbits.py:390-394) or a next step that reads those halos in position order. */
int oa_part_unbucket(const oa_unbucket_args *args, void *stream);

/* Scan the per-halo / per-item apsis counts and gather the records in output order. */
int oa_compact(const oa_compact_args *args, void *stream);

/* ---- multi-GPU output stage (sharding.ShardedEngine.fetch_async) ----------------
 * Replaces the single writer's gather of every per-halo result (track_orbits.py:199-227,
 * save_to_file :366-397): each rank stores its own apsis records at their final
 * positions in one page-locked host buffer that every rank maps, over its own PCIe
 * link, so rank 0 only waits and writes the file. */

/* Page-lock `bytes` of host memory at `host` (e.g. a shared-memory mapping) and return
 * the device-visible address of its first byte in *device_ptr. */
int oa_host_register(void *host, int64_t bytes, void **device_ptr);
int oa_host_unregister(void *host);

/* When the work queued on `stream` so far has completed, store `value` to the host
 * word `*host_addr` (a HIP host callback, release order): a rank tells the writing rank
 * that its records are in place without its host waiting for them. */
int oa_stream_set_flag(void *stream, int64_t *host_addr, int64_t value);

/* dst[0, bytes) = src[0, bytes) by a kernel on `stream`: src any device-accessible
 * address (a page-locked host block from oa_host_register), dst device memory, both
 * 16-byte aligned.  The engines' per-step host tables (halo table, item plan, partition
 * rows) go up this way, not by a copy-engine DMA queued behind an earlier step's
 * records D2H (track_orbits.py:189-227's pipelined form).  ABI 19. */
int oa_copy_bytes(const void *src, void *dst, int64_t bytes, void *stream);

/* *host_status = *status and *host_total = *total, stored by a kernel on `stream`
 * (host_* are device addresses of page-locked host words, oa_host_register): a step's
 * status word and record count reach the host behind the step's kernels without a copy
 * engine, which may still be moving an earlier step's records (track_orbits.py:189-227's
 * pipelined form, OrbitEngine.settle).  ABI 19. */
int oa_post_status(const int32_t *status, const int64_t *total, int32_t *host_status,
                   int64_t *host_total, void *stream);

/* out_ids[dst[i]] = ids[i] (id_bytes 4 or 8 each), out_ang[dst[i]] = ang[i] for
 * i < n; dst values must lie in [0, cap) (a record outside is dropped and counted in
 * *status).  The outputs may be host memory from oa_host_register (zero-copy stores).
 * ids and out_ids may both be NULL: the 16-bit values alone (checkpoint angles at their
 * global snapshot rows, track_orbits.py:390-394).  ang and out_ang may both be NULL: the
 * 4- or 8-byte values alone (the on-the-fly driver's IDs, or its angle changes in the
 * coordinate dtype, track_orbits_onthefly.py:154-174). */
int oa_place_records(const void *ids, const uint16_t *ang, const int64_t *dst, int64_t n,
                     int32_t id_bytes, void *out_ids, uint16_t *out_ang, int64_t cap,
                     int32_t *status, void *stream);

/* ---- block helpers: the module-level functions on arbitrary arrays ---------------- */

/* Device workspace bytes oa_match_ids needs for n_cur current IDs. */
int64_t oa_match_workspace_bytes(int64_t n_cur);

/* For every previous ID, the index of the equal current ID or -1: the in1d / myin1d /
 * setdiff1d join of compare_radial_velocities (track_orbits.py:300-306, utils.py:4-11).
 * Current IDs must be unique (myin1d's precondition).  Open addressing in `workspace`. */
int oa_match_ids(const void *ids_cur, int64_t n_cur, const void *ids_prev, int64_t n_prev,
                 int32_t id_bytes, void *workspace, int64_t *match_out, void *stream);

/* Per previous particle with match[i] >= 0: strict sign-flip flag (:311-314) and the
 * angle change arccos(dot(r̂_prev[i], r̂[match[i]])) in the r̂ dtype (:324-325).
 * vr / vr_prev are float64 (exact copies of the caller's values). */
int oa_compare_pairs(const int64_t *match, int64_t n_prev, const double *vr, const double *vr_prev,
                     const void *rhat, const void *rhat_prev, int32_t td_f64, int32_t mode,
                     uint8_t *flag_out, void *change_out, void *stream);

/* out[i] = float16(angles_prev[i] + change[i]) with NumPy's promotion (f16 + f32 in
 * float32, f16 + f64 in float64, rounded directly to f16): calc_angles :342-351. */
int oa_angle_add(const uint16_t *angles_prev, const void *change, int64_t n, int32_t td_f64,
                 uint16_t *out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* ORBIT_HIP_H */
