/*
 * orbit_post.h — C ABI of the SURVEY.md §8(f) rows f3 and f4 in liborbit_hip.so:
 * the consumer of the orbit path's output (collation of apsis IDs into per-halo
 * orbit counts) and its producer (main-progenitor finding from central particles).
 *
 * Reference interfaces replaced (paths relative to /root/reference/orbitanalysis/):
 *   oa_collate_step        postprocessing.py:118-142  Apsides.collate_apsides: per
 *                          snapshot, append the halo's apsis IDs with angle > cut and
 *                          np.unique(return_counts) the cumulative list per halo
 *   oa_retro_counts        postprocessing.py:215-236  Apsides.save_final_apsis_counts:
 *                          myin1d into the final snapshot's per-halo IDs + gather
 *   oa_central_ids         progenitors.py:38-56       get_central_particle_ids:
 *                          recentre, radius, argsort(...)[:n] per region block
 *   oa_main_progenitors    progenitors.py:82-117      find_main_progenitors: unique
 *                          tracked IDs, in1d/myin1d against halo members, per-block
 *                          plurality halo number
 *
 * Conventions as in orbit_hip.h: DEVICE pointers, element counts, a hipStream_t,
 * int status (0 ok, OA_E_* on bad arguments or launch errors, message from
 * oa_last_error()); no allocation, no synchronisation, no exception across the ABI.
 *
 * ID kinds (`*_kind`): 0 int64, 1 uint64, 2 int32, 3 uint32.  Sorted outputs are in
 * the numeric order of the output kind (np.unique / np.argsort order); internally
 * IDs travel as order-preserving uint64 keys (signed kinds: value ^ 2^63).
 */
#ifndef ORBIT_POST_H
#define ORBIT_POST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OA_ID_I64 0
#define OA_ID_U64 1
#define OA_ID_I32 2
#define OA_ID_U32 3

/* Raw apsis records of one collated chunk per halo: at most this many per halo per
 * oa_collate_step call (the LDS sort capacity); the host splits larger slices into
 * rounds (postprocessing.py:123-128 appends are order-free under np.unique). */
#define OA_COLLATE_CHUNK 4096
/* Largest n of get_central_particle_ids handled by oa_central_ids. */
#define OA_CENTRAL_MAX_N 4096

/* Status bits written by the f3/f4 kernels (int32 device word, OR-ed). */
#define OA_POST_MISSING 1u      /* oa_retro_counts: an ID absent from the final slice  */
#define OA_POST_SENTINEL 2u     /* oa_main_progenitors: an ID equals INT64_MIN           */
#define OA_POST_OVERFLOW 4u     /* oa_main_progenitors: a block's halo tally overflowed  */
#define OA_POST_BOUNDS 8u       /* oa_collate_step: a computed position fell outside its
                                   halo's range (inconsistent workspace); nothing stored  */

/* One round of collate_apsides for one snapshot: merge the kept apsis IDs of every
 * collated halo into its cumulative sorted-unique (key, count) state. */
typedef struct oa_collate_args {
    int32_t n_halos;            /* collated halos (the user's halo_ids order)               */
    int32_t in_kind;            /* dtype of apsis_ids                                      */
    int32_t key_signed;         /* order keys as signed (output kind signed)               */
    int32_t chunk_start;        /* round r: records [r*CHUNK, (r+1)*CHUNK) of each slice   */
    int32_t lds_keys;           /* sort slots: power of two in [64, CHUNK], >= every halo's
                                   record count this round                                */
    int32_t phases;             /* 0 or 3: the whole round; 1: k_collate_rank only (fills
                                   the w_* workspace); 2: k_collate_offsets + k_collate_place
                                   only, from the workspace a phases = 1 call filled        */
    const void *apsis_ids;      /* this snapshot's {peri|apo}center_IDs                    */
    const uint16_t *angles;     /* this snapshot's angles (float16 bits)                   */
    const uint8_t *keep_lut;    /* [65536]: 1 if (float16 value > angle_cut) in NumPy      */
    const int64_t *src_off;     /* [n_halos] start of halo j's slice in apsis_ids          */
    const int64_t *src_cnt;     /* [n_halos] its length (0 = halo not in this snapshot)    */
    const int64_t *new_base;    /* [n_halos] exclusive prefix of this round's chunk sizes  */
    const uint64_t *old_keys;   /* cumulative state in: sorted unique keys per halo, CSR   */
    const int64_t *old_cnt;
    const int64_t *old_off;     /* [n_halos + 1]; every halo's list < 2^31 elements        */
    int64_t n_old;              /* old_off[n_halos]                                        */
    int64_t n_new_cap;          /* sum of this round's chunk sizes                         */
    uint64_t *w_keys;           /* workspace [n_new_cap]: sorted unique new keys per halo  */
    int32_t *w_cnt;             /* [n_new_cap] their multiplicities                        */
    int32_t *w_lb;              /* [n_new_cap] old keys below each                         */
    int32_t *w_fp;              /* [n_new_cap] new keys below each already in the old list */
    int32_t *w_ulen;            /* [n_halos] unique new keys                               */
    int32_t *w_found;           /* [n_halos] of which already in the old list              */
    int64_t *new_off;           /* out [n_halos + 1] merged state offsets                  */
    uint64_t *new_keys;         /* out [n_old + n_new_cap] merged state (prefix used)      */
    int64_t *new_cnt;
    int32_t *status;            /* OR-ed OA_POST_BOUNDS (NULL: not reported).  Every store
                                   is checked against its halo's range first: a workspace
                                   row outside [new_base, n_new_cap), or a merged position
                                   outside [new_off[j], new_off[j + 1]), raises the bit and
                                   is dropped instead of faulting                          */
} oa_collate_args;

int oa_collate_step(const oa_collate_args *args, void *stream);

/* sizeof() of this header's ABI structs (0 oa_collate_args, 1 oa_central_args,
 * 2 oa_mainprog_args) so a binding can verify its layout; -1 otherwise. */
int64_t oa_post_struct_size(int32_t which);

/* Convert order keys back to IDs of `out_kind` (n elements). */
int oa_keys_to_ids(const uint64_t *keys, int64_t n, int32_t key_signed, int32_t out_kind,
                   void *out, void *stream);

/* save_final_apsis_counts for one collated snapshot: for each element e of segment h2
 * (ids[offs[h2]:offs[h2+1]], h2 < n_seg) out[e] = (double) counts_final[p] where p is
 * the position of ids[e] in final slice hinds[h2] (final_off[hinds[h2]] ..
 * final_off[hinds[h2] + 1]); elements outside every segment get 0; an ID absent from
 * its final slice sets OA_POST_MISSING in *status (the reference raises there). */
int oa_retro_counts(const void *ids, int32_t kind, int64_t n, const int64_t *offs,
                    const int64_t *hinds, int32_t n_seg, const void *ids_final,
                    const int64_t *final_off, const int64_t *counts_final,
                    double *out, int32_t *status, void *stream);

/* get_central_particle_ids over every region block. */
typedef struct oa_central_args {
    const void *coords;         /* (N,3) AoS, float32 or float64                           */
    int32_t coord_f64;
    int32_t dx_f64;             /* dtype of coordinates - position (NumPy promotion)       */
    const double *positions;    /* (n_halos,3) halo centres (values of the dx dtype)       */
    const void *ids;            /* (N,) raw IDs, id_bytes each                             */
    int32_t id_bytes;           /* 4 or 8 (copied through)                                 */
    int32_t n_halos;
    const int64_t *offsets;     /* [n_halos + 1] region block bounds                       */
    const int64_t *out_offsets; /* [n_halos] where block h's min(n, len) IDs go            */
    int32_t n;                  /* central particles per halo, <= OA_CENTRAL_MAX_N        */
    int32_t n_box_dims;         /* dims recentred (0 = no box_size; 1-element quirk = 1)   */
    int32_t wrap_f64[3];        /* comparison/subtraction dtype per dim                    */
    double box[3];              /* bs per dim, in that dtype                               */
    double half[3];             /* bs/2 as NumPy computes it, in that dtype                */
    uint64_t *scratch;          /* [N] radius keys for blocks larger than the LDS cache    */
    void *out_ids;              /* [sum min(n, len)]                                       */
} oa_central_args;

int oa_central_ids(const oa_central_args *args, void *stream);

/* find_main_progenitors.  IDs are compared as int64 values (kinds 0, 2, 3). */
typedef struct oa_mainprog_args {
    const void *halo_pids; int32_t halo_kind; int64_t n_halo_pids;
    const int64_t *halo_offsets; int32_t n_halos;
    const void *tracked; int32_t tracked_kind; int64_t n_tracked;
    const int64_t *tracked_offsets; int32_t n_blocks;   /* [n_blocks + 1]                 */
    int32_t max_block;          /* longest tracked block (sizes the per-block tally)       */
    uint64_t *tab_keys;         /* workspace: oa_mainprog_workspace_bytes()                */
    int64_t *result;            /* out [n_blocks]: halo number or -1                       */
    int32_t *status;
} oa_mainprog_args;

int64_t oa_mainprog_workspace_bytes(int64_t n_halo_pids, int64_t n_tracked);
int oa_main_progenitors(const oa_mainprog_args *args, void *stream);

/* Diagnostic builds only (-DOA_STAMPS=1): k_central's per-block phase timestamps of its
 * last launch (8 per block, s_memrealtime at 100 MHz).  Returns the number of values
 * copied, -1 in normal builds. */
int64_t oa_debug_central_stamps(uint64_t *host, int64_t n);

#ifdef __cplusplus
}
#endif

#endif /* ORBIT_POST_H */
