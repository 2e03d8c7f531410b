/*
 * pss.h -- C-ABI of the MI355X partial-shuffle sampler (libpss.so).
 *
 * The reference (microsoft/PartiallyShuffleDistributedSampler) is pure Python; its index
 * generation lives inside two `torch.utils.data.Sampler` subclasses:
 *   V1 = DistributedSamplerViaLocallyShuffle.py, V2 = DistributedSamplerViaLocallyShuffleV2.py.
 * Each entry point below replaces the reference code cited next to it; the Python facade in
 * partiallyshuffledistributedsampler_amd/ binds them with ctypes.
 *
 * Conventions
 *   - every function returns PSS_OK (0) or a PSS_E* code; pss_last_error() has the text
 *     (thread-local).  No C++ exception crosses this boundary.
 *   - `*_dev` arguments are device pointers on the sampler's device; `stream` is a
 *     hipStream_t (NULL = default stream).  Device work is stream-ordered and asynchronous;
 *     nothing on the per-epoch path allocates once workspaces have grown to their size.
 *     Calls of one handle may use different streams without host synchronisation (e.g. epoch
 *     e + 1 generated on a second stream while epoch e is consumed): work that uses the
 *     handle's device tables and workspaces waits on the device for the last such call on
 *     another stream; whole-stream V2 counter-order generation (ranks as kernel arguments)
 *     uses none of them and overlaps with the previous epoch's.
 *   - a handle is not thread-safe; distinct handles share no state.
 *   - CPU mode: a handle created with device = PSS_DEVICE_CPU runs the same schedule on host
 *     threads (bit-identical to the GPU); every `*_dev` pointer is then a HOST pointer, `stream`
 *     is ignored and calls return when their work is done.  No HIP call is made, so it also
 *     runs on a machine without a GPU (BASELINE configs[0]).
 */
#ifndef PSS_H
#define PSS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pss_sampler pss_sampler;

#define PSS_OK 0
#define PSS_EINVAL 1    /* bad argument */
#define PSS_EHIP 2      /* HIP runtime error (text has hipGetErrorString) */
#define PSS_ENOTSUP 3   /* configuration outside what the kernels implement */
#define PSS_ESTATE 4    /* call out of order (e.g. generate before init_iter) */
#define PSS_EDEVICE 5   /* a kernel reported a device-side error flag */

#define PSS_DEVICE_CPU (-1)   /* pss_create device: the CPU mode */

const char *pss_last_error(void);
int pss_abi_version(void);

/* Version of the counter-order schedule (PSS_ORDER_COUNTER, DESIGN.md §3: the keyed
 * bijections, the slot hash, the grouped-pool layout).  It changes whenever some geometry's
 * counter-order id stream changes, so a resume position (find_ckpt_position) recorded under
 * another version would not continue the same permutation: the facade's state_dict() records it
 * and load_state_dict() refuses a mismatch.  The exact order is the reference's and never
 * changes. */
int pss_schedule_version(void);

/* Constructor math of __init__ (V1:16-56, V2:16-52):
 *   files_len[F]  -- per-file sample counts in dataset.files order (files_len dict, or the
 *                    reader(path, get_data=False) probe, V1:186-189)
 *   total_size    -- ori_total_size: sum over ALL files_len keys (V1:29-31), else total_size
 *   num_samples   =  int(math.ceil(total_size * 1.0 / num_replicas)) (V1:42)
 *   version       -- 1 (one pool) or 2 (two pools, TF-like); shuffle is ignored by V2.
 *   seed          -- Philox key of the pool permutations (extension; the reference has none)
 *   device        -- HIP device ordinal used for every device call of this handle, or
 *                    PSS_DEVICE_CPU for the CPU mode.
 * No device memory is touched until the first device call. */
int pss_create(const int64_t *files_len, int64_t num_files, int64_t total_size,
               int32_t num_replicas, int64_t shuffle_buffer, int32_t version, int32_t shuffle,
               uint64_t seed, int32_t device, pss_sampler **out);
int pss_destroy(pss_sampler *h);
int pss_num_samples(const pss_sampler *h, int64_t *num_samples);   /* __len__ (V1:261-262) */

/* One init_iter() for `epoch` (V1:100-132, V2:124-159): the cumulative file-order shuffle
 * (seed(e+1) in V1 / seed(e) in V2, CPython MT19937, exact), V1's cumulative block shuffle
 * (seed(e+2)) or V2's reset+shuffle (seed(e+1)), old/new start_num per rank.  Host-side,
 * O(F + R).  Every later device call works on this epoch. */
int pss_init_iter(pss_sampler *h, int64_t epoch);
int pss_file_order(const pss_sampler *h, int32_t *order /* [F] dataset positions */);
int pss_blocks(const pss_sampler *h, int32_t *blocks /* [R] */);
int pss_rank_starts(const pss_sampler *h, int64_t *old_start /* [R] */, int64_t *new_start /* [R] */);

/* Upload the epoch descriptors and run the device prefix scan over the shuffled files_len
 * (replaces the lazy past_files_samples scan, V1:181-190).  Implied by the calls below:
 * pss_generate needs only the upload; pss_map / pss_partition run the scan on first use. */
int pss_prepare(pss_sampler *h, void *stream);

/* Index generation (V1:151-172 / V2:96-116,170-176): positions [pos_lo, pos_lo+count) of
 * the per-epoch streams of logical ranks [rank_lo, rank_hi), written rank-major to
 * out_dev[(r - rank_lo) * count + (pos - pos_lo)] as int64 global sample ids.
 * Positions past num_samples are left untouched.  pos_lo = step*batch_size gives an O(1)
 * resume (find_ckpt_position, V1:134-140 / V2:118-122). */
int pss_generate(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo,
                 int64_t count, int64_t *out_dev, void *stream);

/* id -> (position in the shuffled file order, offset in that file) (V1:181-221).  Ids at or
 * past the scanned total are reflected as V1:191-196 does and flagged by
 * file_pos = -1 - f (the host moves them to the end of their batch). */
int pss_map(pss_sampler *h, const int64_t *ids_dev, int64_t n, int32_t *file_pos_dev,
            int64_t *offset_dev, void *stream);

/* Fused hand-off: the positions of pss_generate delivered directly as
 * (int32 file position in the shuffled order, int32 offset) -- 8 bytes per id, the form the
 * reader and an on-GPU gather consume (V1:181-221).  Same layout as pss_generate
 * ([r - rank_lo][pos - pos_lo]) and the same reflection flag as pss_map.  Counter order (V1,
 * and V2 on the exchange replays): one kernel, each id mapped where it is emitted (V2 pools up
 * to 16384 through a per-tile LDS map of the files its ids can come from, grouped pools
 * through the bucket-indexed map).  Exact order: the pipeline's output kernels map each id
 * through the bucket-indexed map where they would write it (no id scratch).  Only the V2
 * collision-probe path generates into handle scratch and then maps.  PSS_ENOTSUP if a file
 * holds 2^31 samples or more. */
int pss_generate_mapped(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t pos_lo,
                        int64_t count, int32_t *file_pos_dev, int32_t *offset_dev, void *stream);

/* On-GPU gather of rows of device-resident files (V1:243-248): out_dev[i] = the row_bytes-byte
 * row base_rows_dev[f] + offset_dev[i] of data_dev, f = the dataset-order index of shuffled file
 * position file_pos_dev[i] (reflected ids, file_pos < 0, read file -1 - file_pos).  base_rows_dev
 * has one entry per dataset file: its first row in data_dev.  Uses the current epoch's order. */
int pss_gather(pss_sampler *h, const void *data_dev, int64_t row_bytes, const int64_t *base_rows_dev,
               const int32_t *file_pos_dev, const int32_t *offset_dev, int64_t n, void *out_dev,
               void *stream);

/* File -> rank partition: for ranks [rank_lo, rank_hi), the (file position, lo, hi) segments
 * their epoch reads, in stream order of the id ranges.  seg_off_dev[0..n] is always written
 * (exclusive offsets); segments only when seg_cap >= seg_off_dev[n]. */
int pss_partition(pss_sampler *h, int32_t rank_lo, int32_t rank_hi, int64_t *seg_off_dev,
                  int32_t *seg_file_dev, int64_t *seg_lo_dev, int64_t *seg_hi_dev,
                  int64_t seg_cap, void *stream);

/* Coverage digest: *acc_dev += sum(splitmix64(id)) mod 2^64 (commutative, duplicate-
 * sensitive).  pss_digest_range digests the ids lo..hi-1. */
int pss_digest(const int64_t *ids_dev, int64_t n, uint64_t *acc_dev, void *stream);
int pss_digest_range(int64_t lo, int64_t hi, uint64_t *acc_dev, void *stream);
/* the same on host memory (CPU mode, or any host id array) */
int pss_digest_host(const int64_t *ids, int64_t n, uint64_t *acc);
int pss_digest_range_host(int64_t lo, int64_t hi, uint64_t *acc);

/* device ordinal of the handle, or PSS_DEVICE_CPU */
int pss_device(const pss_sampler *h, int32_t *device);

/* Kernel timing: enable = 1 brackets every launch of this handle with HIP events on its
 * stream; enable = n >= 2 only the index-generation kernels (v1_window, v2_emit), every
 * (n - 1)-th of their launches (two events per timed generate: live timing of the dominant
 * kernel at a fraction of the events' cost).  pss_profile_read synchronises on
 * them and returns, per kernel kind (0 scan, 1 v1_window, 2 v2_lastocc, 3 v2_emit, 4 v2_tail,
 * 5 map, 6 partition, 7 digest), the summed milliseconds and launch counts since the last
 * read; it then clears them. */
int pss_profile(pss_sampler *h, int32_t enable);
int pss_profile_read(pss_sampler *h, double *total_ms, int64_t *launches, int32_t nkinds);

/* Synchronise `stream` and report any device-side error flag of the handle. */
int pss_check(pss_sampler *h, void *stream);

/* Asynchronous form: enqueue on `stream` a copy of the device error word into *dst (pinned
 * host memory); nonzero once the stream has reached it means a kernel of this handle flagged
 * an error (a queued lookahead pass of a later epoch reports in a later snapshot).  The word is
 * sticky until pss_check clears it.  CPU mode: *dst = 0 at once. */
int pss_error_snapshot(pss_sampler *h, int32_t *dst, void *stream);

/* id -> (file position, offset) on the host against a caller-owned exclusive prefix of
 * `nfiles` files (prefix[0..nfiles]); same reflection rule and flags as pss_map.  Used by the
 * facade when file lengths are probed lazily in scan order (V1:181-190). */
int pss_map_prefix_host(const int64_t *prefix, int64_t nfiles, const int64_t *ids, int64_t n,
                        int32_t *file_pos, int64_t *offset);

/* V2 replay kernel selection (no effect on results, which are identical on every path):
 * 0 = auto (one LDS exchange per step when the device passed the start-up lane-order check,
 * else the collision-probe kernel), 1 = exchange kernel (PSS_ENOTSUP if the check failed),
 * 2 = collision-probe kernel.  pss_emit_path reports the path `auto` resolves to. */
int pss_set_emit_path(pss_sampler *h, int32_t path);
int pss_emit_path(pss_sampler *h, int32_t *path);

/* Order of the ids inside a pool (extension; the multiset and the file / rank assignment are
 * the reference's in both modes):
 *   PSS_ORDER_COUNTER (0, default) -- the counter-based schedule (Philox / Feistel, DESIGN.md
 *       §3): per-sampler, independent of the process-global `random` state;
 *   PSS_ORDER_EXACT   (1) -- the reference's own draws with CPython's MT19937, so the id
 *       stream is bit-identical to the reference's: V1 windows `seed(epoch + b*10000);
 *       shuffle(range(n))` (V1:102,114-115,165-171, shuffle_buffer < 2^31); V2 get_index's
 *       choice / remove / append with its per-window and per-tail-step reseeding (V2:96-116,
 *       num_samples < 2^31, shuffle_buffer < 2^30).  PSS_ENOTSUP outside those bounds.
 *       Device workspace: V1 windows beyond 16000 entries take ~18 B per entry of the windows
 *       one pass resolves (J, S, H, PART as u32 and PARTP as u16: <= 2.3 GB up to 2^27-entry
 *       windows, one window per pass beyond: ~19 GB at shuffle_buffer = 2^30, ~39 GB near
 *       2^31), windows up to 16000 entries 2 B per position and 2.5 KB per window (its
 *       seeded MT state); V2 ~28 B per position of num_samples and 2.5 KB per pool2 window --
 *       one decode serves every rank of a call, whatever their number.  A workspace the
 *       device cannot hold makes pss_generate return PSS_EHIP.  After calls for consecutive
 *       epochs of one shape, the MT draws of the next epochs (up to 8) are made ahead on the
 *       handle's own low-priority streams where they are few long streams (shuffle_buffer
 *       beyond 4096 with few windows), within pss_set_lookahead's bounds (1 GiB of draw slots
 *       by default); pss_destroy waits for them.
 * Replaces nothing in the reference: its order IS the exact one. */
#define PSS_ORDER_COUNTER 0
#define PSS_ORDER_EXACT 1
int pss_set_order_mode(pss_sampler *h, int32_t mode);
int pss_order_mode(const pss_sampler *h, int32_t *mode);

/* Bounds of the work a handle does ahead of its calls, and the device memory it holds for it
 * (extension; results never depend on them):
 *   exact_depth     -- exact order: epochs whose MT draws are made ahead (-1: by geometry, the
 *                      default -- up to 8 where a call's draws are few long serial streams, 0
 *                      where they fill the chip; 0: none; at most 8);
 *   exact_max_bytes -- the bytes ALL the exact draw slots together may hold, the one a call is
 *                      reading included (default 1 GiB; 0: none); the depth shrinks to fit;
 *   v2_depth        -- V2 counter order (pools up to 16384): epochs whose last-occurrence pass
 *                      is queued ahead on a low-priority stream (-1: 2, the default; 0: the pass
 *                      runs in line; 1 or 2), each in its own VAL buffer (v2 VAL ring).
 * Slot memory beyond the bounds is released by later calls once idle (no host wait).  The
 * lookaheads are best effort: an error while preparing one (e.g. hipMalloc of a slot) turns
 * the exact lookahead off for the handle and the call still returns PSS_OK; a later
 * pss_set_lookahead turns it back on.  PSS_EXACT_LOOKAHEAD=0 / PSS_V2_LOOKAHEAD=0 still force
 * them off process-wide. */
int pss_set_lookahead(pss_sampler *h, int32_t exact_depth, int64_t exact_max_bytes, int32_t v2_depth);
/* Device bytes the handle holds now: tables, workspaces, VAL ring, draw slots. */
int pss_workspace_bytes(const pss_sampler *h, int64_t *bytes);
/* Counters since create: stats[0] exact draw slots made ahead, [1] exact calls that used one,
 * [2] V2 passes queued ahead, [3] V2 replays that used one. */
int pss_lookahead_stats(const pss_sampler *h, int64_t *stats /* [4] */);

/* Self-test of the wave64 DPP scan primitive: out_dev[2i] = 64-bit inclusive wave scan,
 * out_dev[2i+1] = 32-bit one (low words), for n inputs. */
int pss_debug_wave_scan(const uint64_t *in_dev, uint64_t *out_dev, int64_t n, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PSS_H */
