// pss_kernels.h -- launch interface of the gfx950 kernels (implemented in pss_kernels.hip).
// Everything here is stream-ordered and allocation-free; workspaces are owned by the caller
// (pss_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pss {

struct RankDesc {       // per logical rank, uploaded once per init_iter
    int64_t old_start;  // start_num before this init_iter (V2 pools 0/1, V2:135-138)
    int64_t new_start;  // start_num after it (V1:121, V2:148)
};

struct Geometry {       // per-epoch constants of one sampler
    int64_t N;          // ori_total_size (V1:28-31)
    int64_t ns;         // num_samples = ceil(N/R) (V1:42)
    int64_t B;          // shuffle_buffer
    int32_t R;          // num_replicas
    int32_t version;    // 1 or 2
    int32_t shuffle;    // V1 only; V2 always shuffles (V2:142-152)
    uint32_t key0, key1;  // Philox key = epoch_key(seed, epoch)
};

struct V2Plan {         // slot-machine tiling of one V2 stream
    int64_t P1;         // slots = min(B, ns)
    int64_t T;          // replacement steps = ns - P1
    int64_t L;          // steps per tile
    int64_t G;          // tiles per rank = ceil(T / L)
    int32_t fold;       // 1: every virtual id < 2^24, probe byte folded into the slot word
    int64_t emit_lds;   // dynamic LDS of one k_v2_emit wave (padded to cap waves per CU)
    // 32-bit constants of the replay, computed on the host so that no kernel prologue runs a
    // 64-bit division (each one is ~100 scalar instructions of cold code per wave)
    uint32_t B32, L32, T32;    // shuffle_buffer, tile length, steps (T < 2^32)
    uint32_t hB, walk_full;    // Feistel half width of a full window; 1 if it needs walking
    uint32_t w_last, len_last, h_last;   // last pool2 window (may be short)
    uint32_t twoB;             // min(2B, ns): virtual ids below come from the OLD start
};

// optional per-kernel timing: `mark(ctx, kind, stream)` is called right before each launch
// and once more (kind = -1) after the last one; the runtime records HIP events there.
enum KernelKind { K_SCAN = 0, K_V1 = 1, K_V2_LASTOCC = 2, K_V2_EMIT = 3, K_V2_TAIL = 4,
                  K_MAP = 5, K_PARTITION = 6, K_DIGEST = 7, K_NUM_KINDS = 8 };
struct Marker {
    void (*mark)(void *ctx, int kind, hipStream_t s) = nullptr;
    void *ctx = nullptr;
    void operator()(int kind, hipStream_t s) const { if (mark) mark(ctx, kind, s); }
};

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kMarkBytes = 4096;    // V2 collision-probe bytes in LDS (slot & 4095)
constexpr int kBucketCap = 8192;    // largest bucket the HBM multi-pass sort finishes in LDS

// tiling of a launch over nr ranks: sized so that k_v2_emit fills every SIMD with two waves
V2Plan v2_plan(const Geometry &g, int32_t nr);

// rank descriptors host -> device through kernel arguments (128 per launch), R <= kArgRanksMax
constexpr int32_t kArgRanks = 128;
constexpr int32_t kArgRanksMax = 1024;
hipError_t launch_put_ranks(const RankDesc *host, int32_t R, RankDesc *dst, hipStream_t s);
// bytes (a multiple of 4) from pinned host memory (hipHostMalloc) to device memory by a kernel
hipError_t launch_upload(const void *host_pinned, void *dst, size_t bytes, hipStream_t s);
// up to kArgRanks rank descriptors by value (kernel arguments): [0, nr) = ranks rank_lo..
struct RankArgs { RankDesc r[kArgRanks]; };

// exclusive prefix over the shuffled file order: prefix[f] = sum_{j<f} len[order[j]]
// scratch: scan_scratch_words(F) words
hipError_t launch_scan_prefix(const int64_t *lens, const int32_t *order, int64_t F,
                              int64_t *prefix, uint64_t *scratch, hipStream_t s);
size_t scan_scratch_words(int64_t F);

// per-rank file segments of ranks [rank_lo, rank_lo+nr); counts-only when seg_cap == 0
hipError_t launch_partition(const Geometry &g, const RankDesc *ranks, int32_t rank_lo,
                            int32_t nr, const int64_t *prefix, int64_t F, int64_t *seg_off,
                            int32_t *seg_file, int64_t *seg_lo, int64_t *seg_hi,
                            int64_t seg_cap, int32_t *err, hipStream_t s);

// bucket index of the prefix (pss_map.h map_one_bucketed), then the map itself: int64 offsets
// into `off`, or int32 ones into `off32` when that is non-null
hipError_t launch_bucket_index(const int64_t *prefix, int64_t F, int32_t kb, int64_t nb, int32_t *BT,
                               hipStream_t s);
hipError_t launch_map(const int64_t *prefix, int64_t F, const int32_t *BT, int32_t kb, int64_t nb,
                      const int64_t *ids, int64_t n, int32_t *fpos, int64_t *off, int32_t *off32,
                      hipStream_t s);
// rows of device-resident files: out[i] = data row base[order[|f_i|]] + off_i
hipError_t launch_gather(const void *data, int64_t row_bytes, const int64_t *base, const int32_t *order,
                         const int32_t *fpos, const int32_t *off, int64_t n, void *out, hipStream_t s);

hipError_t launch_digest(const int64_t *ids, int64_t n, uint64_t *acc, hipStream_t s);
hipError_t launch_digest_range(int64_t lo, int64_t hi, uint64_t *acc, hipStream_t s);

// the epoch's prefix + bucket index, and (int32 file, int32 offset) outputs of a mapped launch
struct MapArgs {
    const int64_t *prefix;
    int64_t F;
    const int32_t *BT;
    int32_t kb;
    int64_t nb;
    int32_t *fpos, *off;
    // host-known shortcuts of the map (map_shortcuts, pss_runtime.cpp; all zero = none):
    int64_t T;          // scanned total prefix[F] = sum of the dataset files' lengths
    // pack: every (file position, offset) pair fits 31 bits as (file << pob) | offset (the
    // exchange replay then carries pairs in its slot table)
    uint32_t pack, pob;
    // uni: every file holds uL samples and T < 2^32: file = id / uL by the round-up magic
    // (um, ul) of udiv_magic, offset = id - file * uL, for ids < T
    uint32_t uni, uL, um, ul;
};

// u32 division by an invariant d >= 1 (Granlund-Montgomery round-up form): l = ceil(log2 d),
// m = floor(2^32 (2^l - d) / d) + 1; q = (t + ((n - t) >> 1)) >> (l - 1), t = mulhi(m, n);
// d = 1: l = 0, m = 0 and q = n (udiv_apply's l == 0 case)
inline void udiv_magic(uint32_t d, uint32_t &m, uint32_t &l) {
    l = 0;
    while (l < 32 && ((uint64_t)1 << l) < d) l++;
    m = d <= 1 ? 0u : (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
}
__host__ __device__ inline uint32_t udiv_apply(uint32_t n, uint32_t m, uint32_t l) {
    if (l == 0) return n;
    const uint32_t t = (uint32_t)(((uint64_t)m * n) >> 32);   // v_mul_hi_u32 on the device
    return (t + ((n - t) >> 1)) >> (l - 1);
}

// V1: ids of positions [pos_lo, pos_lo+count) of ranks [rank_lo, rank_lo+nr) -> out[r][count];
// each window ordered by its keyed Feistel bijection (key table of the windows in key_ws).
// mapped != nullptr: (file position, offset) into mapped->fpos / off instead (out unused).
// rank_args != nullptr (nr <= kArgRanks): ranks [rank_lo, rank_lo+nr)'s descriptors by value;
// the device table `ranks` is then refreshed from them only where a kernel reads it
hipError_t launch_v1(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *key_ws,
                     hipStream_t s, const Marker &mk = Marker(), const MapArgs *mapped = nullptr,
                     const RankArgs *rank_args = nullptr);
size_t v1_workspace_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count);

// V1 in the reference's exact order (CPython MT19937 per window, pss_v1exact.hip): windows up
// to kV1ExactMaxB elements resolve in LDS ((624 + n + 1) words and 3n u16 <= 160 KB), larger
// ones (shuffle_buffer < 2^31) through HBM-staged draw and bucket arrays
constexpr int64_t kV1ExactMaxB = 16000;
bool v1_exact_supported(const Geometry &g);
size_t v1_exact_ws_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count);
// mapped != nullptr (pss_generate_mapped): (file, offset) pairs into mapped->fpos / off in
// place of the ids (out unused), through the global bucketed map -- same values as pss_map
hipError_t launch_v1_exact(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                           int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out, void *ws,
                           hipStream_t s, const MapArgs *mapped = nullptr, uint32_t *slot = nullptr);
// a draw slot of a call's windows (0 bytes: none -- windows through HBM in several passes) and
// the epochs the runtime draws ahead for it (as the V2 slots below)
size_t v1_exact_slot_bytes(const Geometry &g, int64_t pos_lo, int64_t count);
int v1_exact_lookahead_depth(const Geometry &g, int64_t pos_lo, int64_t count);
hipError_t launch_v1_exact_draws(const Geometry &g, int64_t pos_lo, int64_t count, int64_t epoch,
                                 uint32_t *slot, hipStream_t s);

// V2 in the reference's exact order (pss_v2exact.hip): shuffle_buffer < 2^30, ns < 2^31
bool v2_exact_supported(const Geometry &g);
size_t v2_exact_ws_bytes(const Geometry &g, int32_t nr);
// a draw slot: one epoch's MT draws (they depend on the epoch and (ns, B) only); the runtime
// fills slots of coming epochs ahead of their calls and passes one as `slot` (else the call
// draws into its workspace's own slot)
size_t v2_exact_slot_bytes(const Geometry &g);
int v2_exact_lookahead_depth(const Geometry &g);   // epochs drawn ahead (0: none)
hipError_t launch_v2_exact_draws(const Geometry &g, int64_t epoch, uint32_t *slot, hipStream_t s);
// V1's long windows drawn in the split form (pss_v2split.h; pss_v2exact.hip): false when the
// workgroup form should run instead (scratch null: draws made ahead into a slot)
bool v1x_draws_split(int64_t w_lo, uint32_t nj, uint32_t n_full, uint32_t n_last, uint32_t B, uint32_t nbk,
                     int64_t epoch, uint32_t *J, uint32_t *BCNT, uint32_t *scratch, size_t scratch_words,
                     bool wg_form, hipStream_t s);
hipError_t launch_v2_exact(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                           int64_t pos_lo, int64_t count, int64_t epoch, int64_t *out, uint32_t *ws,
                           hipStream_t s, const MapArgs *mapped = nullptr, uint32_t *slot = nullptr);

// V2 replay kernel: EMIT_XCHG = one LDS exchange per step (needs the lane-ordered exchange the
// start-up check confirms), EMIT_PROBE = collision probe + per-clash fix-up (any hardware)
enum EmitPath { EMIT_AUTO = 0, EMIT_XCHG = 1, EMIT_PROBE = 2 };
enum V2Stage { V2_STAGE_ALL = 0, V2_STAGE_PRE = 1, V2_STAGE_EMIT = 2 };
bool lds_xchg_ordered();   // result of the start-up check on the current device
bool lds_write_ordered();  // same-word lanes of one plain LDS store: the highest lane wins
bool lds_add_ordered();    // same-word lanes of one ds_add_rtn are served in lane order

// V2: same contract; val_ws holds the per-tile slot tables
hipError_t launch_v2(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *val_ws,
                     uint32_t *buf_ws, uint32_t *sort_ws, int32_t *err, hipStream_t s,
                     const Marker &mk = Marker(), int emit_path = EMIT_AUTO,
                     int stage = V2_STAGE_ALL, const MapArgs *mapped = nullptr,
                     const RankArgs *rank_args = nullptr);
// launch_v2 can take this launch's rank descriptors by value (rank_args, nr <= kArgRanks): the
// exchange replay then reads no device rank table, and the epoch path launches no upload
bool v2_ranks_by_value(const Geometry &g, int32_t nr, int emit_path);
// mapped != nullptr (v2_mapped_fused shapes only): (file, offset) instead of ids
bool v2_mapped_fused(const Geometry &g, int emit_path);
size_t v2_val_bytes(const Geometry &g, int32_t nr);
// V2 tail from per-tile VAL tables (walk-back), positions [pos_lo, pos_lo+count) past T
hipError_t launch_v2_tail_vals(const Geometry &g, const V2Plan &pl, const RankDesc *ranks,
                               int32_t rank_lo, int32_t nr, const uint32_t *VAL, int64_t pos_lo,
                               int64_t count, int64_t *out, hipStream_t s,
                               const MapArgs *mapped = nullptr, const RankArgs *rank_args = nullptr);
// pools beyond LDS (P1 > kLdsSlotMax): the grouped slot machine (pss_v2grp.hip); its key
// table and per-tile tables live in val_ws (v2_val_bytes)
bool v2_grouped(const Geometry &g);
size_t v2_grp_val_bytes(const Geometry &g, int32_t nr);
int64_t v2_grp_tiles(const Geometry &g, int32_t nr);   // tiles per (rank, group) stream
hipError_t launch_v2_grp(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                         int64_t pos_lo, int64_t count, int64_t *out, uint32_t *val_ws,
                         hipStream_t s, const Marker &mk, bool ordered, int stage,
                         const RankArgs *rank_args = nullptr, const MapArgs *mapped = nullptr);
hipError_t init_kernel_attributes_v2grp();
// launch_v2 splits into V2_STAGE_PRE / V2_STAGE_EMIT for this shape and emit path (EMIT_AUTO resolved)
bool v2_stage_split(const Geometry &g, int32_t nr, int emit_path);
size_t v2_buf_bytes(const Geometry &g, int32_t nr);
size_t v2_sort_bytes(const Geometry &g, int32_t nr);

// self-test of the wave64 DPP scan (device vs serial), used by the GPU tests
hipError_t launch_debug_wave_scan(const uint64_t *in, uint64_t *out, int64_t n, hipStream_t s);

hipError_t init_kernel_attributes();
hipError_t init_kernel_attributes_v2();



}  // namespace pss
