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
    int32_t global_buf; // 1: slot table lives in HBM scratch (P1 beyond the LDS budget)
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

constexpr int kLdsSortMax = 16384;  // largest pool sorted entirely in LDS
constexpr int kLdsSlotMax = 16384;  // largest V2 slot table kept in LDS
constexpr uint32_t kNone = 0xFFFFFFFFu;

V2Plan v2_plan(const Geometry &g);

// exclusive prefix over the shuffled file order: prefix[f] = sum_{j<f} len[order[j]]
hipError_t launch_scan_prefix(const int64_t *lens, const int32_t *order, int64_t F,
                              int64_t *prefix, hipStream_t s);

// per-rank file segments of ranks [rank_lo, rank_lo+nr); counts-only when seg_cap == 0
hipError_t launch_partition(const Geometry &g, const RankDesc *ranks, int32_t rank_lo,
                            int32_t nr, const int64_t *prefix, int64_t F, int64_t *seg_off,
                            int32_t *seg_file, int64_t *seg_lo, int64_t *seg_hi,
                            int64_t seg_cap, int32_t *err, hipStream_t s);

hipError_t launch_map(const int64_t *prefix, int64_t F, const int64_t *ids, int64_t n,
                      int32_t *fpos, int64_t *off, hipStream_t s);

hipError_t launch_digest(const int64_t *ids, int64_t n, uint64_t *acc, hipStream_t s);
hipError_t launch_digest_range(int64_t lo, int64_t hi, uint64_t *acc, hipStream_t s);

// V1: ids of positions [pos_lo, pos_lo+count) of ranks [rank_lo, rank_lo+nr) -> out[r][count]
hipError_t launch_v1(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *sort_ws,
                     int32_t *err, hipStream_t s, const Marker &mk = Marker());
size_t v1_workspace_bytes(const Geometry &g, int32_t nr, int64_t pos_lo, int64_t count);

// V2: same contract; val_ws holds the per-tile slot tables
hipError_t launch_v2(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
                     int64_t pos_lo, int64_t count, int64_t *out, uint32_t *val_ws,
                     uint32_t *buf_ws, uint32_t *sort_ws, int32_t *err, hipStream_t s,
                     const Marker &mk = Marker());
size_t v2_val_bytes(const Geometry &g, int32_t nr);
size_t v2_buf_bytes(const Geometry &g, int32_t nr);
size_t v2_sort_bytes(const Geometry &g, int32_t nr);

// self-test of the wave64 DPP scan (device vs serial), used by the GPU tests
hipError_t launch_debug_wave_scan(const uint64_t *in, uint64_t *out, int64_t n, hipStream_t s);

hipError_t init_kernel_attributes();



}  // namespace pss
