// pss_cpu.h -- the product's CPU mode (device = PSS_DEVICE_CPU): the same counter schedule as
// the gfx950 kernels, computed from the same pss_common.h definitions on host threads, so it
// matches the GPU bit for bit; plus the reference's exact order (CPython MT19937).
// BASELINE configs[0] (C1) runs here on a box without a GPU.
#pragma once
#include <stdint.h>

#include "pss_kernels.h"

namespace pss {
namespace cpu {

// positions [pos_lo, pos_lo + count) of ranks [rank_lo, rank_lo + nr) -> out[(r - rank_lo) *
// count + (pos - pos_lo)] (host memory); positions past num_samples are left untouched
void generate(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr, int64_t pos_lo,
              int64_t count, int64_t epoch, bool exact, int64_t *out);

// exclusive prefix over the shuffled file order (F + 1 entries)
void scan_prefix(const int64_t *lens, const int32_t *order, int64_t F, int64_t *prefix);

void map(const int64_t *prefix, int64_t F, const int64_t *ids, int64_t n, int32_t *fpos,
         int64_t *off);

// per-rank file segments; counts only (seg_off) when seg_cap == 0; false if seg_cap is short
bool partition(const Geometry &g, const RankDesc *ranks, int32_t rank_lo, int32_t nr,
               const int64_t *prefix, int64_t F, int64_t *seg_off, int32_t *seg_file,
               int64_t *seg_lo, int64_t *seg_hi, int64_t seg_cap);

uint64_t digest(const int64_t *ids, int64_t n);
uint64_t digest_range(int64_t lo, int64_t hi);

int threads();   // worker threads (PSS_CPU_THREADS, else the process's CPU affinity)

}  // namespace cpu
}  // namespace pss
