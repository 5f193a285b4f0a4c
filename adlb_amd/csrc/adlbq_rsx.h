// adlbq_rsx.h -- hand-written LSD radix sort of (u64 key, int value) pairs on
// gfx950, the engine's general-purpose device sort (the targeted index's full
// build, the candidate lists' fallback sorts).  Stable, ascending or
// descending, over the key bits [lo, hi).
//
// One pass per 8-bit digit, three launches each:
//   k_rsx_hist     per tile of RSX_TILE keys, the 256-digit histogram
//                  (digit-major: hist[d][tile]);
//   k_rsx_scan     per digit, the exclusive prefix of its row over the tiles
//                  and the row total;
//   k_rsx_scatter  per tile: digit base (exclusive prefix of the row totals,
//                  recomputed by every workgroup from 256 words) + the tile's
//                  row prefix + the rank within the tile, which keeps input
//                  order (each wave ranks its run of 64-key steps in order:
//                  lanes with equal digits by a ballot match, the steps by a
//                  running count per digit; waves by a prefix over the waves).
// Passes alternate between the output and a scratch pair so that the last
// one writes the output and the input is left as it was.
#ifndef ADLBQ_RSX_H
#define ADLBQ_RSX_H

#include <hip/hip_runtime.h>

#include <cstddef>

namespace adlbq {

constexpr int RSX_THREADS = 256;
constexpr int RSX_STEPS = 8;                                  // 64-key steps per wave
constexpr int RSX_TILE = (RSX_THREADS / 64) * RSX_STEPS * 64;  // 2048 keys per workgroup

// bytes of scratch for n keys (query), then the sort itself (enqueued on s)
size_t rsx_temp_bytes(long long n);
int rsx_sort_pairs(void *tmp, size_t tmp_bytes, const unsigned long long *kin, unsigned long long *kout,
                   const int *vin, int *vout, long long n, int lo_bit, int hi_bit, bool descending, hipStream_t s);

}  // namespace adlbq

#endif
