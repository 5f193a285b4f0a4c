// adlbq_donor.h -- device-side steal donor selection (one wavefront, lanes = servers).
//
// find_cand_rank_with_worktype (src/adlb.c:3487-3534): the first tq entry for
// (rank, type) wins (tq_find_first_rt, xq.c:539-554); otherwise the server i !=
// self, without an outstanding RFR (rfr_out), with qlen_unpin_untarg > 0, whose
// type_hi_prio for the type (wildcard: over all types) is largest, strictly above
// ADLB_LOWEST_PRIO, lowest index on ties.  The reference walks servers in a
// scalar loop; here 64 servers are compared per wave instruction and the
// (value desc, index asc) argmax is one 64-bit wave max.
#pragma once
#include "adlbq_impl.h"

namespace adlbq {

struct DonorCtx {
    const int *qm_hi;     // [S][T]
    const int *qm_qlen;   // [S]
    const int *tq;        // [n_tq][4]
    const int *utypes;    // [T]
    int *rfr_out;         // [num_world]
    int *rfr_to_rank;     // [A]
    int S, T, n_tq, master, my_world, A, num_world;
};

// L1-bypassing (sc1) accesses for state that one wave writes and later re-reads
// (per-CU vector L1 is not refreshed by stores: MI355X_MICROARCH.md, Workgroup dispatch)
__device__ __forceinline__ int ld_agent(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long w = __shfl_xor(v, o, 64);
        v = v > w ? v : w;
    }
    return v;
}

// wave-uniform call; returns the donor server's world rank or -1
__device__ inline int find_cand(const DonorCtx &c, int for_rank, int work_type) {
    const int lane = __lane_id();
    for (int base = 0; base < c.n_tq; base += 64) {
        int k = base + lane;
        bool hit = false;
        int srv = -1;
        if (k < c.n_tq) {
            const int *e = c.tq + 4 * k;
            hit = e[0] == for_rank && (work_type == -1 || work_type == e[1]);
            srv = e[2];
        }
        unsigned long long b = __ballot(hit);
        if (b) return __shfl(srv, __ffsll((long long)b) - 1, 64);
    }
    int ti = -1;
    if (work_type >= 0) {
        for (int base = 0; base < c.T; base += 64) {
            int k = base + lane;
            unsigned long long b = __ballot(k < c.T && c.utypes[k] == work_type);
            if (b) { ti = base + __ffsll((long long)b) - 1; break; }
        }
        if (ti < 0) return -1;  // undeclared type: no candidate (reference reads out of bounds here)
    }
    unsigned long long best = 0;
    for (int base = 0; base < c.S; base += 64) {
        int i = base + lane;
        unsigned long long key = 0;
        if (i < c.S) {
            int srv = c.master + i;
            if (srv != c.my_world && !ld_agent(c.rfr_out + srv) && c.qm_qlen[i] > 0) {
                int v = LOWEST;
                const int *row = c.qm_hi + (long long)i * c.T;
                if (work_type < 0) {
                    for (int j = 0; j < c.T; j++) v = row[j] > v ? row[j] : v;
                } else {
                    v = row[ti];
                }
                if (v > LOWEST)
                    key = ((unsigned long long)((unsigned int)v ^ 0x80000000u) << 32) |
                          (unsigned long long)(0xffffffffu - (unsigned int)i);
            }
        }
        key = wave_max_u64(key);
        if (key > best) best = key;  // earlier chunks hold lower indices: keep them on ties
    }
    if (!best) return -1;
    return c.master + (int)(0xffffffffu - (unsigned int)(best & 0xffffffffu));
}

// Could find_cand return a server at all (tq aside)?  Some server i != self
// without an outstanding RFR, qlen > 0 and a type above LOWEST.  Once none is
// left, every later parked request of the batch gets no donor.  Wave-uniform.
__device__ inline bool any_donor(const DonorCtx &c) {
    const int lane = __lane_id();
    for (int base = 0; base < c.S; base += 64) {
        const int i = base + lane;
        bool ok = false;
        if (i < c.S) {
            const int srv = c.master + i;
            if (srv != c.my_world && !ld_agent(c.rfr_out + srv) && c.qm_qlen[i] > 0) {
                const int *row = c.qm_hi + (long long)i * c.T;
                for (int j = 0; j < c.T && !ok; j++) ok = row[j] > LOWEST;
            }
        }
        if (__ballot(ok)) return true;
    }
    return false;
}

DonorCtx donor_ctx(adlbq_server *h);  // host: snapshot of the device pointers / sizes

// the RFR part of FA_RESERVE / check_remote (adlb.c:1280-1308, 3549-3577)
__device__ inline int rfr_select(const DonorCtx &c, int rank, const int *types16) {
    for (int i = 0; i < NREQ; i++) {
        int t = types16[i];
        if (t < -1) break;
        int cand = find_cand(c, rank, t);
        if (cand >= 0) {
            if (__lane_id() == 0) {
                if (rank >= 0 && rank < c.A) st_agent(c.rfr_to_rank + rank, cand);
                if (cand < c.num_world) st_agent(c.rfr_out + cand, 1);
            }
            __builtin_amdgcn_s_waitcnt(0);  // stores reach L2 before this wave's next sc1 loads
            return cand;
        }
    }
    return -1;
}

}  // namespace adlbq
