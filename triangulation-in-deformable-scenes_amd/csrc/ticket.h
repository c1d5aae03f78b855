// ticket.h — "am I the last workgroup of this launch?" without every workgroup hitting one address.
// Workgroup b counts in group counter 1 + (b % 8) (the XCD it runs on); the group's last workgroup
// then counts in the top counter cnt[0]; the last of those is the launch's last workgroup.  Call from
// one thread after its workgroup's partials are published and acknowledged; cnt[0..8] are zero
// between launches (the counters are reset by the workgroups that finish them).
// DEFTRI_FLAT_TICKET=1 selects the single-counter ticket for A/Bs.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

namespace deftri {

__device__ __forceinline__ bool ticket_last(int *cnt, int nblk, int bid, bool flat = false) {
    if (flat) {                                            // one counter for every workgroup (A/B)
        if (__hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nblk - 1) return false;
        cnt[0] = 0;
        return true;
    }
    const int x = bid & 7;
    const int gsize = (nblk - x + 7) >> 3;                 // workgroups b < nblk with b % 8 == x
    if (__hip_atomic_fetch_add(cnt + 1 + x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gsize - 1) return false;
    cnt[1 + x] = 0;                                        // the group is done: nobody else touches it
    const int ngroups = nblk < 8 ? nblk : 8;
    if (__hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ngroups - 1) return false;
    cnt[0] = 0;
    return true;
}

// the DEFTRI_FLAT_TICKET switch, read once on the host
inline bool flat_ticket() {
    static const bool v = std::getenv("DEFTRI_FLAT_TICKET") != nullptr;
    return v;
}

}  // namespace deftri
