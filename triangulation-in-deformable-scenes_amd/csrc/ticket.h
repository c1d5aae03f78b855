// ticket.h — "am I the last workgroup of this launch?" without every workgroup hitting one address.
// Workgroup b counts in group counter 1 + (b % 8) (the XCD it runs on); the group's last workgroup
// then counts in the top counter cnt[0]; the last of those is the launch's last workgroup.  Call from
// one thread after its workgroup's partials are published and acknowledged; cnt[0..8] are zero
// between launches (the counters are reset, by agent-scope stores like the atomics that count in
// them, by the workgroups that finish them).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

namespace deftri {

// agent-scope relaxed loads / stores through the GLOBAL address space (global_load/store ... sc1):
// the hand-off values another workgroup of the same launch wrote; a generic pointer would lower to
// flat_ instructions, whose sc1 loads the MI355X memory-model notes do not count as bypassing a
// CU's stale L1 line
template <class T>
__device__ __forceinline__ T ld_sc1(const T *p) {
    using GP = const __attribute__((address_space(1))) T *;
    return __hip_atomic_load((GP)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_sc1(T *p, T v) {
    using GP = __attribute__((address_space(1))) T *;
    __hip_atomic_store((GP)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool ticket_last(int *cnt, int nblk, int bid) {
    const int x = bid & 7;
    const int gsize = (nblk - x + 7) >> 3;                 // workgroups b < nblk with b % 8 == x
    if (__hip_atomic_fetch_add(cnt + 1 + x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gsize - 1) return false;
    st_sc1(cnt + 1 + x, 0);                                // the group is done: nobody else touches it
    const int ngroups = nblk < 8 ? nblk : 8;
    if (__hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ngroups - 1) return false;
    st_sc1(cnt, 0);
    return true;
}

}  // namespace deftri
