// wave.h — fixed-order 64-lane wave reductions for gfx950 (no LDS).
#pragma once
#include <hip/hip_runtime.h>

namespace deftri {
namespace wv {

// xor butterflies over the 64 lanes without LDS: lane ^ 1 and ^ 2 by DPP quad_perm, ^ 4 and ^ 8 by
// row_half_mirror / row_mirror (equivalent once the quads / half-rows are uniform), ^ 16 and ^ 32
// by v_permlane16_swap / v_permlane32_swap.  Every lane ends with the same value (each step adds
// the same two operands on both lanes of a pair).
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {      // the 64-bit value as two 32-bit DPP moves
    int2 p = __builtin_bit_cast(int2, v);
    p.x = __builtin_amdgcn_update_dpp(0, p.x, CTRL, 0xf, 0xf, true);     // every lane has a source
    p.y = __builtin_amdgcn_update_dpp(0, p.y, CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, p);
}
__device__ __forceinline__ void swap16(double v, double &a, double &b) {   // a: rows (0,0,2,2), b: rows (1,1,3,3)
    const int2 p = __builtin_bit_cast(int2, v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)p.x, (unsigned)p.x, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)p.y, (unsigned)p.y, false, false);
    a = __builtin_bit_cast(double, make_int2((int)lo[0], (int)hi[0]));
    b = __builtin_bit_cast(double, make_int2((int)lo[1], (int)hi[1]));
}
__device__ __forceinline__ void swap32(double v, double &a, double &b) {   // a: rows (0,1,0,1), b: rows (2,3,2,3)
    const int2 p = __builtin_bit_cast(int2, v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)p.x, (unsigned)p.x, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)p.y, (unsigned)p.y, false, false);
    a = __builtin_bit_cast(double, make_int2((int)lo[0], (int)hi[0]));
    b = __builtin_bit_cast(double, make_int2((int)lo[1], (int)hi[1]));
}
__device__ __forceinline__ double wave_sum(double v) {
    v += dpp<0xB1>(v);      // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);      // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);     // row_half_mirror
    v += dpp<0x140>(v);     // row_mirror
    double a, b;
    swap16(v, a, b);
    v = a + b;
    swap32(v, a, b);
    return a + b;
}

__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, dpp<0xB1>(v));
    v = fmax(v, dpp<0x4E>(v));
    v = fmax(v, dpp<0x141>(v));
    v = fmax(v, dpp<0x140>(v));
    double a, b;
    swap16(v, a, b);
    v = fmax(a, b);
    swap32(v, a, b);
    return fmax(a, b);
}

}  // namespace wv
}  // namespace deftri
