// metrics.hip — calculatePixelsStandDev (reference Modules/Utils/Geometry.cc:370-498) on the device.
//
// Per matched slot of a keyframe pair the reference projects the MapPoint with the homogeneous
// fp32 product T.matrix() * [p; 1] (:423-431), KB8-projects it in fp32 and accumulates
// |obs - uv| and its square in u and v for both cameras (:440-452).  One thread per match computes
// the two error vectors; each workgroup reduces its 256 matches in a fixed tree order into one
// partial of 8 doubles (sum |e| and sum e^2, u and v, camera 1 then 2); the host adds the partials
// of each pair in order and replays the reference's per-pair formulas (deftri_pixels_stand_dev).
#include <hip/hip_runtime.h>

#include "device_math.h"
#include "kernels.h"

namespace deftri {
namespace dev {

// fp32, no contraction: Eigen's lazy 4x4 * 4x1 product, column by column (:426)
#pragma clang fp contract(off)
__device__ __forceinline__ void pix_err(const float *cam, const float *p, const float *obs, double e[2]) {
    // cam: R (row-major 3x3, from the fp32 unit quaternion), t (3), kb8 (8)
    float pc[3];
#pragma unroll
    for (int r = 0; r < 3; r++) pc[r] = ((cam[3 * r] * p[0] + cam[3 * r + 1] * p[1]) + cam[3 * r + 2] * p[2]) + cam[9 + r];
    float uv[2];
    kb8_project(cam + 12, pc, uv);
    e[0] = fabs((double)obs[0] - (double)uv[0]);
    e[1] = fabs((double)obs[1] - (double)uv[1]);
}

// matches [m0, m1) of one pair; block b of the launch covers matches blk_first[b] .. +256 within
// its pair (blocks never straddle pairs), camera slots c1/c2 of the pair
__global__ void __launch_bounds__(256) k_pix_partial(const int32_t *__restrict__ blk_first, const int32_t *__restrict__ blk_last,
                                                     const int32_t *__restrict__ blk_pair, const int32_t *__restrict__ pair_cams,
                                                     const float *__restrict__ cams, const float *__restrict__ pts,
                                                     const float *__restrict__ obs, double *__restrict__ part) {
    __shared__ double red[8][256];
    const int b = blockIdx.x;
    const int m = blk_first[b] + (int)threadIdx.x;
    double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (m < blk_last[b]) {
        const int pr = blk_pair[b];
        double e1[2], e2[2];
        pix_err(cams + 20 * pair_cams[2 * pr], pts + 6 * (int64_t)m, obs + 4 * (int64_t)m, e1);
        pix_err(cams + 20 * pair_cams[2 * pr + 1], pts + 6 * (int64_t)m + 3, obs + 4 * (int64_t)m + 2, e2);
        v[0] = e1[0]; v[1] = e1[1]; v[2] = e1[0] * e1[0]; v[3] = e1[1] * e1[1];
        v[4] = e2[0]; v[5] = e2[1]; v[6] = e2[0] * e2[0]; v[7] = e2[1] * e2[1];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) red[q][threadIdx.x] = v[q];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
#pragma unroll
            for (int q = 0; q < 8; q++) red[q][threadIdx.x] += red[q][threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x < 8) part[8 * (int64_t)b + threadIdx.x] = red[threadIdx.x][0];
}
#pragma clang fp contract(on)

}  // namespace dev

void launch_pixel_partials(int nblk, const int32_t *blk_first, const int32_t *blk_last, const int32_t *blk_pair,
                           const int32_t *pair_cams, const float *cams, const float *pts, const float *obs,
                           double *part, hipStream_t st) {
    if (nblk > 0)
        hipLaunchKernelGGL(dev::k_pix_partial, dim3(nblk), dim3(256), 0, st, blk_first, blk_last, blk_pair, pair_cams,
                           cams, pts, obs, part);
}

}  // namespace deftri
