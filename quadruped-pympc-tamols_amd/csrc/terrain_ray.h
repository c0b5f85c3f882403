// terrain_ray.h -- vertical rays against the device-resident terrain scene (float64).
// Shared by terrain_patch_kernel (terrain_kernel.hip) and the fused TAMOLS launch (tamols_kernel.hip),
// so a patch point is computed one way everywhere (bit-identical to oracle/terrain_oracle.py under
// -ffp-contract=off).  A ray's result is the highest surface top at or below ray_z, a maximum, so the
// surfaces may be split over several lanes and the partial results combined in any order (ray_merge).
#pragma once

#include <math.h>

#include "srbd_launch.h"

namespace srbd {

__device__ __forceinline__ void ray_consider(double top, double ray_z, double& best, int& hit) {
    if (top <= ray_z && top > best) {
        best = top;
        hit = 1;
    }
}

// x, y of point (i, k) of a rows x cols patch centred at (cx, cy), yawed by (c, s) = (cos, sin).
__device__ __forceinline__ void ray_xy(double cx, double cy, double c, double s, int rows, int cols, int i, int k,
                                       double dist_x, double dist_y, double& x, double& y) {
    const double dx = ((double)i - (double)(rows - 1) / 2.0) * dist_x;
    const double dy = ((double)k - (double)(cols - 1) / 2.0) * dist_y;
    x = cx + c * dx - s * dy;
    y = cy + s * dx + c * dy;
}

// Primitives [q0, q1) of the scene (yawed box tops, upright cylinder tops); `prims` / `cs` may point
// into LDS.  Every lane of a wave walks the same range, so the primitive loads are wave-uniform.
__device__ __forceinline__ void ray_walk_prims(const srbd_terrain_prim* prims, const double* cs, int q0, int q1,
                                               double x, double y, double ray_z, double& best, int& hit) {
#pragma unroll 4
    for (int q = q0; q < q1; ++q) {
        const srbd_terrain_prim& pr = prims[q];
        const double ux = x - pr.cx, uy = y - pr.cy;
        bool in;
        if (pr.type == SRBD_PRIM_BOX) {
            const double cb = cs[2 * q], sb = cs[2 * q + 1];
            const double u = cb * ux + sb * uy, v = cb * uy - sb * ux;
            in = fabs(u) <= pr.a && fabs(v) <= pr.b;
        } else {
            in = ux * ux + uy * uy <= pr.a * pr.a;
        }
        if (in) ray_consider(pr.cz + pr.c, ray_z, best, hit);
    }
}

// The same over the primitives listed in idx[q0, q1) (the ones a patch can touch, TAMOLS's culled list).
__device__ __forceinline__ void ray_walk_list(const srbd_terrain_prim* prims, const double* cs, const int* idx, int q0,
                                              int q1, double x, double y, double ray_z, double& best, int& hit) {
#pragma unroll 2
    for (int n = q0; n < q1; ++n) {
        const int q = idx[n];
        const srbd_terrain_prim& pr = prims[q];
        const double ux = x - pr.cx, uy = y - pr.cy;
        bool in;
        if (pr.type == SRBD_PRIM_BOX) {
            const double cb = cs[2 * q], sb = cs[2 * q + 1];
            const double u = cb * ux + sb * uy, v = cb * uy - sb * ux;
            in = fabs(u) <= pr.a && fabs(v) <= pr.b;
        } else {
            in = ux * ux + uy * uy <= pr.a * pr.a;
        }
        if (in) ray_consider(pr.cz + pr.c, ray_z, best, hit);
    }
}

// The ground plane and the height field (cells split along the (i, j)-(i+1, j+1) diagonal).
__device__ __forceinline__ void ray_walk_fields(const TerrainDev& t, double x, double y, double ray_z, double& best,
                                                int& hit) {
    if (t.has_ground) ray_consider(t.ground_z, ray_z, best, hit);
    if (t.hf) {
        const double fx = (x - t.hf_x0) / t.hf_dx, fy = (y - t.hf_y0) / t.hf_dy;
        if (fx >= 0.0 && fy >= 0.0 && fx <= (double)(t.hf_nx - 1) && fy <= (double)(t.hf_ny - 1)) {
            int i0 = (int)floor(fx), j0 = (int)floor(fy);
            i0 = i0 > t.hf_nx - 2 ? t.hf_nx - 2 : i0;
            j0 = j0 > t.hf_ny - 2 ? t.hf_ny - 2 : j0;
            const double tx = fx - (double)i0, ty = fy - (double)j0;
            const double z00 = t.hf[i0 * t.hf_ny + j0], z10 = t.hf[(i0 + 1) * t.hf_ny + j0];
            const double z01 = t.hf[i0 * t.hf_ny + j0 + 1], z11 = t.hf[(i0 + 1) * t.hf_ny + j0 + 1];
            const double z =
                tx >= ty ? z00 + tx * (z10 - z00) + ty * (z11 - z10) : z00 + ty * (z01 - z00) + tx * (z11 - z01);
            ray_consider(z, ray_z, best, hit);
        }
    }
}

// Combine two partial results of one ray (max of the surfaces found; order-free).
__device__ __forceinline__ void ray_merge(double b2, int h2, double& best, int& hit) {
    if (h2 && (!hit || b2 > best)) {
        best = b2;
        hit = 1;
    }
}

// One whole ray: point (i, k) -> o = (x, y, z or t.miss_z).
__device__ __forceinline__ void terrain_ray_point(const TerrainDev& t, double cx, double cy, double c, double s,
                                                  int rows, int cols, int i, int k, double dist_x, double dist_y,
                                                  double ray_z, double* o) {
    double x, y;
    ray_xy(cx, cy, c, s, rows, cols, i, k, dist_x, dist_y, x, y);
    double best = -INFINITY;
    int hit = 0;
    ray_walk_fields(t, x, y, ray_z, best, hit);
    ray_walk_prims(t.prims, t.cs, 0, t.nprims, x, y, ray_z, best, hit);
    o[0] = x;
    o[1] = y;
    o[2] = hit ? best : t.miss_z;
}

}  // namespace srbd
