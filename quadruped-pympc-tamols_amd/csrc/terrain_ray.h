// terrain_ray.h -- one vertical ray against the device-resident terrain scene (float64).
// Shared by terrain_patch_kernel (terrain_kernel.hip) and the fused TAMOLS launch (tamols_kernel.hip),
// so a patch point is computed one way everywhere (bit-identical to oracle/terrain_oracle.py under
// -ffp-contract=off).
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

// Point (i, k) of a rows x cols patch centred at (cx, cy), yawed by (c, s) = (cos, sin): its x, y and the
// highest surface at or below ray_z (ground plane, yawed box tops, upright cylinder tops, then the height
// field split along one diagonal), else t.miss_z.  Every lane walks the same primitive list, so the
// primitive loads are wave-uniform.
__device__ __forceinline__ void terrain_ray_point(const TerrainDev& t, double cx, double cy, double c, double s,
                                                  int rows, int cols, int i, int k, double dist_x, double dist_y,
                                                  double ray_z, double* o) {
    const double dx = ((double)i - (double)(rows - 1) / 2.0) * dist_x;
    const double dy = ((double)k - (double)(cols - 1) / 2.0) * dist_y;
    const double x = cx + c * dx - s * dy;
    const double y = cy + s * dx + c * dy;
    double best = -INFINITY;
    int hit = 0;
    if (t.has_ground) ray_consider(t.ground_z, ray_z, best, hit);
    // unrolled so several primitives' (wave-uniform, scalar) loads are in flight per round trip
#pragma unroll 4
    for (int q = 0; q < t.nprims; ++q) {
        const srbd_terrain_prim& pr = t.prims[q];
        const double ux = x - pr.cx, uy = y - pr.cy;
        bool in;
        if (pr.type == SRBD_PRIM_BOX) {
            const double cb = t.cs[2 * q], sb = t.cs[2 * q + 1];
            const double u = cb * ux + sb * uy, v = cb * uy - sb * ux;
            in = fabs(u) <= pr.a && fabs(v) <= pr.b;
        } else {
            in = ux * ux + uy * uy <= pr.a * pr.a;
        }
        if (in) ray_consider(pr.cz + pr.c, ray_z, best, hit);
    }
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
    o[0] = x;
    o[1] = y;
    o[2] = hit ? best : t.miss_z;
}

}  // namespace srbd
