// tamols_kernel.hip -- TAMOLS foothold local search on CDNA4 (float64).
//
// Restates VisualFootholdAdaptation.compute_adaptation, strategy 'tamols'
// (quadruped_pympc/helpers/visual_foothold_adaptation.py:153-231, helpers :261-714).
// The leg's heightmap patch (rows x cols points) is staged in LDS.
//   phase A (tamols_nn_kernel, 7 blocks per leg): every nearest-neighbour height query of every
//            candidate (19 per candidate: the candidate, 5 leg-collision samples, 4 edge samples,
//            9 roughness samples) plus the seed, one lane per query, brute force over the LDS
//            patch (strict <: first nearest point wins)
// and then one workgroup per leg (tamols_kernel):
//   phase B: one lane per candidate evaluates the hard constraints and the soft costs
//   phase C: one lane takes the strict-< argmin in candidate order (first minimum wins)
// float64 keeps the host oracle's decisions (reach bounds, argmin) bit-for-bit comparable.
#include "srbd_launch.h"

namespace srbd {

// Query t of a leg (0 <= t < nc * NQ: candidate t / NQ, sample t % NQ; t == nc * NQ: the seed) and its
// nearest-neighbour height over the patch (strict <: the first nearest point wins), FastHeightMap.get_height
// (VFA:31-35).  Shared by the phase-A kernel and nothing else, so every query is computed one way.
__device__ __forceinline__ double tamols_query(const TamolsArgs& a, int leg, int t, const double* px, const double* py,
                                               const double* pz) {
    const int nc = a.ncand, nq = nc * TAMOLS_NQ + 1;
    const srbd_tamols_params& p = a.p;
    const double dl = p.gradient_delta;
    const double hx = a.hips[3 * leg], hy = a.hips[3 * leg + 1];
    const double sx = a.seeds[3 * leg], sy = a.seeds[3 * leg + 1];
    double qx, qy;
    if (t == nq - 1) {
        qx = sx;
        qy = sy;
    } else {
        const int c = t / TAMOLS_NQ, q = t % TAMOLS_NQ;
        const double cx = px[c], cy = py[c];
        if (q == 0) {
            qx = cx;
            qy = cy;
        } else if (q <= 5) {  // VFA:406 p_leg = (1 - alpha) * hip + alpha * candidate
            const double al = p.alphas[q - 1];
            qx = (1.0 - al) * hx + al * cx;
            qy = (1.0 - al) * hy + al * cy;
        } else if (q <= 9) {  // VFA:443 offsets (+d,0), (-d,0), (0,+d), (0,-d)
            const int o = q - 6;
            qx = o == 0 ? cx + dl : (o == 1 ? cx + (-dl) : cx + 0.0);
            qy = o == 2 ? cy + dl : (o == 3 ? cy + (-dl) : cy + 0.0);
        } else {  // VFA:489-493 3x3 grid, i outer, j inner
            const int g = q - 10, i = g / 3 - 1, j = g % 3 - 1;
            qx = cx + (double)i * dl;
            qy = cy + (double)j * dl;
        }
    }
    double bd = INFINITY, bh = 0.0;
    for (int i = 0; i < nc; ++i) {
        const double dx = qx - px[i], dy = qy - py[i];
        const double d2 = dx * dx + dy * dy;
        if (d2 < bd) {
            bd = d2;
            bh = pz[i];
        }
    }
    return bh + 0.02;
}

// Phase A over the whole chip: block (b, leg) answers queries b*256 .. of its leg (one lane each)
// into nn_g[leg][t].  One block per leg did 1 730 queries x 91 points in 22 us; spread over
// ceil(1730 / 256) = 7 blocks per leg each lane answers one.
__global__ void __launch_bounds__(256) tamols_nn_kernel(const TamolsArgs a, const double* __restrict__ hm,
                                                        double* __restrict__ nn_g) {
    __shared__ double pxs[TAMOLS_MAXCAND], pys[TAMOLS_MAXCAND], pzs[TAMOLS_MAXCAND];
    const int leg = blockIdx.y, nc = a.ncand, nq = nc * TAMOLS_NQ + 1;
    const double* H = hm + (size_t)leg * nc * 3;
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        pxs[i] = H[3 * i];
        pys[i] = H[3 * i + 1];
        pzs[i] = H[3 * i + 2];
    }
    __syncthreads();
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nq) nn_g[(size_t)leg * nq + t] = tamols_query(a, leg, t, pxs, pys, pzs);
}

__global__ void __launch_bounds__(1024) tamols_kernel(const TamolsArgs a, const double* __restrict__ hm,
                                                      const double* __restrict__ nn_g, double* __restrict__ scores,
                                                      double* __restrict__ footholds, double* __restrict__ boxes,
                                                      int* __restrict__ valid, double* __restrict__ seedh) {
    extern __shared__ double sm[];
    const int leg = blockIdx.x, tid = threadIdx.x, T = blockDim.x, nc = a.ncand;
    double* px = sm;
    double* py = px + nc;
    double* pz = py + nc;
    double* nn = pz + nc;               // nc * NQ + 1
    double* sc = nn + nc * TAMOLS_NQ + 1;  // nc
    const double* H = hm + (size_t)leg * nc * 3;
    for (int i = tid; i < nc; i += T) {
        px[i] = H[3 * i];
        py[i] = H[3 * i + 1];
        pz[i] = H[3 * i + 2];
    }
    const srbd_tamols_params& p = a.p;
    const double dl = p.gradient_delta;
    const double hx = a.hips[3 * leg], hy = a.hips[3 * leg + 1], hz = a.hips[3 * leg + 2];
    const double sx = a.seeds[3 * leg], sy = a.seeds[3 * leg + 1], sz = a.seeds[3 * leg + 2];

    // ---- phase A (tamols_nn_kernel): the leg's query heights -> LDS
    const int nq = nc * TAMOLS_NQ + 1;
    for (int t = tid; t < nq; t += T) nn[t] = nn_g[(size_t)leg * nq + t];
    __syncthreads();

    // ---- phase B
    for (int c = tid; c < nc; c += T) {
        const double* h = nn + c * TAMOLS_NQ;
        const double cx = px[c], cy = py[c], cz = h[0] + 0.005;  // VFA:192
        double s = INFINITY;
        bool ok = true;
        // kinematic feasibility (VFA:375-395)
        {
            const double dx = cx - hx, dy = cy - hy, dz = cz - hz;
            const double d = sqrt(dx * dx + dy * dy + dz * dz);
            if (!(p.l_min <= d && d <= p.l_max)) ok = false;
            if (ok && a.has_vel) {
                const double lx = hx + a.vel[0] * p.stance_duration, ly = hy + a.vel[1] * p.stance_duration,
                             lz = hz + a.vel[2] * p.stance_duration;
                const double ex = cx - lx, ey = cy - ly, ez = cz - lz;
                const double d2 = sqrt(ex * ex + ey * ey + ez * ez);
                if (!(p.l_min <= d2 && d2 <= p.l_max)) ok = false;
            }
        }
        // leg collision (VFA:397-420)
        if (ok) {
            for (int i = 0; i < 5; ++i) {
                const double al = p.alphas[i];
                const double zz = (1.0 - al) * hz + al * cz;
                const double hg = h[1 + i] - 0.02;
                if (zz < (hg + 0.02)) {
                    ok = false;
                    break;
                }
            }
        }
        if (ok) {
            // edge (VFA:422-466)
            const double gx = fabs(h[6] - h[7]) / (2 * dl);
            const double gy = fabs(h[8] - h[9]) / (2 * dl);
            const double g = sqrt(gx * gx + gy * gy);
            const double edge = g <= p.slope_threshold ? 0.0 : g - p.slope_threshold;
            // roughness (VFA:468-521): least-squares plane on the symmetric 3x3 design (closed form)
            double xs[9], ys[9], sxh = 0, syh = 0, sxx = 0, syy = 0, sh = 0;
            for (int g2 = 0; g2 < 9; ++g2) {
                xs[g2] = (double)(g2 / 3 - 1) * dl;
                ys[g2] = (double)(g2 % 3 - 1) * dl;
                sxh += xs[g2] * h[10 + g2];
                syh += ys[g2] * h[10 + g2];
                sxx += xs[g2] * xs[g2];
                syy += ys[g2] * ys[g2];
                sh += h[10 + g2];
            }
            const double pa = sxh / sxx, pb = syh / syy, pc = sh / 9.0;
            double r[9], mr = 0;
            for (int g2 = 0; g2 < 9; ++g2) {
                r[g2] = h[10 + g2] - ((xs[g2] * pa + ys[g2] * pb) + 1.0 * pc);
                mr += r[g2];
            }
            mr = mr / 9.0;
            double var = 0;
            for (int g2 = 0; g2 < 9; ++g2) var += (r[g2] - mr) * (r[g2] - mr);
            const double rough = var / 9.0;
            // deviation (VFA:344)
            const double ddx = cx - sx, ddy = cy - sy, ddz = cz - sz;
            const double dev = ddx * ddx + ddy * ddy + ddz * ddz;
            // nominal kinematics (VFA:523-553), l_des = (0, 0, -h_des)
            const double nx = hx - (cx - 0.0), ny = hy - (cy - 0.0), nz2 = hz - (cz - (-p.h_des));
            const double nom = nx * nx + ny * ny + nz2 * nz2;
            // reference tracking (VFA:555-609)
            double track = 0.0;
            if (!a.has_vel) {
                const double dx = cx - sx;
                track = dx < 0 ? dx * dx : 0.0;
            } else {
                const double vx = a.vel[0], vy = a.vel[1];
                if (!(sqrt(vx * vx + vy * vy) < 0.01)) {
                    const double dx = cx - sx;
                    if ((vx > 0 && dx < 0) || (vx < 0 && dx > 0)) track = dx * dx;
                }
            }
            // stability (VFA:611-714): distance of the predicted CoM to the diagonal support segment
            double stab = 0.0;
            if (a.has_base && a.has_feet && a.contact[leg] != 1) {
                const int dg = 3 - leg;  // FL<->RR, FR<->RL
                const double vx = a.has_vel ? a.vel[0] : 0.0, vy = a.has_vel ? a.vel[1] : 0.0;
                const double comx = a.base[0] + vx * p.swing_time, comy = a.base[1] + vy * p.swing_time;
                const double vvx = a.feet[3 * dg] - cx, vvy = a.feet[3 * dg + 1] - cy;
                const double wx = comx - cx, wy = comy - cy;
                const double vv = vvx * vvx + vvy * vvy;
                double d;
                if (vv < 1e-8) {
                    d = sqrt(wx * wx + wy * wy);
                } else {
                    double tt = (wx * vvx + wy * vvy) / vv;
                    tt = tt < 0.0 ? 0.0 : (tt > 1.0 ? 1.0 : tt);
                    const double clx = cx + tt * vvx, cly = cy + tt * vvy;
                    const double ex = comx - clx, ey = comy - cly;
                    d = sqrt(ex * ex + ey * ey);
                }
                if (d > p.stability_margin) stab = (d - p.stability_margin) * (d - p.stability_margin);
            }
            s = 0.0 + edge * p.w_edge + rough * p.w_rough + dev * p.w_dev + nom * p.w_nominal + track * p.w_tracking +
                stab * p.w_stability;
        }
        sc[c] = s;
        if (scores) scores[(size_t)leg * nc + c] = s;
    }
    __syncthreads();

    // ---- phase C (VFA:185-228)
    if (tid == 0) {
        int bi = -1;
        double bs = INFINITY;
        for (int c = 0; c < nc; ++c) {
            if (sc[c] < bs) {
                bs = sc[c];
                bi = c;
            }
        }
        double* F = footholds + 3 * leg;
        double* B = boxes + 6 * leg;
        if (bi >= 0) {
            const double cx = px[bi], cy = py[bi], cz = nn[bi * TAMOLS_NQ] + 0.005;
            F[0] = cx;
            F[1] = cy;
            F[2] = cz;
            B[0] = cx - p.box_dx;
            B[1] = cy - p.box_dy;
            B[2] = cz;
            B[3] = cx + p.box_dx;
            B[4] = cy + p.box_dy;
            B[5] = cz;
            valid[leg] = 1;
        } else {
            F[0] = sx;
            F[1] = sy;
            F[2] = nn[nq - 1];
            for (int i = 0; i < 6; ++i) B[i] = NAN;
            valid[leg] = 0;
        }
        if (seedh) seedh[leg] = nn[nq - 1];
    }
}

size_t tamols_smem_bytes(int ncand) { return sizeof(double) * ((size_t)ncand * (4 + TAMOLS_NQ) + 1); }

void launch_tamols(const TamolsArgs& a, const double* hm, double* nn, double* scores, double* footholds,
                   double* boxes, int* valid, double* seedh, hipStream_t s) {
    const int nq = a.ncand * TAMOLS_NQ + 1;
    hipLaunchKernelGGL(tamols_nn_kernel, dim3((nq + 255) / 256, 4), dim3(256), 0, s, a, hm, nn);
    hipLaunchKernelGGL(tamols_kernel, dim3(4), dim3(1024), tamols_smem_bytes(a.ncand), s, a, hm, nn, scores,
                       footholds, boxes, valid, seedh);
}

}  // namespace srbd
