// tamols_kernel.hip -- TAMOLS foothold local search on CDNA4 (float64), one launch per call.
//
// Restates VisualFootholdAdaptation.compute_adaptation, strategy 'tamols'
// (quadruped_pympc/helpers/visual_foothold_adaptation.py:153-231, helpers :261-714).
// Grid (TAMOLS_BPL blocks per leg, 4 legs), 256 threads.  Every block of a leg:
//   patch  : the leg's rows x cols heightmap into LDS -- raycast from the device terrain scene
//            (terrain_ray.h, the heightmap sensor fused in) or read from the caller's patches;
//   phase A: the nearest-neighbour height queries of ITS slice of the candidates (19 per candidate: the
//            candidate, 5 leg-collision samples, 4 edge samples, 9 roughness samples; block 0 also the
//            seed), one lane per query, brute force over the LDS patch (strict <: first nearest wins);
//   phase B: one lane per candidate of the slice: hard constraints and soft costs -> score;
//   phase C: strict-< argmin over the slice in candidate order -> (score, index, height) partial.
// The last block of a leg to finish (agent-scope acq_rel counter) merges the leg's partials in block
// order (strict <, so the first minimum over all candidates wins, VFA:185-190) and writes the leg's
// foothold, box and validity; the last leg to finish publishes the call's sequence number to the host.
// Outputs go straight to host-mapped memory; the host spins on the flag (no copy, no stream sync).
// float64 keeps the host oracle's decisions (reach bounds, argmin) bit-for-bit comparable.
#include "terrain_ray.h"

namespace srbd {

// Query t of a leg (0 <= t < nc * NQ: candidate t / NQ, sample t % NQ; t == nc * NQ: the seed) and its
// nearest-neighbour height over the patch (strict <: the first nearest point wins), FastHeightMap.get_height
// (VFA:31-35).
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

// Score of candidate (cx, cy) with its query heights h[0..NQ) (VFA:192-222): INFINITY when a hard
// constraint fails.
__device__ __forceinline__ double tamols_score(const TamolsArgs& a, int leg, double cx, double cy,
                                               const double* h) {
    const srbd_tamols_params& p = a.p;
    const double dl = p.gradient_delta;
    const double hx = a.hips[3 * leg], hy = a.hips[3 * leg + 1], hz = a.hips[3 * leg + 2];
    const double sx = a.seeds[3 * leg], sy = a.seeds[3 * leg + 1], sz = a.seeds[3 * leg + 2];
    const double cz = h[0] + 0.005;  // VFA:192
    // kinematic feasibility (VFA:375-395)
    {
        const double dx = cx - hx, dy = cy - hy, dz = cz - hz;
        const double d = sqrt(dx * dx + dy * dy + dz * dz);
        if (!(p.l_min <= d && d <= p.l_max)) return INFINITY;
        if (a.has_vel) {
            const double lx = hx + a.vel[0] * p.stance_duration, ly = hy + a.vel[1] * p.stance_duration,
                         lz = hz + a.vel[2] * p.stance_duration;
            const double ex = cx - lx, ey = cy - ly, ez = cz - lz;
            const double d2 = sqrt(ex * ex + ey * ey + ez * ez);
            if (!(p.l_min <= d2 && d2 <= p.l_max)) return INFINITY;
        }
    }
    // leg collision (VFA:397-420)
    for (int i = 0; i < 5; ++i) {
        const double al = p.alphas[i];
        const double zz = (1.0 - al) * hz + al * cz;
        const double hg = h[1 + i] - 0.02;
        if (zz < (hg + 0.02)) return INFINITY;
    }
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
    return 0.0 + edge * p.w_edge + rough * p.w_rough + dev * p.w_dev + nom * p.w_nominal + track * p.w_tracking +
           stab * p.w_stability;
}

constexpr int TAMOLS_SLICE = (TAMOLS_MAXCAND + TAMOLS_BPL - 1) / TAMOLS_BPL;  // candidates per block, max

__global__ void __launch_bounds__(256) tamols_fused_kernel(const TamolsJob j) {
    __shared__ double px[TAMOLS_MAXCAND], py[TAMOLS_MAXCAND], pz[TAMOLS_MAXCAND];
    __shared__ double nn[TAMOLS_SLICE * TAMOLS_NQ + 1];
    __shared__ double sc[TAMOLS_SLICE];
    __shared__ int last;
    const TamolsArgs& a = j.a;
    const int leg = blockIdx.y, b = blockIdx.x, NB = gridDim.x, tid = threadIdx.x, T = blockDim.x;
    const int nc = a.ncand;

    // ---- patch (raycast, or the caller's) -> LDS; block 0 also hands the raycast patch back
    for (int i = tid; i < nc; i += T) {
        double o[3];
        if (j.use_terrain) {
            terrain_ray_point(j.t, a.seeds[3 * leg], a.seeds[3 * leg + 1], j.yaw_c, j.yaw_s, j.rows, j.cols,
                              i / j.cols, i % j.cols, j.dist_x, j.dist_y, j.ray_z, o);
            if (b == 0 && j.hm_out) {
                double* w = j.hm_out + 3 * ((size_t)leg * nc + i);
                w[0] = o[0];
                w[1] = o[1];
                w[2] = o[2];
            }
        } else {
            const double* hm = j.hm + 3 * ((size_t)leg * nc + i);
            o[0] = hm[0];
            o[1] = hm[1];
            o[2] = hm[2];
        }
        px[i] = o[0];
        py[i] = o[1];
        pz[i] = o[2];
    }
    __syncthreads();

    // ---- phase A: this block's candidates [c0, c1), their queries (+ the seed on block 0)
    const int c0 = (int)((long)b * nc / NB), c1 = (int)((long)(b + 1) * nc / NB);
    const int nown = (c1 - c0) * TAMOLS_NQ, nloc = nown + (b == 0 ? 1 : 0);
    for (int t = tid; t < nloc; t += T)
        nn[t] = tamols_query(a, leg, t < nown ? c0 * TAMOLS_NQ + t : nc * TAMOLS_NQ, px, py, pz);
    __syncthreads();

    // ---- phase B
    for (int c = c0 + tid; c < c1; c += T) {
        const double s = tamols_score(a, leg, px[c], py[c], nn + (c - c0) * TAMOLS_NQ);
        sc[c - c0] = s;
        if (j.scores) j.scores[(size_t)leg * nc + c] = s;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's score / patch stores issued and done
    __syncthreads();

    // ---- phase C: the slice's strict-< argmin, then the leg's last block merges the slices in order
    if (tid == 0) {
        int bi = -1;
        double bs = INFINITY;
        for (int c = c0; c < c1; ++c)
            if (sc[c - c0] < bs) {
                bs = sc[c - c0];
                bi = c;
            }
        double* P = j.part + 4 * ((size_t)leg * NB + b);
        P[0] = bs;
        P[1] = (double)bi;
        P[2] = bi >= 0 ? nn[(bi - c0) * TAMOLS_NQ] : 0.0;
        P[3] = b == 0 ? nn[nloc - 1] : 0.0;  // the seed's height
        __threadfence_system();               // partials (device) and scores / patch (host) before the count
        const unsigned old = __hip_atomic_fetch_add(j.cnt + leg, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last = old == (unsigned)(NB - 1);
    }
    __syncthreads();
    if (!last || tid != 0) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    int bi = -1;
    double bs = INFINITY, bh = 0.0;
    for (int q = 0; q < NB; ++q) {
        const double* P = j.part + 4 * ((size_t)leg * NB + q);
        const double s = __hip_atomic_load(P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (s < bs) {
            bs = s;
            bi = (int)__hip_atomic_load(P + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bh = __hip_atomic_load(P + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const double seedh = __hip_atomic_load(j.part + 4 * ((size_t)leg * NB) + 3, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const srbd_tamols_params& p = a.p;
    double* F = j.out + 3 * leg;  // [fh 12 | box 24 | seedh 4 | valid 4 x int32]
    double* B = j.out + 12 + 6 * leg;
    int* valid = reinterpret_cast<int*>(j.out + 40);
    if (bi >= 0) {  // VFA:193-222
        const double cx = px[bi], cy = py[bi], cz = bh + 0.005;
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
    } else {  // VFA:223-228: no feasible candidate -> the seed at its terrain height
        F[0] = a.seeds[3 * leg];
        F[1] = a.seeds[3 * leg + 1];
        F[2] = seedh;
        for (int i = 0; i < 6; ++i) B[i] = NAN;
        valid[leg] = 0;
    }
    j.out[36 + leg] = seedh;
    __hip_atomic_store(j.cnt + leg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next call
    __threadfence_system();
    const unsigned done = __hip_atomic_fetch_add(j.cnt + 4, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (done == 3u) {  // the last leg: every leg's outputs are visible system-wide -> publish
        __hip_atomic_store(j.cnt + 4, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence_system();
        __hip_atomic_store(j.flag, j.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

void launch_tamols_fused(const TamolsJob& j, hipStream_t s) {
    const int nb = j.a.ncand < TAMOLS_BPL ? j.a.ncand : TAMOLS_BPL;
    hipLaunchKernelGGL(tamols_fused_kernel, dim3(nb, 4), dim3(256), 0, s, j);
}

}  // namespace srbd
