// tamols_kernel.hip -- TAMOLS foothold local search on CDNA4 (float64), one launch per call.
//
// Restates VisualFootholdAdaptation.compute_adaptation, strategy 'tamols'
// (quadruped_pympc/helpers/visual_foothold_adaptation.py:153-231, helpers :261-714).
// Grid (TAMOLS_BPL blocks per leg, 4 legs), TAMOLS_THREADS threads.  Every block of a leg:
//   patch  : the leg's rows x cols heightmap into LDS -- raycast from the device terrain scene
//            (terrain_ray.h, the heightmap sensor fused in; up to 8 lanes per ray, each walking a share
//            of the scene staged in LDS) or read from the caller's patches;
//   phase A: the nearest-neighbour height queries of ITS slice of the candidates (19 per candidate: the
//            candidate, 5 leg-collision samples, 4 edge samples, 9 roughness samples; block 0 also the
//            seed), up to 4 lanes per query each scanning a part of the LDS patch (strict <: the first
//            nearest point wins);
//   phase B: one lane per candidate of the slice: hard constraints and soft costs -> score;
//   phase C: strict-< argmin over the slice in candidate order -> (score, index, height) partial.
// The last block of a leg to finish (per-leg counter; partials stored write-through) merges them in block
// order (strict <, so the first minimum over all candidates wins, VFA:185-190) and writes the leg's
// foothold, box and validity as words tagged with the call's sequence number (TAMOLS_OUT_WORDS).
// Outputs go straight to host-mapped memory; the host polls the tagged words (no copy, no stream sync, no
// fence and flag behind the data).  A raycast lattice patch takes one block per leg (TamolsJob::lattice).
// float64 keeps the host oracle's decisions (reach bounds, argmin) bit-for-bit comparable.
#include "terrain_ray.h"

namespace srbd {

// Query t of a leg (0 <= t < nc * NQ: candidate t / NQ, sample t % NQ; t == nc * NQ: the seed): its
// point.  Its height is the nearest patch point's + 0.02 (strict <: the first nearest point wins),
// FastHeightMap.get_height (VFA:31-35).
__device__ __forceinline__ void tamols_query_point(const TamolsArgs& a, int leg, int t, const double* px,
                                                   const double* py, double& qx_out, double& qy_out) {
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
            // alphas[q - 1] by selects over the five (uniform, scalar-loaded) values: indexed by the lane-varying q,
            // the kernel-argument array was read with a per-lane memory load and a vmcnt(0) wait in the query phase
            double al = p.alphas[0];
#pragma unroll
            for (int i = 1; i < 5; ++i) al = q - 1 == i ? p.alphas[i] : al;
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
    qx_out = qx;
    qy_out = qy;
}

// The same query scanned over patch points [i0, i1) only: (squared distance, height) of its first nearest
// point there (strict <), for splitting one query over several lanes.
__device__ __forceinline__ void tamols_query_part(const TamolsArgs& a, int leg, int t, const double* px,
                                                  const double* py, const double* pz, int i0, int i1, double& bd,
                                                  double& bh) {
    double qx, qy;
    tamols_query_point(a, leg, t, px, py, qx, qy);
#pragma unroll 4
    for (int i = i0; i < i1; ++i) {
        const double dx = qx - px[i], dy = qy - py[i];
        const double d2 = dx * dx + dy * dy;
        if (d2 < bd) {
            bd = d2;
            bh = pz[i];
        }
    }
}

// The same query on a raycast patch (TamolsJob::lattice): the patch points are ray_xy's rows x cols lattice about
// the seed (spacing dist_x, dist_y, rotated by the yaw), so the squared distance separates in the lattice frame and
// the nearest point is the per-axis nearest row and column -- one of the two lattice lines bracketing the query's
// coordinate on each axis (clamped to the patch for a query off it; the bracket holds both lines of an exact tie).
// Only those 2 x 2 points are scanned, in index order with strict < as the whole scan does, so the first nearest
// point wins and the height is the full scan's bit for bit (the frame coordinate is computed with reciprocals: an
// error far below half a spacing moves no bracket off the nearest line).
__device__ __forceinline__ double tamols_query_lattice(const TamolsJob& j, int leg, int t, const double* px,
                                                       const double* py, const double* pz) {
    const TamolsArgs& a = j.a;
    double qx, qy;
    tamols_query_point(a, leg, t, px, py, qx, qy);
    const double ex = qx - a.seeds[3 * leg], ey = qy - a.seeds[3 * leg + 1];
    const double u = (j.yaw_c * ex + j.yaw_s * ey) * j.inv_dx + (double)(j.rows - 1) * 0.5;
    const double v = (j.yaw_c * ey - j.yaw_s * ex) * j.inv_dy + (double)(j.cols - 1) * 0.5;
    // the lower bracketing line, clamped so the pair stays on the patch; fmax / fmin return the number when the
    // other operand is NaN (a NaN query: no point is nearer, as in the scan)
    const int i0 = (int)fmin(fmax(floor(u), 0.0), (double)(j.rows > 1 ? j.rows - 2 : 0));
    const int k0 = (int)fmin(fmax(floor(v), 0.0), (double)(j.cols > 1 ? j.cols - 2 : 0));
    const int ni = j.rows > 1 ? 2 : 1, nk = j.cols > 1 ? 2 : 1;
    double bd = INFINITY, bh = 0.0;
#pragma unroll
    for (int di = 0; di < 2; ++di) {
#pragma unroll
        for (int dk = 0; dk < 2; ++dk) {
            if (di >= ni || dk >= nk) continue;
            const int idx = (i0 + di) * j.cols + k0 + dk;
            const double dx = qx - px[idx], dy = qy - py[idx];
            const double d2 = dx * dx + dy * dy;
            if (d2 < bd) {
                bd = d2;
                bh = pz[idx];
            }
        }
    }
    return bh;
}

// Score of candidate (cx, cy) with its query heights h[0..NQ) (VFA:192-222): INFINITY when a hard constraint
// fails.  In four parts, so four waves can form them at once (tamols_score_part); tamols_score is their serial
// composition, the same float64 operations in the same order.
//   part 0: the hard constraints (kinematic reach VFA:375-395, leg collision VFA:397-420): 0.0 or INFINITY
//   part 1: edge (VFA:422-466)   part 2: roughness (VFA:468-521)   part 3: deviation, nominal, tracking, stability
// and tamols_combine sums the weighted terms in the reference's order.
__device__ __forceinline__ double tamols_part_hard(const TamolsArgs& a, int leg, double cx, double cy, const double* h) {
    const srbd_tamols_params& p = a.p;
    const double hx = a.hips[3 * leg], hy = a.hips[3 * leg + 1], hz = a.hips[3 * leg + 2];
    const double cz = h[0] + 0.005;  // VFA:192
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
    for (int i = 0; i < 5; ++i) {
        const double al = p.alphas[i];
        const double zz = (1.0 - al) * hz + al * cz;
        const double hg = h[1 + i] - 0.02;
        if (zz < (hg + 0.02)) return INFINITY;
    }
    return 0.0;
}
__device__ __forceinline__ double tamols_part_edge(const TamolsArgs& a, const double* h) {
    const srbd_tamols_params& p = a.p;
    const double dl = p.gradient_delta;
    const double gx = fabs(h[6] - h[7]) / (2 * dl);
    const double gy = fabs(h[8] - h[9]) / (2 * dl);
    const double g = sqrt(gx * gx + gy * gy);
    return g <= p.slope_threshold ? 0.0 : g - p.slope_threshold;
}
// roughness: least-squares plane on the symmetric 3x3 design (closed form)
__device__ __forceinline__ double tamols_part_rough(const TamolsArgs& a, const double* h) {
    const double dl = a.p.gradient_delta;
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
    return var / 9.0;
}
// deviation (VFA:344), nominal kinematics (VFA:523-553, l_des = (0, 0, -h_des)), reference tracking (VFA:555-609),
// stability (VFA:611-714): the raw terms
__device__ __forceinline__ void tamols_part_rest(const TamolsArgs& a, int leg, double cx, double cy, const double* h,
                                                 double& dev, double& nom, double& track, double& stab) {
    const srbd_tamols_params& p = a.p;
    const double hx = a.hips[3 * leg], hy = a.hips[3 * leg + 1], hz = a.hips[3 * leg + 2];
    const double sx = a.seeds[3 * leg], sy = a.seeds[3 * leg + 1], sz = a.seeds[3 * leg + 2];
    const double cz = h[0] + 0.005;
    const double ddx = cx - sx, ddy = cy - sy, ddz = cz - sz;
    dev = ddx * ddx + ddy * ddy + ddz * ddz;
    const double nx = hx - (cx - 0.0), ny = hy - (cy - 0.0), nz2 = hz - (cz - (-p.h_des));
    nom = nx * nx + ny * ny + nz2 * nz2;
    track = 0.0;
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
    stab = 0.0;
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
}
// VFA:222: 0.0 + edge w_edge + rough w_rough + dev w_dev + nom w_nominal + track w_tracking + stab w_stability
__device__ __forceinline__ double tamols_combine(const srbd_tamols_params& p, double e, double r, double dev,
                                                 double nom, double track, double stab) {
    return 0.0 + e * p.w_edge + r * p.w_rough + dev * p.w_dev + nom * p.w_nominal + track * p.w_tracking +
           stab * p.w_stability;
}
__device__ __forceinline__ double tamols_score(const TamolsArgs& a, int leg, double cx, double cy, const double* h) {
    if (tamols_part_hard(a, leg, cx, cy, h) != 0.0) return INFINITY;
    double dev, nom, track, stab;
    tamols_part_rest(a, leg, cx, cy, h, dev, nom, track, stab);
    return tamols_combine(a.p, tamols_part_edge(a, h), tamols_part_rough(a, h), dev, nom, track, stab);
}

constexpr int TAMOLS_SLICE = TAMOLS_MAXCAND;
static_assert(TAMOLS_BPL <= 64, "the merge loads one slice partial per lane of one wave");

__device__ void tamols_leg_out(const TamolsJob& j, int leg, int bi, const double* px, const double* py, double bh,
                               double seedh, bool feed);

// StepInput's 16-byte words the feed's last leg writes (TamolsJob::Feed): the state's and the reference's feet,
// and the word holding cost_feet.
constexpr int FEED_SF = (int)(offsetof(StepInput, state) + 48) / 16;
constexpr int FEED_RF = (int)(offsetof(StepInput, ref) + 48) / 16;
constexpr int FEED_CF = (int)offsetof(StepInput, cost_feet) / 16;
static_assert((offsetof(StepInput, state) + 48) % 16 == 0 && (offsetof(StepInput, ref) + 48) % 16 == 0,
              "the feet are whole 16-byte words");
static_assert(FEED_CF != FEED_SF && FEED_CF != FEED_SF + 1 && FEED_CF != FEED_SF + 2 && FEED_CF != FEED_RF &&
                  FEED_CF != FEED_RF + 1 && FEED_CF != FEED_RF + 2,
              "cost_feet lies outside the feet words");
__device__ __forceinline__ bool feed_patch_word(int w, bool cf_known) {
    return (w >= FEED_SF && w < FEED_SF + 3) || (w >= FEED_RF && w < FEED_RF + 3) || (w == FEED_CF && !cf_known);
}


// FEED: the kernel's first argument is the MPC step's input (StepInputK), read in the kernarg segment.
template <bool FEED>
__global__ void __launch_bounds__(TAMOLS_THREADS) tamols_fused_kernel(const std::conditional_t<FEED, StepInputK, KsNone> ksi,
                                                                       const TamolsJob j) {
    __shared__ double px[TAMOLS_MAXCAND], py[TAMOLS_MAXCAND], pz[TAMOLS_MAXCAND];
    __shared__ double nn[TAMOLS_SLICE * TAMOLS_NQ + 1];
    __shared__ double sc[TAMOLS_SLICE];
    __shared__ double rbest[TAMOLS_THREADS];
    __shared__ int rhit[TAMOLS_THREADS];
    __shared__ int last;
    __shared__ int plist[TAMOLS_LDS_PRIMS];  // staged primitives that can touch this leg's patch (culled)
    __shared__ int pn;
    extern __shared__ uint4 scene[];  // the terrain's primitives (+ box yaw cos / sin) when they fit
    const TamolsArgs& a = j.a;
    const int leg = blockIdx.y, b = blockIdx.x, NB = gridDim.x, tid = threadIdx.x, T = blockDim.x;
    const int nc = a.ncand;
    // diagnostic stamps (srbd_tamols_phases): s_memrealtime (100 MHz) per block at the phase ends
#define TAM_STAMP(k)                                                                                   \
    if (j.dbg && tid == 0) {                                                                         \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                  \
        j.dbg[((size_t)leg * NB + b) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                  \
    }
    if constexpr (FEED) {  // grid row 4: the MPC step's input, less the words the last leg writes (one writer per word)
        (void)ksi;
        if (leg == 4) {
            if (b == 0 && tid < j.feed.nwords && !feed_patch_word(tid, j.feed.cf_known)) {
                const auto src = (const __attribute__((address_space(4))) uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
                uint4 v;
                v.x = src[4 * tid];
                v.y = src[4 * tid + 1];
                v.z = src[4 * tid + 2];
                v.w = src[4 * tid + 3];
                reinterpret_cast<uint4*>(j.feed.in)[tid] = v;
            }
            return;
        }
    }

    TAM_STAMP(0);

    // ---- patch (raycast, or the caller's) -> LDS; block 0 also hands the raycast patch back
    if (j.use_terrain) {
        const int np = j.t.nprims;
        // lattice mode: the primitives that can touch this leg's patch, culled straight from global memory into a
        // compact list (the query stage `nn`, free until phase A, holds it); past CP_CAP of them, every primitive
        // is walked from global memory.  Else the whole scene staged in the dynamic LDS (TAMOLS_LDS_PRIMS).
        constexpr int CP_CAP = 128;
        double* cpx = nn;
        double* cpy = nn + CP_CAP;
        double* cpa = nn + 2 * CP_CAP;   // box: half size x; cylinder: radius
        double* cpb = nn + 3 * CP_CAP;   // box: half size y
        double* cpt = nn + 4 * CP_CAP;   // top: cz + c
        double* cpc = nn + 5 * CP_CAP;   // box yaw cos / sin
        double* cps = nn + 6 * CP_CAP;
        double* cpk = nn + 7 * CP_CAP;   // 1: box, 0: cylinder
        static_assert(8 * 128 <= TAMOLS_SLICE * TAMOLS_NQ, "the compact list fits the query stage");
        const bool compact = j.lattice && np > 0;
        const bool staged = !compact && np > 0 && np <= TAMOLS_LDS_PRIMS;
        const int w = np * (int)(sizeof(srbd_terrain_prim) / 16);
        int nlist = np;
        if (compact || staged) {
            if (tid == 0) pn = 0;
            if (staged) {  // stage the scene: every ray re-reads every primitive
                const uint4* src = reinterpret_cast<const uint4*>(j.t.prims);
                const uint4* srcc = reinterpret_cast<const uint4*>(j.t.cs);
                for (int i = tid; i < w + np; i += T) scene[i] = i < w ? src[i] : srcc[i - w];
            }
            __syncthreads();
            // cull: a primitive whose bounding circle (cylinder radius a, box half-diagonal, bounded by |a| + |b|)
            // clears the patch's (centre the seed, radius the half-diagonal) by a margin holds no ray of the patch.
            // A ray's result is a maximum over primitives, so the list's order (atomic slots) does not matter.
            const double hx = 0.5 * (double)(j.rows - 1) * fabs(j.dist_x), hy = 0.5 * (double)(j.cols - 1) * fabs(j.dist_y);
            const double rp = sqrt(hx * hx + hy * hy);
            const srbd_terrain_prim* sp = staged ? reinterpret_cast<const srbd_terrain_prim*>(scene) : j.t.prims;
            for (int q = tid; q < np; q += T) {
                const srbd_terrain_prim pr = sp[q];
                const bool box = pr.type == SRBD_PRIM_BOX;
                const double r = box ? fabs(pr.a) + fabs(pr.b) : fabs(pr.a);
                const double dx = pr.cx - a.seeds[3 * leg], dy = pr.cy - a.seeds[3 * leg + 1];
                const double lim = (r + rp) * 1.000001 + 1e-9;
                // keep unless clearly outside (NaN / inf geometry is kept: the walk decides as before)
                if (!(dx * dx + dy * dy > lim * lim)) {
                    const int slot = atomicAdd(&pn, 1);
                    if (staged) {
                        plist[slot] = q;
                    } else if (slot < CP_CAP) {
                        cpx[slot] = pr.cx;
                        cpy[slot] = pr.cy;
                        cpa[slot] = pr.a;
                        cpb[slot] = pr.b;
                        cpt[slot] = pr.cz + pr.c;
                        cpc[slot] = box ? j.t.cs[2 * q] : 0.0;
                        cps[slot] = box ? j.t.cs[2 * q + 1] : 0.0;
                        cpk[slot] = box ? 1.0 : 0.0;
                    }
                }
            }
            __syncthreads();
            nlist = pn;
            TAM_STAMP(6);
        }
        const bool listed = staged || (compact && nlist <= CP_CAP);
        // G lanes per ray, each walking a contiguous share of the primitives (the ray's result is a max).
        // Lanes of one wave share the share (lane -> ray i = u mod ncp, share = u / ncp, ncp = nc rounded
        // up to the wave): the primitive loads are LDS broadcasts and the box / cylinder branch is uniform.
        const int ncp = (nc + 63) & ~63;
        int G = 8;  // the most of 8, 4, 2 that fit the block, else 1 lane per ray in chunks
        while (G > 1 && G * ncp > T) G >>= 1;
        while (G > 1 && listed && G * 4 > nlist) G >>= 1;  // a short culled list: fewer lanes per ray
        for (int u0 = 0; u0 < G * ncp; u0 += T) {
            const int u = u0 + tid, part = u / ncp, i = u - part * ncp;
            const bool on = part < G && i < nc;
            double x, y, best = -INFINITY;
            int hit = 0;
            ray_xy(a.seeds[3 * leg], a.seeds[3 * leg + 1], j.yaw_c, j.yaw_s, j.rows, j.cols, i / j.cols, i % j.cols,
                   j.dist_x, j.dist_y, x, y);
            if (on) {
                if (part == 0) ray_walk_fields(j.t, x, y, j.ray_z, best, hit);
                // two call sites, so the staged walk reads through LDS-typed pointers (ds_read, not flat)
                if (compact && listed) {  // the compact list: the same float64 tests as ray_walk_prims
                    for (int n = part * nlist / G; n < (part + 1) * nlist / G; ++n) {
                        const double ux = x - cpx[n], uy = y - cpy[n];
                        bool in;
                        if (cpk[n] != 0.0) {
                            const double cb = cpc[n], sb = cps[n];
                            const double uu = cb * ux + sb * uy, vv = cb * uy - sb * ux;
                            in = fabs(uu) <= cpa[n] && fabs(vv) <= cpb[n];
                        } else {
                            in = ux * ux + uy * uy <= cpa[n] * cpa[n];
                        }
                        if (in) ray_consider(cpt[n], j.ray_z, best, hit);
                    }
                } else if (staged)
                    ray_walk_list(reinterpret_cast<const srbd_terrain_prim*>(scene),
                                  reinterpret_cast<const double*>(scene + w), plist, part * nlist / G,
                                  (part + 1) * nlist / G, x, y, j.ray_z, best, hit);
                else
                    ray_walk_prims(j.t.prims, j.t.cs, part * np / G, (part + 1) * np / G, x, y, j.ray_z, best, hit);
            }
            rbest[tid] = best;
            rhit[tid] = hit;
            __syncthreads();
            TAM_STAMP(7);
            if (on && part == 0) {
                for (int g = 1; g < G; ++g) ray_merge(rbest[tid + g * ncp], rhit[tid + g * ncp], best, hit);
                const double z = hit ? best : j.t.miss_z;
                px[i] = x;
                py[i] = y;
                pz[i] = z;
                if (b == 0 && j.hm_out) {
                    double* o = j.hm_out + 3 * ((size_t)leg * nc + i);
                    o[0] = x;
                    o[1] = y;
                    o[2] = z;
                }
            }
            __syncthreads();
        }
    } else {
        for (int i = tid; i < nc; i += T) {
            const double* hm = j.hm + 3 * ((size_t)leg * nc + i);
            px[i] = hm[0];
            py[i] = hm[1];
            pz[i] = hm[2];
        }
    }
    __syncthreads();
    TAM_STAMP(1);

    // ---- phase A: this block's candidates [c0, c1), their queries (+ the seed on block 0)
    const int c0 = (int)((long)b * nc / NB), c1 = (int)((long)(b + 1) * nc / NB);
    const int nown = (c1 - c0) * TAMOLS_NQ, nloc = nown + (b == 0 ? 1 : 0);
    if (j.lattice) {  // a raycast lattice patch: four points per query
        // lanes enumerate (sample q, candidate) candidate-fastest, so a wave's lanes share q (its branch of
        // tamols_query_point and its alpha): uniform control flow; nn keeps the (candidate, q) layout
        const int ncb = c1 - c0;
        for (int u = tid; u < nloc; u += T) {
            const int q = u < nown ? u / ncb : 0, cl = u < nown ? u - q * ncb : 0;
            const int at = u < nown ? cl * TAMOLS_NQ + q : nloc - 1;
            nn[at] = tamols_query_lattice(j, leg, u < nown ? (c0 + cl) * TAMOLS_NQ + q : nc * TAMOLS_NQ, px, py, pz) +
                     0.02;
        }
    } else {
        // Q lanes per query (aligned groups of Q consecutive lanes), each scanning a contiguous quarter of the
        // patch; the groups' (d2, first index) minima combine lowest-part-first, so the first nearest point of
        // the whole patch wins exactly as in one serial scan
        int Q = 4;
        while (Q > 1 && Q * nloc > T) Q >>= 1;
        for (int u0 = 0; u0 < nloc * Q; u0 += T) {
            const int u = u0 + tid, t = u / Q, part = u - t * Q;
            const bool on = t < nloc;
            double bd = INFINITY, bh = 0.0;
            if (on)
                tamols_query_part(a, leg, t < nown ? c0 * TAMOLS_NQ + t : nc * TAMOLS_NQ, px, py, pz, part * nc / Q,
                                  (part + 1) * nc / Q, bd, bh);
            for (int m = 1; m < Q; m <<= 1) {  // butterfly within the group; the lower part wins ties
                const double od = __shfl_xor(bd, m, 64), oh = __shfl_xor(bh, m, 64);
                const bool lower = (part & m) != 0;  // the partner holds the lower-index points
                if (od < bd || (lower && od == bd)) {
                    bd = od;
                    bh = oh;
                }
            }
            if (on && part == 0) nn[t] = bh + 0.02;
        }
    }
    __syncthreads();
    TAM_STAMP(2);

    // ---- phase B
    const int ncb = c1 - c0, ncp = (ncb + 63) & ~63;
    if (j.lattice && 4 * ncp <= T) {
        // the four parts of every candidate at once, each on waves of its own (part = wave-uniform); the terms go to
        // query slots only their own part read (hard -> 1, edge -> 6, roughness -> 10, the rest -> 2..5; slot 0,
        // the candidate's height, stays), written after a barrier, then one lane per candidate combines them
        const int part = tid / ncp, cl = tid - part * ncp;
        const bool on = part < 4 && cl < ncb;
        double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
        if (on) {
            const double* h = nn + cl * TAMOLS_NQ;
            const double cx = px[c0 + cl], cy = py[c0 + cl];
            if (part == 0) t0 = tamols_part_hard(a, leg, cx, cy, h);
            else if (part == 1) t0 = tamols_part_edge(a, h);
            else if (part == 2) t0 = tamols_part_rough(a, h);
            else tamols_part_rest(a, leg, cx, cy, h, t0, t1, t2, t3);
        }
        __syncthreads();
        if (on) {
            double* h = nn + cl * TAMOLS_NQ;
            if (part == 0) {
                h[1] = t0;
            } else if (part == 1) {
                h[6] = t0;
            } else if (part == 2) {
                h[10] = t0;
            } else {
                h[2] = t0;
                h[3] = t1;
                h[4] = t2;
                h[5] = t3;
            }
        }
        __syncthreads();
        for (int c = c0 + tid; c < c1; c += T) {
            const double* h = nn + (c - c0) * TAMOLS_NQ;
            const double s = h[1] != 0.0 ? INFINITY : tamols_combine(a.p, h[6], h[10], h[2], h[3], h[4], h[5]);
            sc[c - c0] = s;
            if (j.scores) j.scores[(size_t)leg * nc + c] = s;
        }
    } else {
    for (int c = c0 + tid; c < c1; c += T) {
        const double s = tamols_score(a, leg, px[c], py[c], nn + (c - c0) * TAMOLS_NQ);
        sc[c - c0] = s;
        if (j.scores) j.scores[(size_t)leg * nc + c] = s;
    }
    }
    if (NB != 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's score / patch stores done
    __syncthreads();
    TAM_STAMP(3);

    // ---- phase C: the slice's strict-< argmin, then the leg's last block merges the slices in order
    if (NB == 1) {  // the leg in one block: a parallel argmin -- (score, index) of the scores < INFINITY, the lower
                    // index on equal scores, so the first minimum wins as in the sequential strict-< scan (NaN and
                    // INFINITY never do: bi stays -1)
        double bs = INFINITY;
        int bi = 0x7fffffff;
        for (int c = tid; c < nc; c += T)
            if (sc[c] < bs) {  // strided and increasing: a later equal score never replaces
                bs = sc[c];
                bi = c;
            }
        for (int m = 32; m >= 1; m >>= 1) {
            const double os = __shfl_xor(bs, m, 64);
            const int oi = __shfl_xor(bi, m, 64);
            if (os < bs || (os == bs && oi < bi)) {
                bs = os;
                bi = oi;
            }
        }
        if ((tid & 63) == 0) {
            rbest[tid >> 6] = bs;
            rhit[tid >> 6] = bi;
        }
        // this wave's host-mapped score / patch stores are done (their round trip overlapped with the argmin): the
        // leg's outputs below are stored after every wave's
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid >= 64) return;
        // the host reads the scores / patch once it holds the tagged outputs: a system-scope release orders the
        // block's (completed) host stores before them -- the stores of different addresses take different paths.
        // (System-scope stores of the scores / patch in place of the release measured far slower: one PCIe write
        // per 8-byte store, C4 step p50 44 -> 80 us.)
        if (j.scores || j.hm_out) __threadfence_system();
        TAM_STAMP(4);
        for (int w = 1; w < (T + 63) / 64; ++w)  // every lane of wave 0 folds the same values
            if (rbest[w] < bs || (rbest[w] == bs && rhit[w] < bi)) {
                bs = rbest[w];
                bi = rhit[w];
            }
        tamols_leg_out(j, leg, bs < INFINITY ? bi : -1, px, py, bs < INFINITY ? nn[bi * TAMOLS_NQ] : 0.0, nn[nloc - 1],
                       FEED);
        TAM_STAMP(5);
        return;
    }
    if (tid == 0) {
        int bi = -1;
        double bs = INFINITY;
        for (int c = c0; c < c1; ++c)
            if (sc[c - c0] < bs) {
                bs = sc[c - c0];
                bi = c;
            }
        // partials as write-through (agent-scope) stores, drained before the count: the consumer reads them
        // with agent-scope loads, so no L2 write-back / invalidate is needed (MI355X guide, valid forms)
        double* P = j.part + 4 * ((size_t)leg * NB + b);
        __hip_atomic_store(P, bs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(P + 1, (double)bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(P + 2, bi >= 0 ? nn[(bi - c0) * TAMOLS_NQ] : 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(P + 3, b == 0 ? nn[nloc - 1] : 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // seed
        if (j.scores || j.hm_out) __threadfence_system();  // this block's host-mapped scores / patch
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(j.cnt + leg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = old == (unsigned)(NB - 1);
    }
    __syncthreads();
    TAM_STAMP(4);
    if (!last || tid >= 64) return;
    // wave 0 of the leg's last block: lane q loads slice q's partial (all NB in one round trip -- the loads go past
    // the L2s, ~0.3 us each, and one lane loading them in turn took ~4 us), then every lane folds them in block
    // order through lane shuffles (strict <, the first minimum wins, as the sequential fold)
    double ps = INFINITY, pi = -1.0, ph = 0.0, pseed = 0.0;
    if (tid < NB) {
        const double* P = j.part + 4 * ((size_t)leg * NB + tid);
        ps = __hip_atomic_load(P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pi = __hip_atomic_load(P + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ph = __hip_atomic_load(P + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pseed = __hip_atomic_load(P + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    int bi = -1;
    double bs = INFINITY, bh = 0.0;
    for (int q = 0; q < NB; ++q) {
        const double s = __shfl(ps, q), i = __shfl(pi, q), h = __shfl(ph, q);
        if (s < bs) {
            bs = s;
            bi = (int)i;
            bh = h;
        }
    }
    const double seedh = __shfl(pseed, 0);
    if (tid == 0) __hip_atomic_store(j.cnt + leg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next call's
    tamols_leg_out(j, leg, bi, px, py, bh, seedh, FEED);  // wave 0, every lane the same fold
    TAM_STAMP(5);
#undef TAM_STAMP
}

// The feed's last leg (one lane): the feet words and the cost_feet word of the MPC step's StepInput.  The
// footholds are rounded to float as the host's step staging rounds them; cost_feet is fill_input's sum
// cf = cf + (e * q) * e over the twelve feet coordinates, e = state - ref, in float without contraction.
__device__ void tamols_feed_finish(const TamolsJob& j) {
    const TamolsJob::Feed& f = j.feed;
    const auto kf = (const __attribute__((address_space(4))) float*)__builtin_amdgcn_kernarg_segment_ptr();
    float st[12], rf[12];
    for (int i = 0; i < 12; ++i) {
        const double h = __hip_atomic_load(f.fh + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rf[i] = (float)h;
        st[i] = f.swing[i / 3] ? rf[i] : kf[4 * FEED_SF + i];
    }
    float cf = 0.0f;
    for (int i = 0; i < 12; ++i) {
        const float e = __fsub_rn(st[i], rf[i]);
        cf = __fadd_rn(cf, __fmul_rn(__fmul_rn(e, f.q[i]), e));
    }
    float* in = reinterpret_cast<float*>(f.in);
    for (int i = 0; i < 12; ++i) {
        in[4 * FEED_SF + i] = st[i];
        in[4 * FEED_RF + i] = rf[i];
    }
    constexpr int cfi = (int)offsetof(StepInput, cost_feet) / 4;
    for (int i = 4 * FEED_CF; i < 4 * FEED_CF + 4; ++i) in[i] = i == cfi ? cf : kf[i];
}

// The leg's outputs (wave 0, every lane holding the same bi / bh / seedh): foothold, box and validity of candidate bi
// (-1: none feasible), its query height bh, the seed height, as TAMOLS_OUT_USED tagged words (lane w stores word w,
// system scope), so the host reads them as they land; the host-mapped scores / patch were stored before (every wave
// waited for its stores before the block barrier that precedes this).
__device__ void tamols_leg_out(const TamolsJob& j, int leg, int bi, const double* px, const double* py, double bh,
                               double seedh, bool feed) {
    const TamolsArgs& a = j.a;
    const srbd_tamols_params& p = a.p;
    const int lane = (int)threadIdx.x & 63;
    double f0, f1, f2, b0, b1, b2, b3, b4, b5;
    int valid;
    if (bi >= 0) {  // VFA:193-222
        f0 = px[bi];
        f1 = py[bi];
        f2 = bh + 0.005;
        b0 = f0 - p.box_dx;
        b1 = f1 - p.box_dy;
        b2 = f2;
        b3 = f0 + p.box_dx;
        b4 = f1 + p.box_dy;
        b5 = f2;
        valid = 1;
    } else {  // VFA:223-228: no feasible candidate -> the seed at its terrain height
        f0 = a.seeds[3 * leg];
        f1 = a.seeds[3 * leg + 1];
        f2 = seedh;
        b0 = b1 = b2 = b3 = b4 = b5 = NAN;
        valid = 0;
    }
    const int d = lane >> 1;
    const double v = d == 0 ? f0 : d == 1 ? f1 : d == 2 ? f2 : d == 3 ? b0 : d == 4 ? b1 : d == 5 ? b2
                   : d == 6 ? b3 : d == 7 ? b4 : d == 8 ? b5 : seedh;
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const uint32_t half = lane == 20 ? (uint32_t)valid : (lane & 1) ? (uint32_t)(bits >> 32) : (uint32_t)bits;
    if (lane < TAMOLS_OUT_USED)
        __hip_atomic_store(j.outt + (size_t)TAMOLS_OUT_WORDS * leg + lane, ((uint64_t)j.seq << 32) | half,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!feed || lane != 0) return;
    const double f[3] = {f0, f1, f2};
    if (j.feed.cf_known) {  // this leg's feet of the step input (the words' other floats are other legs')
        const auto kf = (const __attribute__((address_space(4))) float*)__builtin_amdgcn_kernarg_segment_ptr();
        float* in = reinterpret_cast<float*>(j.feed.in);
        for (int i = 0; i < 3; ++i) {
            const float r = (float)f[i];
            in[4 * FEED_RF + 3 * leg + i] = r;
            in[4 * FEED_SF + 3 * leg + i] = j.feed.swing[leg] ? r : kf[4 * FEED_SF + 3 * leg + i];
        }
    } else {  // the foothold write-through into the feed's scratch; the last leg to arrive writes the feet
        for (int i = 0; i < 3; ++i)
            __hip_atomic_store(j.feed.fh + 3 * leg + i, f[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__hip_atomic_fetch_add(j.feed.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3u) {
            __hip_atomic_store(j.feed.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next call
            tamols_feed_finish(j);
        }
    }
}

// Once per TAMOLS context (srbd_tamols_create, on its device): the staged scene needs up to
// TAMOLS_LDS_PRIMS x 80 B = 80 KB of dynamic LDS on top of ~23 KB static, above the default dynamic-LDS
// limit a launch gets without the attribute (round-2 advisor finding; gfx950 has 160 KB per CU).
int tamols_prepare() {
    const int lds = (int)((sizeof(srbd_terrain_prim) + 2 * sizeof(double)) * TAMOLS_LDS_PRIMS);
    const hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(&tamols_fused_kernel<false>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    const hipError_t e1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&tamols_fused_kernel<true>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return e0 == hipSuccess && e1 == hipSuccess ? 0 : -1;
}

// ksi != NULL: the feed (TamolsJob::Feed) -- the MPC step's input by value, the kernel's first argument.
void launch_tamols_fused(const TamolsJob& j, hipStream_t s, const StepInputK* ksi) {
    // a raycast lattice patch: one block per leg (four points per query, no cross-block merge)
    const int nb = j.lattice ? 1 : (j.a.ncand < TAMOLS_BPL ? j.a.ncand : TAMOLS_BPL);
    const int np = j.use_terrain ? j.t.nprims : 0;
    // the staged scene's dynamic LDS (not in lattice mode: its culled list lives in the static query stage)
    const size_t smem = (!j.lattice && np > 0 && np <= TAMOLS_LDS_PRIMS) ? (sizeof(srbd_terrain_prim) + 2 * sizeof(double)) * np : 0;
    if (ksi && j.feed.in)  // a fifth grid row copies the step input (off the legs' critical path)
        hipLaunchKernelGGL(tamols_fused_kernel<true>, dim3(nb, 5), dim3(TAMOLS_THREADS), smem, s, *ksi, j);
    else
        hipLaunchKernelGGL(tamols_fused_kernel<false>, dim3(nb, 4), dim3(TAMOLS_THREADS), smem, s, KsNone{0}, j);
}

}  // namespace srbd
