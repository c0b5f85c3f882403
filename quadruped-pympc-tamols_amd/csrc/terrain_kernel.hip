// terrain_kernel.hip -- heightmap patches by vertical ray casts against a device-resident scene
// (C-ABI in include/srbd_mpc.h, srbd_terrain_*).
//
// Replaces gym_quadruped's HeightMap.update_height_map, which casts one MuJoCo ray per patch point
// on the CPU (quadruped_pympc/interfaces/wb_interface.py:233-234; HeightMap(13, 7, 0.04, 0.04) at
// simulation/simulation.py:490-511).  One lane per ray; every lane of a launch walks the same
// primitive list, so the primitive loads are wave-uniform (scalar-cache broadcasts).  float64 and
// -ffp-contract=off: the points are bit-identical to oracle/terrain_oracle.py.
#include <math.h>

#include <string>

#include "terrain_ray.h"

namespace srbd {

__global__ void __launch_bounds__(256) terrain_patch_kernel(const TerrainDev t, const PatchJob j) {
    const int per = j.rows * j.cols;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= j.npatch * per) return;
    const int p = g / per, r = g % per, i = r / j.cols, k = r % j.cols;
    terrain_ray_point(t, j.centers[3 * p], j.centers[3 * p + 1], j.cs_yaw[2 * p], j.cs_yaw[2 * p + 1], j.rows, j.cols,
                      i, k, j.dist_x, j.dist_y, j.ray_z, j.out + 3 * (size_t)g);
}

void launch_terrain_patches(const TerrainDev& t, const PatchJob& j, hipStream_t s) {
    const int n = j.npatch * j.rows * j.cols;
    hipLaunchKernelGGL(terrain_patch_kernel, dim3((n + 255) / 256), dim3(256), 0, s, t, j);
}

}  // namespace srbd

using namespace srbd;

static std::string g_terrain_error;

static int terrain_fail(srbd_terrain* t, int code, const std::string& m) {
    (t ? t->err : g_terrain_error) = m;
    return code;
}

#define TER_TRY(t, expr)                                                                       \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) return terrain_fail((t), SRBD_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

extern "C" void srbd_terrain_destroy(srbd_terrain* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    (void)hipFree(t->d_prims);
    (void)hipFree(t->d_cs);
    (void)hipFree(t->d_hf);
    (void)hipFree(t->d_job);
    (void)hipFree(t->d_out);
    if (t->h_job) (void)hipHostFree(t->h_job);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

extern "C" const char* srbd_terrain_last_error(const srbd_terrain* t) {
    return t ? t->err.c_str() : g_terrain_error.c_str();
}

extern "C" int srbd_terrain_create(int32_t device_id, const srbd_terrain_prim* prims, int32_t nprims, int32_t has_ground,
                                   double ground_z, const double* hfield, int32_t hf_nx, int32_t hf_ny, double hf_x0,
                                   double hf_y0, double hf_dx, double hf_dy, double miss_z, srbd_terrain** out) {
    if (!out || nprims < 0 || (nprims > 0 && !prims)) return terrain_fail(nullptr, SRBD_E_INVALID, "bad arguments");
    *out = nullptr;
    if (hfield && (hf_nx < 2 || hf_ny < 2 || !(hf_dx > 0.0) || !(hf_dy > 0.0)))
        return terrain_fail(nullptr, SRBD_E_INVALID, "height field needs >= 2 x 2 points and positive spacing");
    for (int q = 0; q < nprims; ++q)
        if (prims[q].type != SRBD_PRIM_BOX && prims[q].type != SRBD_PRIM_CYLINDER)
            return terrain_fail(nullptr, SRBD_E_INVALID, "unknown primitive type");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || device_id < 0 || device_id >= ndev)
        return terrain_fail(nullptr, SRBD_E_NODEVICE, "no HIP device visible (this library has no CPU fallback)");
    srbd_terrain* t = new srbd_terrain();
    t->device = device_id;
    t->dev.nprims = nprims;
    t->dev.has_ground = has_ground != 0;
    t->dev.ground_z = ground_z;
    t->dev.miss_z = miss_z;
    t->dev.hf_nx = hfield ? hf_nx : 0;
    t->dev.hf_ny = hfield ? hf_ny : 0;
    t->dev.hf_x0 = hf_x0;
    t->dev.hf_y0 = hf_y0;
    t->dev.hf_dx = hf_dx;
    t->dev.hf_dy = hf_dy;
    {
        const auto ok = [](double v) { return std::isfinite(v) && fabs(v) < 1e30; };
        bool b = !has_ground || ok(ground_z);  // miss_z: checked per call (a ray below the ground misses)
        for (int q = 0; b && q < nprims; ++q) {
            const srbd_terrain_prim& p = prims[q];
            b = ok(p.cx) && ok(p.cy) && ok(p.cz) && ok(p.a) && ok(p.b) && ok(p.c) && ok(p.yaw);
        }
        if (hfield) {
            b = b && ok(hf_x0) && ok(hf_y0) && ok(hf_dx) && ok(hf_dy);
            for (size_t i = 0; b && i < (size_t)hf_nx * hf_ny; ++i) b = ok(hfield[i]);
        }
        t->bounded = b;
    }
    auto bad = [&](hipError_t e) {
        const std::string m = std::string("terrain upload: ") + hipGetErrorString(e);
        srbd_terrain_destroy(t);
        return terrain_fail(nullptr, SRBD_E_HIP, m);
    };
    hipError_t e;
    if ((e = hipSetDevice(device_id)) != hipSuccess) return bad(e);
    if ((e = hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking)) != hipSuccess) return bad(e);
    if (nprims > 0) {
        std::vector<double> cs(2 * (size_t)nprims);
        for (int q = 0; q < nprims; ++q) {
            cs[2 * q] = cos(prims[q].yaw);
            cs[2 * q + 1] = sin(prims[q].yaw);
        }
        if ((e = hipMalloc((void**)&t->d_prims, sizeof(srbd_terrain_prim) * nprims)) != hipSuccess) return bad(e);
        if ((e = hipMalloc((void**)&t->d_cs, sizeof(double) * 2 * nprims)) != hipSuccess) return bad(e);
        if ((e = hipMemcpy(t->d_prims, prims, sizeof(srbd_terrain_prim) * nprims, hipMemcpyHostToDevice)) != hipSuccess)
            return bad(e);
        if ((e = hipMemcpy(t->d_cs, cs.data(), sizeof(double) * 2 * nprims, hipMemcpyHostToDevice)) != hipSuccess)
            return bad(e);
    }
    if (hfield) {
        const size_t b = sizeof(double) * (size_t)hf_nx * hf_ny;
        if ((e = hipMalloc((void**)&t->d_hf, b)) != hipSuccess) return bad(e);
        if ((e = hipMemcpy(t->d_hf, hfield, b, hipMemcpyHostToDevice)) != hipSuccess) return bad(e);
    }
    t->dev.prims = t->d_prims;
    t->dev.cs = t->d_cs;
    t->dev.hf = t->d_hf;
    *out = t;
    return SRBD_OK;
}

// Job inputs (centres, yaw cos / sin) staged through pinned memory and one H2D copy into d_job; the
// output buffer grows on demand.  Returns the device output pointer in *d_out.
int srbd::terrain_enqueue(srbd_terrain* t, const double* centers, const double* yaws, int npatch, int rows, int cols,
                    double dist_x, double dist_y, double ray_z, hipStream_t s, double** d_out) {
    if (!t || !centers || !yaws || npatch < 1 || rows < 1 || cols < 1)
        return terrain_fail(t, SRBD_E_INVALID, "bad patch arguments");
    const size_t need_out = (size_t)npatch * rows * cols * 3, need_job = 5 * (size_t)npatch;
    if (t->cap_job < need_job) {
        TER_TRY(t, hipStreamSynchronize(s));
        (void)hipFree(t->d_job);
        if (t->h_job) (void)hipHostFree(t->h_job);
        t->d_job = t->h_job = nullptr;
        t->cap_job = 0;
        TER_TRY(t, hipMalloc((void**)&t->d_job, sizeof(double) * need_job));
        TER_TRY(t, hipHostMalloc((void**)&t->h_job, sizeof(double) * need_job, hipHostMallocDefault));
        t->cap_job = need_job;
    }
    if (t->cap_out < need_out) {
        (void)hipFree(t->d_out);
        t->d_out = nullptr;
        TER_TRY(t, hipMalloc((void**)&t->d_out, sizeof(double) * need_out));
        t->cap_out = need_out;
    }
    // the previous call's copy out of h_job has completed: every call ends with a stream synchronise
    for (int p = 0; p < npatch; ++p) {
        for (int q = 0; q < 3; ++q) t->h_job[3 * p + q] = centers[3 * p + q];
        t->h_job[3 * npatch + 2 * p] = cos(yaws[p]);
        t->h_job[3 * npatch + 2 * p + 1] = sin(yaws[p]);
    }
    TER_TRY(t, hipMemcpyAsync(t->d_job, t->h_job, sizeof(double) * need_job, hipMemcpyHostToDevice, s));
    PatchJob j;
    j.centers = t->d_job;
    j.cs_yaw = t->d_job + 3 * npatch;
    j.npatch = npatch;
    j.rows = rows;
    j.cols = cols;
    j.dist_x = dist_x;
    j.dist_y = dist_y;
    j.ray_z = ray_z;
    j.out = t->d_out;
    launch_terrain_patches(t->dev, j, s);
    TER_TRY(t, hipGetLastError());
    *d_out = t->d_out;
    return SRBD_OK;
}

extern "C" int srbd_terrain_patches(srbd_terrain* t, const double* centers, const double* yaws, int32_t npatch,
                                    int32_t rows, int32_t cols, double dist_x, double dist_y, double ray_z, double* out) {
    if (!t || !out) return terrain_fail(t, SRBD_E_INVALID, "bad arguments");
    TER_TRY(t, hipSetDevice(t->device));
    double* d_out = nullptr;
    if (int rc = terrain_enqueue(t, centers, yaws, npatch, rows, cols, dist_x, dist_y, ray_z, t->stream, &d_out))
        return rc;
    TER_TRY(t, hipMemcpyAsync(out, d_out, sizeof(double) * 3 * (size_t)npatch * rows * cols, hipMemcpyDeviceToHost,
                              t->stream));
    TER_TRY(t, hipStreamSynchronize(t->stream));
    return SRBD_OK;
}
