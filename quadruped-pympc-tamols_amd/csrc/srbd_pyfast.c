/* srbd_pyfast.c -- CPython glue of the per-MPC-step host path (module quadruped_pympc_amd._srbd_fast).
 *
 * The 100 Hz controller loop of the reference calls, per MPC step, PeriodicGaitGenerator.compute_contact_sequence
 * (periodic_gait_generator.py:93-118) and SRBDControllerInterface.compute_control (srbd_controller_interface.py:
 * 113-180).  Both run their work in libsrbd_hip.so (srbd_pgg_contact_sequence; srbd_interface_step: prepare_state,
 * with_newkey, the device step, the GRF mask).  What is left in Python is glue: gathering the state / reference
 * dicts into flat float64 rows, staging the contact sequence and the warm start, and building the returned arrays
 * -- about as long as the device step at N = 10 000 when written with NumPy calls.  This module does that glue in
 * C against the CPython / NumPy C APIs.  It computes nothing itself: it calls the library through function
 * pointers the binding hands it (bind(), addresses from _lib's CDLL), so it always calls the library instance
 * _lib loaded (the sanitizer variant included).
 *
 * interface_step() returns None without touching anything when an input is not in the form it handles (float64
 * ndarrays of three values per dict entry, a float64 / float32 (4, >= H) contact sequence): the caller then runs
 * the Python chain, which makes the same library calls.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_20_API_VERSION
#include <numpy/arrayobject.h>
#include <stdint.h>
#include <string.h>

#include "../../include/srbd_host.h"
#include "../../include/srbd_mpc.h"

typedef int (*iface_fn_t)(srbd_ctx*, srbd_interface_io*, const float*, const double*, int32_t, float*, int32_t,
                          float*, srbd_result*);
typedef int (*pgg_seq_fn_t)(srbd_pgg*, const double*, const int32_t*, int32_t, double*, int32_t);
typedef int (*foothold_fn_t)(srbd_tamols_ctx*, srbd_terrain*, const srbd_tamols_params*, srbd_ctx*, srbd_foothold_io*,
                             const float*, int32_t, float*, int32_t, uint64_t, uint64_t, srbd_result*);
typedef int (*split_fn_t)(const uint32_t*, int32_t, int32_t, uint32_t*);

static iface_fn_t g_iface;
static pgg_seq_fn_t g_pgg_seq;
static foothold_fn_t g_foothold;
static split_fn_t g_split;

static const char* const STATE_KEYS[8] = {"position", "linear_velocity", "orientation", "angular_velocity",
                                          "foot_FL",  "foot_FR",         "foot_RL",     "foot_RR"};
static const char* const REF_KEYS[8] = {"ref_position", "ref_linear_velocity", "ref_orientation",
                                        "ref_angular_velocity", "ref_foot_FL", "ref_foot_FR", "ref_foot_RL",
                                        "ref_foot_RR"};
static PyObject* k_state[8];
static PyObject* k_ref[8];
static PyObject* k_zero;  /* the int 0 (ref_foot_*[0]) */

/* bind(srbd_interface_step, srbd_pgg_contact_sequence, srbd_foothold_mpc_step, srbd_jax_split addresses) */
static PyObject* bind(PyObject* self, PyObject* args) {
    unsigned long long a, b, c, d;
    (void)self;
    if (!PyArg_ParseTuple(args, "KKKK", &a, &b, &c, &d)) return NULL;
    g_iface = (iface_fn_t)(uintptr_t)a;
    g_pgg_seq = (pgg_seq_fn_t)(uintptr_t)b;
    g_foothold = (foothold_fn_t)(uintptr_t)c;
    g_split = (split_fn_t)(uintptr_t)d;
    Py_RETURN_NONE;
}

static void* addr_of(PyObject* o) { return PyLong_AsVoidPtr(o); }

/* pgg_contact_sequence(pgg_address, dts, lens) -> (4, cols) float64 ndarray (PeriodicGaitGenerator.
 * compute_contact_sequence: dts as float64, lens cast to int32 as np.asarray(..., dtype=np.int32) does). */
static PyObject* pgg_contact_sequence(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    (void)self;
    if (nargs != 3) {
        PyErr_SetString(PyExc_TypeError, "pgg_contact_sequence(pgg, dts, lens)");
        return NULL;
    }
    if (!g_pgg_seq) {
        PyErr_SetString(PyExc_RuntimeError, "_srbd_fast: bind() first");
        return NULL;
    }
    srbd_pgg* g = (srbd_pgg*)addr_of(args[0]);
    if (!g) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "pgg_contact_sequence: null generator");
        return NULL;
    }
    PyArrayObject* d = (PyArrayObject*)PyArray_FROM_OTF(args[1], NPY_FLOAT64, NPY_ARRAY_IN_ARRAY);
    if (!d) return NULL;
    PyArrayObject* l = (PyArrayObject*)PyArray_FROM_OTF(args[2], NPY_INT32, NPY_ARRAY_IN_ARRAY | NPY_ARRAY_FORCECAST);
    if (!l) {
        Py_DECREF(d);
        return NULL;
    }
    if (PyArray_SIZE(l) < PyArray_SIZE(d) && g->gait_type != SRBD_GAIT_FULL_STANCE) {
        /* fewer lengths than dts: the library reads lengths[j] for j < n_dts, so walk the reference's index first
         * (PGG:111-115) -- it raises IndexError where it would read past the lengths */
        const int32_t* lp = (const int32_t*)PyArray_DATA(l);
        const npy_intp nl = PyArray_SIZE(l), nd = PyArray_SIZE(d);
        npy_intp j = 0;
        int past = 0;
        for (int i = 1; i < g->horizon; ++i) {
            if (j >= nl) {  /* lengths[j] read past the end */
                past = 1;
                break;
            }
            if (i >= lp[j]) ++j;
            if (j >= nd) break;  /* dts[j] past the end: the library reports it */
        }
        if (past) {
            Py_DECREF(d);
            Py_DECREF(l);
            PyErr_SetString(PyExc_IndexError, "compute_contact_sequence: contact_sequence_lenghts too short");
            return NULL;
        }
    }
    double out[8 * SRBD_MAX_HORIZON];
    const int H = g->horizon;
    const int cap = 8 * H < 8 * SRBD_MAX_HORIZON ? 8 * H : 8 * SRBD_MAX_HORIZON;
    const int cols = g_pgg_seq(g, (const double*)PyArray_DATA(d), (const int32_t*)PyArray_DATA(l),
                               (int32_t)PyArray_SIZE(d), out, cap);
    Py_DECREF(d);
    Py_DECREF(l);
    if (cols < 0) {
        PyErr_Format(PyExc_ValueError, "compute_contact_sequence failed (%d)", cols);
        return NULL;
    }
    npy_intp dims[2] = {4, cols};
    PyObject* a = PyArray_SimpleNew(2, dims, NPY_FLOAT64);
    if (!a) return NULL;
    memcpy(PyArray_DATA((PyArrayObject*)a), out, sizeof(double) * 4 * (size_t)cols);
    return a;
}

/* Three float64 values of a dict entry (a C-contiguous float64 ndarray of size 3); 0 when it is not one. */
static int get3(PyObject* dict, PyObject* key, double* dst, PyObject** item) {
    PyObject* v = PyDict_Check(dict) ? PyDict_GetItemWithError(dict, key) : NULL;  /* borrowed */
    if (!v) return 0;
    if (!PyArray_Check(v)) return 0;
    PyArrayObject* a = (PyArrayObject*)v;
    if (PyArray_TYPE(a) != NPY_FLOAT64 || PyArray_SIZE(a) != 3 || !PyArray_IS_C_CONTIGUOUS(a)) return 0;
    memcpy(dst, PyArray_DATA(a), 3 * sizeof(double));
    if (item) *item = v;
    return 1;
}

static PyObject* new_1d(int type, npy_intp n, const void* src, size_t elem) {
    PyObject* a = PyArray_SimpleNew(1, &n, type);
    if (a && src) memcpy(PyArray_DATA((PyArrayObject*)a), src, elem * (size_t)n);
    return a;
}

/* interface_step(ctx, io, state, ref, contact_sequence, best, previous_contact, master_key, calls, iterations,
 *                sigma_reset, best_buf, sigma_buf, result)
 *   ctx, io, result : addresses of the srbd_ctx, a srbd_interface_io (horizon / rng / cem set) and a srbd_result
 *   best_buf / sigma_buf : the persistent float32 (P,) staging of the warm start / CEM sigma (sigma_buf None: not CEM)
 * -> None (an input not handled here: nothing was touched), or
 *    (rc, stage, current_contact) when a call of the chain failed, or
 *    (grf (4, 3) float64, predicted_state (24,) float32, best (P,) float32, sigma (P,) float32 | None,
 *     master_key, calls, current_contact (4,) float64, (ref_foot_FL[0], ..., ref_foot_RR[0])) */
static PyObject* interface_step(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    (void)self;
    if (nargs != 14) {
        PyErr_SetString(PyExc_TypeError, "interface_step takes 14 arguments");
        return NULL;
    }
    if (!g_iface) {
        PyErr_SetString(PyExc_RuntimeError, "_srbd_fast: bind() first");
        return NULL;
    }
    srbd_ctx* ctx = (srbd_ctx*)addr_of(args[0]);
    srbd_interface_io* io = (srbd_interface_io*)addr_of(args[1]);
    srbd_result* res = (srbd_result*)addr_of(args[13]);
    if (PyErr_Occurred()) return NULL;
    PyObject *state = args[2], *ref = args[3], *cs = args[4], *best = args[5], *prev = args[6], *mk = args[7];
    PyObject *best_buf = args[11], *sigma_buf = args[12];
    const int H = io->horizon;

    /* ---- validate and gather (no side effects before every input is known to fit) */
    double st[24], rf[24];
    for (int i = 0; i < 8; ++i) {
        if (!get3(state, k_state[i], st + 3 * i, NULL) || !get3(ref, k_ref[i], rf + 3 * i, NULL)) {
            if (PyErr_Occurred()) return NULL;
            Py_RETURN_NONE;
        }
    }
    if (!PyArray_Check(cs)) Py_RETURN_NONE;
    PyArrayObject* ca = (PyArrayObject*)cs;
    const int ctype = PyArray_TYPE(ca);
    if (PyArray_NDIM(ca) != 2 || PyArray_DIM(ca, 0) != 4 || PyArray_DIM(ca, 1) < H || !PyArray_IS_C_CONTIGUOUS(ca) ||
        (ctype != NPY_FLOAT64 && ctype != NPY_FLOAT32))
        Py_RETURN_NONE;
    const int32_t stride = (int32_t)PyArray_DIM(ca, 1);
    if (!PyArray_Check(best_buf) || PyArray_TYPE((PyArrayObject*)best_buf) != NPY_FLOAT32 ||
        !PyArray_IS_C_CONTIGUOUS((PyArrayObject*)best_buf)) {
        PyErr_SetString(PyExc_TypeError, "best_buf: float32 C-contiguous");
        return NULL;
    }
    const npy_intp P = PyArray_SIZE((PyArrayObject*)best_buf);
    if (io->cem && (!PyArray_Check(sigma_buf) || PyArray_TYPE((PyArrayObject*)sigma_buf) != NPY_FLOAT32 ||
                    PyArray_SIZE((PyArrayObject*)sigma_buf) != P)) {
        PyErr_SetString(PyExc_TypeError, "sigma_buf: float32 (P,) for CEM");
        return NULL;
    }
    const int iterations = (int)PyLong_AsLong(args[9]);
    const long long calls = PyLong_AsLongLong(args[8]);
    double sigma_reset = 0.0;
    if (io->cem) sigma_reset = PyFloat_AsDouble(args[10]);
    if (PyErr_Occurred()) return NULL;
    PyArrayObject* b = (PyArrayObject*)PyArray_FROM_OTF(best, NPY_FLOAT32, NPY_ARRAY_IN_ARRAY | NPY_ARRAY_FORCECAST);
    if (!b) return NULL;
    if (PyArray_SIZE(b) != P) {
        Py_DECREF(b);
        Py_RETURN_NONE;
    }
    PyArrayObject* pv = (PyArrayObject*)PyArray_FROM_OTF(prev, NPY_FLOAT64, NPY_ARRAY_IN_ARRAY | NPY_ARRAY_FORCECAST);
    if (!pv) {
        Py_DECREF(b);
        return NULL;
    }
    const int philox = io->rng == SRBD_RNG_PHILOX;
    PyArrayObject* kk = (PyArrayObject*)PyArray_FROM_OTF(mk, philox ? NPY_UINT64 : NPY_UINT32,
                                                         NPY_ARRAY_IN_ARRAY | NPY_ARRAY_FORCECAST);
    if (!kk) {
        Py_DECREF(b);
        Py_DECREF(pv);
        return NULL;
    }
    if (PyArray_SIZE(pv) != 4 || PyArray_SIZE(kk) != 2) {  /* with_newkey / pack_key take a two-word key */
        Py_DECREF(b);
        Py_DECREF(pv);
        Py_DECREF(kk);
        Py_RETURN_NONE;
    }

    /* ---- the call */
    memcpy(io->state_in, st, sizeof(st));
    memcpy(io->ref_in, rf, sizeof(rf));
    const char* cdata = (const char*)PyArray_DATA(ca);
    for (int l = 0; l < 4; ++l)
        io->current_contact[l] = ctype == NPY_FLOAT64 ? ((const double*)cdata)[(size_t)l * stride]
                                                      : (double)((const float*)cdata)[(size_t)l * stride];
    memcpy(io->previous_contact, PyArray_DATA(pv), 4 * sizeof(double));
    Py_DECREF(pv);
    if (philox) {
        const uint64_t* k = (const uint64_t*)PyArray_DATA(kk);
        io->key[0] = k[0];
        io->key[1] = k[1];
    } else {
        const uint32_t* k = (const uint32_t*)PyArray_DATA(kk);
        io->key[0] = ((uint64_t)k[0] << 32) | k[1];
        io->key[1] = (uint64_t)calls;
    }
    Py_DECREF(kk);
    io->iterations = iterations;
    io->sigma_reset = sigma_reset;
    float* bb = (float*)PyArray_DATA((PyArrayObject*)best_buf);
    memcpy(bb, PyArray_DATA(b), sizeof(float) * (size_t)P);
    Py_DECREF(b);
    float* sg = io->cem ? (float*)PyArray_DATA((PyArrayObject*)sigma_buf) : NULL;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_iface(ctx, io, ctype == NPY_FLOAT32 ? (const float*)cdata : NULL,
                 ctype == NPY_FLOAT64 ? (const double*)cdata : NULL, stride, bb, (int32_t)(P / 4), sg, res);
    Py_END_ALLOW_THREADS
    PyObject* cur = new_1d(NPY_FLOAT64, 4, io->current_contact, sizeof(double));
    if (!cur) return NULL;
    if (rc != 0) return Py_BuildValue("(iiN)", rc, io->stage, cur);

    /* ---- outputs */
    npy_intp d43[2] = {4, 3};
    PyObject* grf = PyArray_SimpleNew(2, d43, NPY_FLOAT64);
    PyObject* pred = new_1d(NPY_FLOAT32, 24, res->predicted_state, sizeof(float));
    PyObject* nb = new_1d(NPY_FLOAT32, P, bb, sizeof(float));
    PyObject* ns = io->cem ? new_1d(NPY_FLOAT32, P, sg, sizeof(float)) : (Py_INCREF(Py_None), Py_None);
    PyObject* nk = NULL;
    if (philox) {
        const uint64_t k2[2] = {io->key[0], io->key[1]};
        nk = new_1d(NPY_UINT64, 2, k2, sizeof(uint64_t));
    } else {
        const uint32_t k2[2] = {(uint32_t)(io->key[0] >> 32), (uint32_t)io->key[0]};
        nk = new_1d(NPY_UINT32, 2, k2, sizeof(uint32_t));
    }
    PyObject* fh = PyTuple_New(4);
    if (!grf || !pred || !nb || !ns || !nk || !fh) goto fail;
    memcpy(PyArray_DATA((PyArrayObject*)grf), io->grf, sizeof(io->grf));
    for (int l = 0; l < 4; ++l) {
        /* ref_state["ref_foot_*"][0], looked up again now: the GIL was released around the call, so a reference
         * borrowed from the dict before it may no longer be alive */
        PyObject* v = PyDict_GetItemWithError(ref, k_ref[4 + l]);  /* borrowed, used at once */
        if (!v) {
            if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, k_ref[4 + l]);
            goto fail;
        }
        PyObject* f = PyObject_GetItem(v, k_zero);
        if (!f) goto fail;
        PyTuple_SET_ITEM(fh, l, f);
    }
    return Py_BuildValue("(NNNNNLNN)", grf, pred, nb, ns, nk, (long long)(philox ? 0 : (long long)io->key[1]), cur, fh);
fail:
    Py_XDECREF(grf);
    Py_XDECREF(pred);
    Py_XDECREF(nb);
    Py_XDECREF(ns);
    Py_XDECREF(nk);
    Py_XDECREF(fh);
    Py_DECREF(cur);
    return NULL;
}

static PyObject* k_legs[4];  /* "FL" .. "RR" (LegsAttr attributes) */

/* Three float64 values of an attribute / item (a C-contiguous float64 ndarray of >= 3 values). */
static int get3_arr(PyObject* v, double* dst) {
    if (!v || !PyArray_Check(v)) return 0;
    PyArrayObject* a = (PyArrayObject*)v;
    if (PyArray_TYPE(a) != NPY_FLOAT64 || PyArray_SIZE(a) < 3 || !PyArray_IS_C_CONTIGUOUS(a)) return 0;
    memcpy(dst, PyArray_DATA(a), 3 * sizeof(double));
    return 1;
}
static int get_legs(PyObject* legs, double* dst) {  /* a LegsAttr's FL FR RL RR rows -> dst[12] */
    for (int l = 0; l < 4; ++l) {
        PyObject* v = PyObject_GetAttr(legs, k_legs[l]);
        if (!v) {
            PyErr_Clear();
            return 0;
        }
        const int ok = get3_arr(v, dst + 3 * l);
        Py_DECREF(v);
        if (!ok) return 0;
    }
    return 1;
}

/* foothold_step(tamols, terrain, params, ctx, io, state, ref_base, seeds, hips, base_lin_vel, base_ori, contact_sequence,
 *               best, previous_contact, master_key, calls, best_buf, contact_buf, result, params_per_leg, rng)
 * helpers/foothold_pipeline.py TamolsMpcStep._step_fused's staging and its one srbd_foothold_mpc_step call (the
 * key split of compute_control's with_newkey included):
 * -> None (an input form not handled here: nothing touched), or
 *    (rc, stage, current_contact, master_key, calls) when a call of the chain failed, or
 *    (0, 3, current_contact, master_key, calls, GRF rows (4 x (3,) float64, masked), predicted_state (24,) float32,
 *     best (P,) float32, foothold rows (4 x (3,) float64), constraint boxes (4 x [lower, upper] | None),
 *     patches (4 x (rows, cols, 1, 3) float64), or without io->heightmaps the maps' pending (seed (3,), yaw) pairs,
 *     scores (4, rows cols) float64 | None) */
static PyObject* foothold_step(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    (void)self;
    if (nargs != 21) {
        PyErr_SetString(PyExc_TypeError, "foothold_step takes 21 arguments");
        return NULL;
    }
    if (!g_foothold || !g_split) {
        PyErr_SetString(PyExc_RuntimeError, "_srbd_fast: bind() first");
        return NULL;
    }
    srbd_tamols_ctx* tam = (srbd_tamols_ctx*)addr_of(args[0]);
    srbd_terrain* ter = (srbd_terrain*)addr_of(args[1]);
    const srbd_tamols_params* prm = (const srbd_tamols_params*)addr_of(args[2]);
    srbd_ctx* ctx = (srbd_ctx*)addr_of(args[3]);
    srbd_foothold_io* io = (srbd_foothold_io*)addr_of(args[4]);
    srbd_result* res = (srbd_result*)addr_of(args[18]);
    const int ppl = (int)PyLong_AsLong(args[19]), rng = (int)PyLong_AsLong(args[20]);
    const long long calls = PyLong_AsLongLong(args[15]);
    if (PyErr_Occurred()) return NULL;
    PyObject *state = args[5], *refb = args[6], *cs = args[11], *best = args[12], *prev = args[13], *mk = args[14];
    PyObject *best_buf = args[16], *contact_buf = args[17];

    /* ---- validate and gather */
    double st[24], rb[12], sd[12], hp[12], fv[3], yaw;
    for (int i = 0; i < 8; ++i)
        if (!get3(state, k_state[i], st + 3 * i, NULL)) goto decline;
    for (int i = 0; i < 4; ++i)
        if (!get3(refb, k_ref[i], rb + 3 * i, NULL)) goto decline;
    if (!get_legs(args[7], sd) || !get_legs(args[8], hp) || !get3_arr(args[9], fv)) goto decline;
    {
        PyObject* o = args[10];
        if (!PyArray_Check(o) || PyArray_TYPE((PyArrayObject*)o) != NPY_FLOAT64 ||
            PyArray_SIZE((PyArrayObject*)o) < 3 || !PyArray_IS_C_CONTIGUOUS((PyArrayObject*)o))
            goto decline;
        yaw = ((const double*)PyArray_DATA((PyArrayObject*)o))[2];
    }
    if (!PyArray_Check(cs)) goto decline;
    PyArrayObject* ca = (PyArrayObject*)cs;
    if (!PyArray_Check(contact_buf) || PyArray_TYPE((PyArrayObject*)contact_buf) != NPY_FLOAT32 ||
        PyArray_NDIM((PyArrayObject*)contact_buf) != 2 || !PyArray_IS_C_CONTIGUOUS((PyArrayObject*)contact_buf)) {
        PyErr_SetString(PyExc_TypeError, "contact_buf: float32 (4, H)");
        return NULL;
    }
    const int H = (int)PyArray_DIM((PyArrayObject*)contact_buf, 1);
    if (PyArray_NDIM(ca) != 2 || PyArray_DIM(ca, 0) != 4 || PyArray_DIM(ca, 1) < H || !PyArray_IS_C_CONTIGUOUS(ca) ||
        PyArray_TYPE(ca) != NPY_FLOAT64)
        goto decline;
    if (!PyArray_Check(best_buf) || PyArray_TYPE((PyArrayObject*)best_buf) != NPY_FLOAT32 ||
        !PyArray_IS_C_CONTIGUOUS((PyArrayObject*)best_buf)) {
        PyErr_SetString(PyExc_TypeError, "best_buf: float32 C-contiguous");
        return NULL;
    }
    const npy_intp P = PyArray_SIZE((PyArrayObject*)best_buf);
    PyArrayObject* b = (PyArrayObject*)PyArray_FROM_OTF(best, NPY_FLOAT32, NPY_ARRAY_IN_ARRAY | NPY_ARRAY_FORCECAST);
    if (!b) return NULL;
    PyArrayObject* pv = (PyArrayObject*)PyArray_FROM_OTF(prev, NPY_FLOAT64, NPY_ARRAY_IN_ARRAY | NPY_ARRAY_FORCECAST);
    if (!pv) {
        Py_DECREF(b);
        return NULL;
    }
    const int philox = rng == SRBD_RNG_PHILOX;
    PyArrayObject* kk = (PyArrayObject*)PyArray_FROM_OTF(mk, philox ? NPY_UINT64 : NPY_UINT32,
                                                         NPY_ARRAY_IN_ARRAY | NPY_ARRAY_FORCECAST);
    if (!kk) {
        Py_DECREF(b);
        Py_DECREF(pv);
        return NULL;
    }
    if (PyArray_SIZE(b) != P || PyArray_SIZE(pv) != 4 || PyArray_SIZE(kk) != 2) {
        Py_DECREF(b);
        Py_DECREF(pv);
        Py_DECREF(kk);
        goto decline;
    }

    /* ---- staging (as _step_fused) and the key split of with_newkey */
    memcpy(io->state_in, st, sizeof(st));
    memcpy(io->ref_base, rb, sizeof(rb));
    memcpy(io->seeds, sd, sizeof(sd));
    memcpy(io->hips, hp, sizeof(hp));
    memcpy(io->forward_vel, fv, sizeof(fv));
    const double* cd = (const double*)PyArray_DATA(ca);
    const npy_intp cstr = PyArray_DIM(ca, 1);
    for (int l = 0; l < 4; ++l) io->current_contact[l] = cd[(size_t)l * cstr];
    memcpy(io->previous_contact, PyArray_DATA(pv), 4 * sizeof(double));
    Py_DECREF(pv);
    io->yaw = yaw;
    float* cf = (float*)PyArray_DATA((PyArrayObject*)contact_buf);
    for (int l = 0; l < 4; ++l)
        for (int k = 0; k < H; ++k) cf[l * H + k] = (float)cd[(size_t)l * cstr + k];
    float* bb = (float*)PyArray_DATA((PyArrayObject*)best_buf);
    memcpy(bb, PyArray_DATA(b), sizeof(float) * (size_t)P);
    Py_DECREF(b);
    uint64_t seed, counter, nk0, nk1;
    if (philox) {
        const uint64_t* k = (const uint64_t*)PyArray_DATA(kk);
        nk0 = k[0];
        nk1 = k[1] + 1;
        seed = nk0;
        counter = nk1;
    } else {
        const uint32_t* k = (const uint32_t*)PyArray_DATA(kk);
        uint32_t o[4];
        g_split(k, 2, rng == SRBD_RNG_JAX ? 1 : 0, o);
        nk0 = o[0];
        nk1 = o[1];
        seed = ((uint64_t)o[0] << 32) | o[1];
        counter = (uint64_t)calls + 1;
    }
    Py_DECREF(kk);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_foothold(tam, ter, prm, ctx, io, cf, H, bb, ppl, seed, counter, res);
    Py_END_ALLOW_THREADS
    PyObject* cur = new_1d(NPY_FLOAT64, 4, io->current_contact, sizeof(double));
    PyObject* nk;
    if (philox) {
        const uint64_t k2[2] = {nk0, nk1};
        nk = new_1d(NPY_UINT64, 2, k2, sizeof(uint64_t));
    } else {
        const uint32_t k2[2] = {(uint32_t)nk0, (uint32_t)nk1};
        nk = new_1d(NPY_UINT32, 2, k2, sizeof(uint32_t));
    }
    if (!cur || !nk) {
        Py_XDECREF(cur);
        Py_XDECREF(nk);
        return NULL;
    }
    const long long ncalls = philox ? calls : calls + 1;
    if (rc != 0) return Py_BuildValue("(iiNNL)", rc, io->stage, cur, nk, ncalls);
    /* the objects the step hands out, made here rather than as numpy views in Python (one array each) */
    PyObject* pred = new_1d(NPY_FLOAT32, 24, res->predicted_state, sizeof(float));
    PyObject* nb = new_1d(NPY_FLOAT32, P, bb, sizeof(float));
    PyObject* grows = PyTuple_New(4);  /* leg l's GRFs times current_contact[l], float64 (the mask's promotion) */
    PyObject* frows = PyTuple_New(4);  /* the adapted footholds */
    PyObject* boxes = PyTuple_New(4);  /* [lower corner, upper corner] of a valid leg, else None */
    PyObject* hms = NULL;              /* the raycast patches, (rows, cols, 1, 3) each */
    PyObject* scores = NULL;           /* (4, rows * cols) */
    int ok = pred && nb && grows && frows && boxes;
    for (int l = 0; ok && l < 4; ++l) {
        double g[3];
        for (int c = 0; c < 3; ++c) g[c] = (double)res->grf[3 * l + c] * io->current_contact[l];
        PyObject* gr = new_1d(NPY_FLOAT64, 3, g, sizeof(double));
        PyObject* fr = new_1d(NPY_FLOAT64, 3, io->footholds + 3 * l, sizeof(double));
        PyObject* bx = NULL;
        if (io->valid[l]) {
            PyObject* lo = new_1d(NPY_FLOAT64, 3, io->boxes + 6 * l, sizeof(double));
            PyObject* hi = new_1d(NPY_FLOAT64, 3, io->boxes + 6 * l + 3, sizeof(double));
            bx = lo && hi ? PyList_New(2) : NULL;
            if (bx) {
                PyList_SET_ITEM(bx, 0, lo);
                PyList_SET_ITEM(bx, 1, hi);
            } else {
                Py_XDECREF(lo);
                Py_XDECREF(hi);
            }
        } else {
            bx = Py_None;
            Py_INCREF(bx);
        }
        if (gr) PyTuple_SET_ITEM(grows, l, gr);
        if (fr) PyTuple_SET_ITEM(frows, l, fr);
        if (bx) PyTuple_SET_ITEM(boxes, l, bx);
        ok = gr && fr && bx;
    }
    const npy_intp nc = (npy_intp)io->rows * io->cols;
    if (ok && io->heightmaps) {
        hms = PyTuple_New(4);
        npy_intp dh[4] = {io->rows, io->cols, 1, 3};
        for (int l = 0; ok && hms && l < 4; ++l) {
            PyObject* h = PyArray_SimpleNew(4, dh, NPY_FLOAT64);
            if (h) {
                memcpy(PyArray_DATA((PyArrayObject*)h), io->heightmaps + (size_t)l * nc * 3, sizeof(double) * 3 * nc);
                PyTuple_SET_ITEM(hms, l, h);
            }
            ok = h != NULL;
        }
        ok = ok && hms;
    } else if (ok) {  /* patches not copied out: each map stays pending -- (its seed (3,), the yaw) -- and raycasts on
                       * access (GpuHeightMap.data), the same values */
        hms = PyTuple_New(4);
        for (int l = 0; ok && hms && l < 4; ++l) {
            PyObject* c = new_1d(NPY_FLOAT64, 3, io->seeds + 3 * l, sizeof(double));
            PyObject* pnd = c ? Py_BuildValue("(Nd)", c, io->yaw) : NULL;
            if (pnd) PyTuple_SET_ITEM(hms, l, pnd);
            ok = pnd != NULL;
        }
        ok = ok && hms;
    }
    if (ok && io->scores) {
        npy_intp ds[2] = {4, nc};
        scores = PyArray_SimpleNew(2, ds, NPY_FLOAT64);
        if (scores) memcpy(PyArray_DATA((PyArrayObject*)scores), io->scores, sizeof(double) * 4 * nc);
        ok = scores != NULL;
    }
    if (!ok) {
        Py_XDECREF(pred);
        Py_XDECREF(nb);
        Py_XDECREF(grows);
        Py_XDECREF(frows);
        Py_XDECREF(boxes);
        Py_XDECREF(hms);
        Py_XDECREF(scores);
        Py_DECREF(cur);
        Py_DECREF(nk);
        return NULL;
    }
    if (!hms) {
        hms = Py_None;
        Py_INCREF(hms);
    }
    if (!scores) {
        scores = Py_None;
        Py_INCREF(scores);
    }
    return Py_BuildValue("(iiNNLNNNNNNN)", 0, io->stage, cur, nk, ncalls, grows, pred, nb, frows, boxes, hms, scores);
decline:
    if (PyErr_Occurred()) return NULL;
    Py_RETURN_NONE;
}

static PyMethodDef methods[] = {
    {"foothold_step", (PyCFunction)(void (*)(void))foothold_step, METH_FASTCALL,
     "TamolsMpcStep's one-call step through srbd_foothold_mpc_step"},
    {"bind", bind, METH_VARARGS, "bind(the library's entry point addresses)"},
    {"pgg_contact_sequence", (PyCFunction)(void (*)(void))pgg_contact_sequence, METH_FASTCALL,
     "pgg_contact_sequence(pgg_address, dts, lens) -> (4, cols) float64"},
    {"interface_step", (PyCFunction)(void (*)(void))interface_step, METH_FASTCALL,
     "SRBDControllerInterface.compute_control's sampling branch through srbd_interface_step"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_srbd_fast", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__srbd_fast(void) {
    import_array();
    for (int i = 0; i < 8; ++i) {
        k_state[i] = PyUnicode_InternFromString(STATE_KEYS[i]);
        k_ref[i] = PyUnicode_InternFromString(REF_KEYS[i]);
        if (!k_state[i] || !k_ref[i]) return NULL;
    }
    static const char* const legs[4] = {"FL", "FR", "RL", "RR"};
    for (int l = 0; l < 4; ++l)
        if (!(k_legs[l] = PyUnicode_InternFromString(legs[l]))) return NULL;
    k_zero = PyLong_FromLong(0);
    if (!k_zero) return NULL;
    return PyModule_Create(&moddef);
}
