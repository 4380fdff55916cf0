// The SciPy driver's request loop in native code (dhcos/_scipy_loop, a CPython extension).
//
// calibrate() with the SciPy driver (dhcos/calibrator.py run_starts) alternates SciPy's L-BFGS-B
// steps (scipy.optimize._lbfgsb.setulb, reverse communication) with one function+gradient
// request per live start group on the device (dh_surface_fg_begin / _end).  In Python the glue
// around each request -- the generator per start (lbfgsb_steps), fd_models, the slot calls, the
// bookkeeping of _consume -- costs ~20 us, twice the C1 request itself.  This
// module runs the same loop with the same calls:
//   - setulb is SciPy's own function object, called with the same argument objects and values
//     (the reference's optimizer bits; lbfgs_calibrator.py:259-269 -> minimize(L-BFGS-B));
//   - the model params of x0 and x0 + h are NumPy's exp / tanh ufuncs applied in place to packed
//     columns (the same inner loops as fd_models, so the same bits: tests/test_scipy_loop.py);
//   - the loop around setulb restates lbfgsb_steps (scipy/optimize/_lbfgsb_py.py, SciPy 1.15.3:
//     ScalarFunction's re-evaluation test, the maxiter / maxfun stops) and _advance_pipelined /
//     _consume (groups of starts on their own request slots, per-start n_calls and best loss).
// The device calls are libdhcos's C-ABI through addresses the caller passes (no link-time
// dependency), or -- for the CPU tests -- two Python callables begin(k, S) / end(k, S).
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <ctime>
#include <algorithm>
#include <vector>

namespace {

constexpr int kN = 13;                       // unconstrained parameters
constexpr int kPts = kN + 1;                 // points per function+gradient request
constexpr int kExpCols[10] = {0, 1, 2, 3, 5, 6, 7, 8, 10, 12};   // lbfgs_calibrator.py:62-87
constexpr int kTanhCols[2] = {4, 9};
constexpr int kMaxGroups = 4;            // include/dhcos.h DH_FG_SLOTS

typedef int (*begin_fn)(void*, const void*, const double*, const double*, int, double, double, int,
                        double, int);
typedef int (*end_fn)(void*, const void*, int, int, double*, double*, double*);
typedef int (*cancel_fn)(void*, int);

// a writable C-contiguous buffer of a Python object, released with the loop
struct Buffers {
    std::vector<Py_buffer> views;
    ~Buffers() {
        for (auto& v : views) PyBuffer_Release(&v);
    }
    template <class T>
    T* get(PyObject* o, Py_ssize_t min_bytes) {
        Py_buffer v;
        if (PyObject_GetBuffer(o, &v, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) return nullptr;
        if (v.len < min_bytes) {
            PyBuffer_Release(&v);
            PyErr_SetString(PyExc_ValueError, "buffer too small");
            return nullptr;
        }
        views.push_back(v);
        return (T*)v.buf;
    }
};

// one L-BFGS-B run: lbfgsb_steps' locals
struct Start {
    PyObject* arr[12];                       // x lo up nbd wa iwa task lsave isave dsave ln_task gs
    double* x;
    int32_t* task;
    double* gs;                              // the g handed to setulb (g.astype(float64))
    double sf_x[kN], sf_g[kN], sf_f = 0.0;   // ScalarFunction's last point and values
    double f = 0.0, g[kN] = {};              // the loop's f, g (0 before the first setulb call)
    long nfev = 0, nit = 0;
    bool first = true;
    int state = 2;                           // 0 finished, 1 dropped (setulb raised), 2 live
    double t_done = 0.0;
    long n_calls = 0;
    double best = HUGE_VAL;
};

struct Loop {
    PyObject *setulb, *m, *factr, *pgtol, *maxls, *np_exp, *np_tanh;
    long maxiter, maxfun;
    double h, sqrt_eps;
};

// host-time split of the loop (ns; read and cleared by stats()): setulb calls, fd_models,
// request begin, request end (its wait included), loops
enum { kTSetulb, kTModels, kTBegin, kTEnd, kTCount };
long long g_t[kTCount + 1] = {};
inline long long now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (long long)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}
struct Tick {
    int b;
    long long t0 = now_ns();
    explicit Tick(int bucket) : b(bucket) {}
    ~Tick() { g_t[b] += now_ns() - t0; }
};

double wall_time() {                         // time.time()
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

// lbfgsb_steps from the top of its loop until it needs (f, g) at a new point (0: s.sf_x holds
// it), finishes (1) or setulb raises an Exception (-1: the start is dropped, as the reference's
// per-start except -> continue); -2: a BaseException other than Exception (propagates).
int advance(Start& s, const Loop& L) {
    for (;;) {
        std::memcpy(s.gs, s.g, sizeof(s.g));
        PyObject* f = PyFloat_FromDouble(s.f);
        if (!f) return -2;
        PyObject* args = PyTuple_Pack(17, L.m, s.arr[0], s.arr[1], s.arr[2], s.arr[3], f,
                                      s.arr[11], L.factr, L.pgtol, s.arr[4], s.arr[5], s.arr[6],
                                      s.arr[7], s.arr[8], s.arr[9], L.maxls, s.arr[10]);
        Py_DECREF(f);
        if (!args) return -2;
        PyObject* r;
        {
            Tick tk(kTSetulb);
            r = PyObject_Call(L.setulb, args, nullptr);
        }
        Py_DECREF(args);
        if (!r) {
            if (PyErr_ExceptionMatches(PyExc_Exception)) {
                PyErr_Clear();
                return -1;
            }
            return -2;
        }
        Py_DECREF(r);
        // the loop's g is the array setulb received (g.astype makes it): setulb writes it when a
        // line search fails (it restores the previous iterate's gradient)
        std::memcpy(s.g, s.gs, sizeof(s.g));
        const int t = s.task[0];
        if (t == 3) {                        // FG: ScalarFunction.fun_and_grad
            bool same = true;
            for (int i = 0; i < kN; ++i) same = same && (s.x[i] == s.sf_x[i]);
            if (!same) {
                std::memcpy(s.sf_x, s.x, sizeof(s.sf_x));
                return 0;
            }
            s.f = s.sf_f;
            std::memcpy(s.g, s.sf_g, sizeof(s.g));
        } else if (t == 1) {                 // NEW_X
            if (++s.nit >= L.maxiter) {
                s.task[0] = 5;
                s.task[1] = 504;
            } else if (s.nfev > L.maxfun) {
                s.task[0] = 5;
                s.task[1] = 502;
            }
        } else {
            return 1;
        }
    }
}

// (f, g) at s.sf_x arrive: the value of lbfgsb_steps' yield
void receive(Start& s, double f0, const double* g0) {
    s.sf_f = f0;
    std::memcpy(s.sf_g, g0, sizeof(s.sf_g));
    if (s.first) {                           // ScalarFunction.__init__: nfev = 1, f / g stay 0
        s.first = false;
        s.nfev = 1;
        return;
    }
    ++s.nfev;
    s.f = f0;
    std::memcpy(s.g, g0, sizeof(s.g));
}

struct Slot {
    double *x, *model, *f, *g, *low;
    PyObject *exp_views, *tanh_views;        // lists indexed by S: packed [2 S 10] / [2 S 2]
    std::vector<double*> eptr, tptr;         // their buffers
    std::vector<int> ids;                    // the starts of the request in flight
    bool busy = false;
};

// fd_models (dhcos/calibrator.py): model [2][S][13] of the slot's x rows and of x + h
int fd_models(Slot& sl, int S, const Loop& L) {
    Tick tk(kTModels);
    double* P = sl.model;
    for (int j = 0; j < S; ++j) {
        const double* x = sl.x + (size_t)j * kN;
        double* pb = P + (size_t)j * kN;
        double* pp = P + ((size_t)S + j) * kN;
        for (int i = 0; i < kN; ++i) {
            double xh = x[i] + L.h;
            if (xh - x[i] == 0.0) {          // the absolute step vanishes: SciPy's relative step
                const double sign = x[i] >= 0.0 ? 1.0 : -1.0;
                const double a = std::fabs(x[i]);     // np.maximum: NaN propagates
                xh = x[i] + L.sqrt_eps * sign * (a != a ? a : (a > 1.0 ? a : 1.0));
            }
            pb[i] = x[i];
            pp[i] = xh;
        }
    }
    PyObject* ev = PyList_GET_ITEM(sl.exp_views, S);
    PyObject* tv = PyList_GET_ITEM(sl.tanh_views, S);
    double* E = sl.eptr[S];
    double* Tn = sl.tptr[S];
    const int R = 2 * S;
    for (int q = 0; q < R; ++q) {
        for (int c = 0; c < 10; ++c) E[q * 10 + c] = P[(size_t)q * kN + kExpCols[c]];
        for (int c = 0; c < 2; ++c) Tn[q * 2 + c] = P[(size_t)q * kN + kTanhCols[c]];
    }
    PyObject* r = PyObject_CallFunctionObjArgs(L.np_exp, ev, ev, nullptr);
    if (!r) return -1;
    Py_DECREF(r);
    r = PyObject_CallFunctionObjArgs(L.np_tanh, tv, tv, nullptr);
    if (!r) return -1;
    Py_DECREF(r);
    for (int q = 0; q < R; ++q) {
        for (int c = 0; c < 10; ++c) P[(size_t)q * kN + kExpCols[c]] = E[q * 10 + c];
        for (int c = 0; c < 2; ++c) P[(size_t)q * kN + kTanhCols[c]] = Tn[q * 2 + c];
    }
    return 0;
}

struct Device {
    begin_fn begin = nullptr;
    end_fn end = nullptr;
    cancel_fn cancel = nullptr;
    void* ctx[kMaxGroups] = {};              // slot k's context (its stream and scratch)
    const void* surf = nullptr;
    double S0 = 0, r = 0, L = 0;
    int N = 0;
    PyObject *begin_cb = nullptr, *end_cb = nullptr;   // CPU tests: Python callables
};

// 0 ok, > 0 a libdhcos error code, -1 a Python exception
int dev_begin(Device& D, Slot& sl, int k, int S) {
    Tick tk(kTBegin);
    if (D.begin_cb) {
        PyObject* r = PyObject_CallFunction(D.begin_cb, "ii", k, S);
        if (!r) return -1;
        Py_DECREF(r);
        return 0;
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = D.begin(D.ctx[k], D.surf, sl.x, sl.model, S, D.S0, D.r, D.N, D.L, k);
    Py_END_ALLOW_THREADS
    return rc;
}

int dev_end(Device& D, Slot& sl, int k, int S) {
    Tick tk(kTEnd);
    if (D.end_cb) {
        PyObject* r = PyObject_CallFunction(D.end_cb, "ii", k, S);
        if (!r) return -1;
        Py_DECREF(r);
        return 0;
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = D.end(D.ctx[k], D.surf, k, S, sl.f, sl.g, sl.low);
    Py_END_ALLOW_THREADS
    return rc;
}

void cancel_busy(Device& D, Slot* slots, int G) {
    for (int k = 0; k < G; ++k) {
        if (!slots[k].busy) continue;
        slots[k].busy = false;
        if (D.cancel) {
            Py_BEGIN_ALLOW_THREADS
            (void)D.cancel(D.ctx[k], k);
            Py_END_ALLOW_THREADS
        }
    }
}

double as_double(PyObject* t, Py_ssize_t i) { return PyFloat_AsDouble(PyTuple_GET_ITEM(t, i)); }

// run(device, groups, slots, starts, setulb, exp, tanh, (m, factr, pgtol, maxls, maxiter, maxfun,
//     h, sqrt_eps))
//   device: (begin_addr, end_addr, cancel_addr, ctx, surf, S0, r, N, L) or (begin_cb, end_cb);
//           ctx: one context handle, or a tuple with slot k's context at k
//   groups: up to kMaxGroups lists of ascending start ids; group k uses request slot k
//   slots:  per group (x [s_max 13], model [2 s_max 13], f [s_max], g [s_max 13], low [s_max],
//           exp_views, tanh_views)
//   starts: per start (x, lo, up, nbd, wa, iwa, task, lsave, isave, dsave, ln_task, g_scratch),
//           x holding x0
// -> (rc, launches, loss_evals, [(state, f, g, nfev, nit, t_done, n_calls, best_loss)])
//    rc != 0: the libdhcos error a begin / end returned (slots cancelled; the caller raises)
PyObject* run(PyObject*, PyObject* args) {
    PyObject *dev, *groups, *slots_in, *starts_in, *setulb, *np_exp, *np_tanh, *consts;
    if (!PyArg_ParseTuple(args, "O!O!O!O!OOOO!", &PyTuple_Type, &dev, &PyList_Type, &groups,
                          &PyList_Type, &slots_in, &PyList_Type, &starts_in, &setulb, &np_exp,
                          &np_tanh, &PyTuple_Type, &consts))
        return nullptr;
    if (PyTuple_GET_SIZE(consts) != 8) {
        PyErr_SetString(PyExc_ValueError, "consts: (m, factr, pgtol, maxls, maxiter, maxfun, h, sqrt_eps)");
        return nullptr;
    }
    Loop L{setulb, PyTuple_GET_ITEM(consts, 0), PyTuple_GET_ITEM(consts, 1),
           PyTuple_GET_ITEM(consts, 2), PyTuple_GET_ITEM(consts, 3), np_exp, np_tanh,
           PyLong_AsLong(PyTuple_GET_ITEM(consts, 4)), PyLong_AsLong(PyTuple_GET_ITEM(consts, 5)),
           as_double(consts, 6), as_double(consts, 7)};
    if (PyErr_Occurred()) return nullptr;

    Device D;
    if (PyTuple_GET_SIZE(dev) == 2) {
        D.begin_cb = PyTuple_GET_ITEM(dev, 0);
        D.end_cb = PyTuple_GET_ITEM(dev, 1);
    } else if (PyTuple_GET_SIZE(dev) == 9) {
        D.begin = (begin_fn)PyLong_AsVoidPtr(PyTuple_GET_ITEM(dev, 0));
        D.end = (end_fn)PyLong_AsVoidPtr(PyTuple_GET_ITEM(dev, 1));
        D.cancel = (cancel_fn)PyLong_AsVoidPtr(PyTuple_GET_ITEM(dev, 2));
        PyObject* cx = PyTuple_GET_ITEM(dev, 3);     // one context, or one per slot
        for (int k = 0; k < kMaxGroups; ++k) {
            PyObject* c = PyTuple_Check(cx) ? (k < PyTuple_GET_SIZE(cx) ? PyTuple_GET_ITEM(cx, k)
                                                                        : nullptr)
                                            : cx;
            D.ctx[k] = c ? PyLong_AsVoidPtr(c) : nullptr;
        }
        D.surf = PyLong_AsVoidPtr(PyTuple_GET_ITEM(dev, 4));
        D.S0 = as_double(dev, 5);
        D.r = as_double(dev, 6);
        D.N = (int)PyLong_AsLong(PyTuple_GET_ITEM(dev, 7));
        D.L = as_double(dev, 8);
        if (PyErr_Occurred()) return nullptr;
        if (!D.begin || !D.end || !D.cancel || !D.ctx[0] || !D.surf) {
            PyErr_SetString(PyExc_ValueError, "null device entry point or handle");
            return nullptr;
        }
    } else {
        PyErr_SetString(PyExc_ValueError, "device: 9-tuple of the C-ABI or (begin, end)");
        return nullptr;
    }

    const int G = (int)PyList_GET_SIZE(groups);
    const int n = (int)PyList_GET_SIZE(starts_in);
    if (G < 1 || G > kMaxGroups || PyList_GET_SIZE(slots_in) != G) {
        PyErr_SetString(PyExc_ValueError, "1 .. 4 groups, one slot each");
        return nullptr;
    }
    if (!D.begin_cb)
        for (int k = 0; k < G; ++k)
            if (!D.ctx[k]) {
                PyErr_SetString(PyExc_ValueError, "no context for a group's slot");
                return nullptr;
            }
    Buffers B;
    std::vector<Start> st(n);
    for (int s = 0; s < n; ++s) {
        PyObject* t = PyList_GET_ITEM(starts_in, s);
        if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 12) {
            PyErr_SetString(PyExc_ValueError, "start: 12-tuple of arrays");
            return nullptr;
        }
        for (int i = 0; i < 12; ++i) st[s].arr[i] = PyTuple_GET_ITEM(t, i);
        st[s].x = B.get<double>(st[s].arr[0], kN * 8);
        st[s].task = B.get<int32_t>(st[s].arr[6], 8);
        st[s].gs = B.get<double>(st[s].arr[11], kN * 8);
        if (!st[s].x || !st[s].task || !st[s].gs) return nullptr;
        std::memcpy(st[s].sf_x, st[s].x, sizeof(st[s].sf_x));   // the first request: x0
    }
    Slot slots[kMaxGroups];
    std::vector<std::vector<int>> grp(G);
    for (int k = 0; k < G; ++k) {
        PyObject* gl = PyList_GET_ITEM(groups, k);
        PyObject* t = PyList_GET_ITEM(slots_in, k);
        if (!PyList_Check(gl) || !PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 7) {
            PyErr_SetString(PyExc_ValueError, "group: list of ids; slot: 7-tuple");
            return nullptr;
        }
        for (Py_ssize_t j = 0; j < PyList_GET_SIZE(gl); ++j) {
            const long id = PyLong_AsLong(PyList_GET_ITEM(gl, j));
            if (id < 0 || id >= n) {
                if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "start id out of range");
                return nullptr;
            }
            grp[k].push_back((int)id);
        }
        const Py_ssize_t smax = (Py_ssize_t)std::max<size_t>(1, grp[k].size());
        Slot& sl = slots[k];
        sl.x = B.get<double>(PyTuple_GET_ITEM(t, 0), smax * kN * 8);
        sl.model = B.get<double>(PyTuple_GET_ITEM(t, 1), 2 * smax * kN * 8);
        sl.f = B.get<double>(PyTuple_GET_ITEM(t, 2), smax * 8);
        sl.g = B.get<double>(PyTuple_GET_ITEM(t, 3), smax * kN * 8);
        sl.low = B.get<double>(PyTuple_GET_ITEM(t, 4), smax * 8);
        sl.exp_views = PyTuple_GET_ITEM(t, 5);
        sl.tanh_views = PyTuple_GET_ITEM(t, 6);
        if (!sl.x || !sl.model || !sl.f || !sl.g || !sl.low) return nullptr;
        if (!PyList_Check(sl.exp_views) || !PyList_Check(sl.tanh_views) ||
            PyList_GET_SIZE(sl.exp_views) <= smax || PyList_GET_SIZE(sl.tanh_views) <= smax) {
            PyErr_SetString(PyExc_ValueError, "exp / tanh views: lists indexed 1 .. s_max");
            return nullptr;
        }
        sl.eptr.assign(smax + 1, nullptr);
        sl.tptr.assign(smax + 1, nullptr);
        for (Py_ssize_t S = 1; S <= smax; ++S) {
            sl.eptr[S] = B.get<double>(PyList_GET_ITEM(sl.exp_views, S), 2 * S * 10 * 8);
            sl.tptr[S] = B.get<double>(PyList_GET_ITEM(sl.tanh_views, S), 2 * S * 2 * 8);
            if (!sl.eptr[S] || !sl.tptr[S]) return nullptr;
        }
    }

    long launches = 0, loss_evals = 0;
    int rc = 0;
    bool py_err = false;
    // submit(k): the group's live starts' points into the slot, their model params, the request
    auto submit = [&](int k) -> bool {
        Slot& sl = slots[k];
        sl.ids.clear();
        for (int id : grp[k])
            if (st[id].state == 2) sl.ids.push_back(id);
        const int S = (int)sl.ids.size();
        if (S == 0) return true;
        for (int j = 0; j < S; ++j)
            std::memcpy(sl.x + (size_t)j * kN, st[sl.ids[j]].sf_x, kN * sizeof(double));
        if (fd_models(sl, S, L)) {
            py_err = true;
            return false;
        }
        loss_evals += (long)S * kPts;
        const int e = dev_begin(D, sl, k, S);
        if (e) {
            if (e < 0) py_err = true;
            else rc = e;
            return false;
        }
        sl.busy = true;
        return true;
    };
    // consume(k): the request's results to its starts (run_starts' _consume)
    auto consume = [&](int k) -> bool {
        Slot& sl = slots[k];
        for (size_t j = 0; j < sl.ids.size(); ++j) {
            Start& s = st[sl.ids[j]];
            s.n_calls += kPts;
            if (sl.low[j] < s.best) s.best = sl.low[j];
            receive(s, sl.f[j], sl.g + j * kN);
            const int a = advance(s, L);
            if (a == -2) {
                py_err = true;
                return false;
            }
            if (a == 1) {
                s.state = 0;
                s.t_done = wall_time();
            } else if (a == -1) {
                s.state = 1;
            }
        }
        return true;
    };

    const long long t_run = now_ns();
    bool ok = true;
    for (int k = 0; k < G && ok; ++k) ok = submit(k);
    while (ok) {
        bool any = false;
        for (int k = 0; k < G && ok; ++k) {
            Slot& sl = slots[k];
            if (!sl.busy) continue;
            any = true;
            const int e = dev_end(D, sl, k, (int)sl.ids.size());
            if (e) {
                if (e < 0) py_err = true;
                else rc = e;
                ok = false;
                break;
            }
            sl.busy = false;
            ++launches;
            ok = consume(k) && submit(k);
            if (ok && PyErr_CheckSignals() != 0) {
                py_err = true;
                ok = false;
            }
        }
        if (!any) break;
    }
    g_t[kTCount] += now_ns() - t_run;
    if (!ok) {
        PyObject *et = nullptr, *ev = nullptr, *tb = nullptr;
        if (py_err) PyErr_Fetch(&et, &ev, &tb);
        cancel_busy(D, slots, G);
        if (py_err) {
            PyErr_Restore(et, ev, tb);
            return nullptr;
        }
    }
    PyObject* out = PyList_New(n);
    if (!out) return nullptr;
    for (int s = 0; s < n; ++s) {
        const Start& S = st[s];
        PyObject* g = PyTuple_New(kN);
        if (!g) {
            Py_DECREF(out);
            return nullptr;
        }
        for (int i = 0; i < kN; ++i) PyTuple_SET_ITEM(g, i, PyFloat_FromDouble(S.g[i]));
        PyObject* row = Py_BuildValue("(idNlldld)", S.state, S.f, g, S.nfev, S.nit, S.t_done,
                                      S.n_calls, S.best);
        if (!row) {
            Py_DECREF(out);
            return nullptr;
        }
        PyList_SET_ITEM(out, s, row);
    }
    return Py_BuildValue("(illN)", rc, launches, loss_evals, out);
}

// stats() -> (setulb, fd_models, begin, end, loop) host ns summed over the runs since the last
// call (a diagnostic: tools/calib_profile.py)
PyObject* stats(PyObject*, PyObject*) {
    PyObject* r = Py_BuildValue("(LLLLL)", g_t[0], g_t[1], g_t[2], g_t[3], g_t[4]);
    std::memset(g_t, 0, sizeof(g_t));
    return r;
}

PyMethodDef kMethods[] = {
    {"stats", stats, METH_NOARGS, "stats(): the loop's host-time split since the last call"},
    {"run", run, METH_VARARGS,
     "run(device, groups, slots, starts, setulb, exp, tanh, consts): the SciPy driver's request "
     "loop (see dh_scipy_loop.cpp)"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_scipy_loop",
                       "The SciPy driver's request loop in native code.", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__scipy_loop(void) { return PyModule_Create(&kModule); }
