// torch_ext.cpp -- LaplaceLearningSparseHard.apply as native code over the C ABI of include/gll.h.
//
// The reference's LaplaceLearningSparseHard is a Python torch.autograd.Function
// (/root/reference/GLL.py:10-177).  At ~10^4 calls/s the host side of a call is on the step's
// critical path, so everything `apply` does before and after its kernels lives here:
//   * `apply(X, label_matrix, tau=0, epsilon='auto', k=25)` is a METH_FASTCALL CPython function
//     (no pybind dispatch, no Python frame): argument checks with the reference's error
//     behaviour, tensor marshalling, the workspace from torch's caching allocator, gll_forward on
//     the current HIP stream, and -- when X requires grad -- one autograd Node with its saved
//     state in plain members (no IValue map, no torch::autograd::Function bookkeeping);
//   * the device status words (tiny eps, CG non-convergence, grid-barrier failure) accumulate in
//     a sticky per-device sink that is copied to pinned memory every kFlushEvery calls and turned
//     into the reference's warnings (GLL.py:240-241, 273-274) at a later call, with no host sync.
// A leading batch dimension (X: B x n x d, label_matrix: B x base x C or shared base x C) runs
// B independent graphs through gll_forward_batched / gll_backward_batched.
// No numerics here.
#include <Python.h>
#include <torch/extension.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/functions/utils.h>
#include <torch/csrc/autograd/python_variable.h>
#include <torch/csrc/autograd/saved_variable.h>
#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "gll.h"

namespace {

using torch::autograd::variable_list;

constexpr int64_t kDefaultK = 25;       // GLL.py:27
constexpr int64_t kMaxK = 257;          // include/gll.h: 2 <= K <= 257
constexpr int kMaxIter = 1000;
constexpr float kRtol = 1e-6f;
constexpr int kFlushEvery = 64;         // calls between status copies
constexpr int kRing = 8;                // status copies in flight per device

// ------------------------------------------------------------------------------------------
// Python-level errors raised from C++ (the functions below hold the GIL)
// ------------------------------------------------------------------------------------------
struct PyErrSet {};   // a Python exception is set: unwind to the CPython entry point

[[noreturn]] void raise_py(PyObject* type, const std::string& msg) {
    PyErr_SetString(type, msg.c_str());
    throw PyErrSet{};
}

void warn_py(PyObject* category, const std::string& msg) {
    if (PyErr_WarnEx(category, msg.c_str(), 1) < 0) throw PyErrSet{};   // -W error
}

// ------------------------------------------------------------------------------------------
// Status sink per device (GLL_ST_* words; include/gll.h gll_problem.status_sink)
// ------------------------------------------------------------------------------------------
struct StatusCopy {
    hipEvent_t ev = nullptr;
    int32_t* host = nullptr;   // pinned, GLL_ST_NWORDS
    bool busy = false;
};

struct DeviceStatus {
    at::Tensor sink;           // int32 [GLL_ST_NWORDS] on the device, sticky between flushes
    int calls = 0;
    StatusCopy ring[kRing];
    std::deque<int> order;     // ring slots in flight, oldest first
};

std::mutex g_status_mu;
std::vector<DeviceStatus*> g_status;   // by device index (never freed: process lifetime)

DeviceStatus& status_of(int dev) {
    std::lock_guard<std::mutex> lk(g_status_mu);
    if (int(g_status.size()) <= dev) g_status.resize(dev + 1, nullptr);
    DeviceStatus*& s = g_status[dev];
    if (!s) {
        s = new DeviceStatus;
        s->sink = at::zeros({GLL_ST_NWORDS},
                            at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev));
    }
    return *s;
}

// Turn one completed copy of the status words into the reference's warnings (GLL.py:240-241
// warns; a non-converged CG prints at GLL.py:273-274) or an error (a lost grid barrier).
void report(const int32_t* st) {
    if (st[GLL_ST_SOLVE_FAILED])
        raise_py(PyExc_RuntimeError,
                 "GLL: the fused backward's gradient gave up waiting for the adjoint solves; "
                 "its grad_X was written as NaN");
    if (st[GLL_ST_GRID_RESCUED])
        warn_py(PyExc_RuntimeWarning,
                "GLL: " + std::to_string(st[GLL_ST_GRID_RESCUED]) +
                    " whole-GPU CG solve(s) lost their grid barrier (other kernels held the "
                    "CUs) and were solved by one workgroup instead: correct, slower");
    if (st[GLL_ST_TINY_EPS]) warn_py(PyExc_UserWarning, "Epsilon in KNN is very close to zero.");
    if (st[GLL_ST_FWD_NONCONV])
        warn_py(PyExc_RuntimeWarning,
                "GLL forward CG: " + std::to_string(st[GLL_ST_FWD_NONCONV]) +
                    " column solve(s) reached max_iter (" + std::to_string(st[GLL_ST_FWD_ITERS]) +
                    " iterations)");
    if (st[GLL_ST_BWD_NONCONV])
        warn_py(PyExc_RuntimeWarning,
                "GLL adjoint CG: " + std::to_string(st[GLL_ST_BWD_NONCONV]) +
                    " column solve(s) reached max_iter (" + std::to_string(st[GLL_ST_BWD_ITERS]) +
                    " iterations)");
}

// Completed copies (all of them when `block`), oldest first.
void poll(DeviceStatus& s, bool block) {
    while (!s.order.empty()) {
        StatusCopy& c = s.ring[s.order.front()];
        if (block) {
            (void)hipEventSynchronize(c.ev);
        } else if (hipEventQuery(c.ev) != hipSuccess) {
            (void)hipGetLastError();   // hipErrorNotReady must not linger as the last error
            return;
        }
        s.order.pop_front();
        c.busy = false;
        int32_t st[GLL_ST_NWORDS];
        std::memcpy(st, c.host, sizeof(st));
        report(st);
    }
}

// Copy the sink to pinned memory behind this stream's work, then clear it.
void flush(DeviceStatus& s, int dev, hipStream_t stream) {
    int slot = -1;
    for (int q = 0; q < kRing; ++q)
        if (!s.ring[q].busy) {
            slot = q;
            break;
        }
    if (slot < 0) {   // every copy still in flight: wait for the oldest
        poll(s, false);
        if (s.order.size() == size_t(kRing)) {
            StatusCopy& c = s.ring[s.order.front()];
            (void)hipEventSynchronize(c.ev);
            poll(s, false);
        }
        for (int q = 0; q < kRing; ++q)
            if (!s.ring[q].busy) {
                slot = q;
                break;
            }
        if (slot < 0) return;
    }
    StatusCopy& c = s.ring[slot];
    if (!c.ev) {
        c10::DeviceGuard g(c10::Device(c10::kCUDA, dev));
        if (hipEventCreateWithFlags(&c.ev, hipEventDisableTiming) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&c.host), GLL_ST_NWORDS * sizeof(int32_t),
                          hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            raise_py(PyExc_RuntimeError, "GLL: cannot allocate the status copy buffers");
        }
    }
    void* sink = s.sink.data_ptr();
    if (hipMemcpyAsync(c.host, sink, GLL_ST_NWORDS * sizeof(int32_t), hipMemcpyDeviceToHost,
                       stream) != hipSuccess ||
        hipEventRecord(c.ev, stream) != hipSuccess ||
        hipMemsetAsync(sink, 0, GLL_ST_NWORDS * sizeof(int32_t), stream) != hipSuccess) {
        (void)hipGetLastError();
        raise_py(PyExc_RuntimeError, "GLL: status copy failed");
    }
    c.busy = true;
    s.order.push_back(slot);
    s.calls = 0;
}

hipStream_t current_stream(int dev) { return c10::hip::getCurrentHIPStream(dev).stream(); }

void after_call(DeviceStatus& s, int dev, hipStream_t stream) {
    if (++s.calls >= kFlushEvery) flush(s, dev, stream);
}

// ------------------------------------------------------------------------------------------
// Tensor marshalling
// ------------------------------------------------------------------------------------------
int dtype_code(at::Tensor& t) {
    switch (t.scalar_type()) {
        case at::kFloat: return GLL_DT_F32;
        case at::kDouble: return GLL_DT_F64;
        case at::kLong: return GLL_DT_I64;
        default: t = t.to(at::kFloat); return GLL_DT_F32;
    }
}

at::Tensor features(const at::Tensor& X, const c10::Device& dev) {
    // the common case (fp32, contiguous, aligned, on the device) needs no new tensor
    if (X.device() == dev && X.scalar_type() == at::kFloat && X.is_contiguous() &&
        reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0)
        return X;
    at::Tensor X32 = X.detach().to(dev, at::kFloat).contiguous();
    if (reinterpret_cast<uintptr_t>(X32.data_ptr()) % 16) X32 = X32.clone();  // 16-B vector path
    return X32;
}

void check_rc(int rc, const char* what) {
    TORCH_CHECK(rc == GLL_OK, what, " failed: ", gll_strerror(rc), " (code ", rc, ")");
}

gll_problem make_problem(int64_t n, int64_t d, int64_t base, int64_t C, int64_t k, double tau,
                         double eps, int32_t* sink) {
    gll_problem p;
    p.n = int32_t(n);
    p.d = int32_t(d);
    p.base = int32_t(base);
    p.C = int32_t(C);
    p.K = int32_t(std::min<int64_t>(k, n));
    p.max_iter = kMaxIter;
    p.tau = float(tau);
    p.eps = float(eps);
    p.rtol = kRtol;
    p.flags = 0;
    p.status_sink = sink;
    return p;
}

// Exploding-gradient report of the adversarial scripts' inline copy
// (train_and_adversarial.py:177-183): < 0 = off (the default).
double g_grad_diag = -1.0;

// ------------------------------------------------------------------------------------------
// The autograd node: gll_backward over the saved workspace (GLL.py:76-177)
// ------------------------------------------------------------------------------------------
struct LaplaceBackward : public torch::autograd::Node {
    torch::autograd::SavedVariable X_;
    at::Tensor ws_;
    gll_problem p_{};
    int64_t B_ = 1;
    double diag_ = -1.0;

    std::string name() const override { return "LaplaceLearningSparseHardBackward"; }

    void release_variables() override {
        std::lock_guard<std::mutex> lk(mutex_);
        X_.reset_data();
        ws_.reset();
    }

    variable_list apply(variable_list&& grads) override {
        std::lock_guard<std::mutex> lk(mutex_);
        const at::Tensor X = X_.unpack(shared_from_this());   // raises on a second backward
        if (!grads[0].defined()) return {at::Tensor()};
        const c10::Device dev = ws_.device();
        c10::DeviceGuard guard(dev);
        at::Tensor X32 = features(X, dev);
        at::Tensor g = grads[0].device() == dev ? grads[0] : grads[0].to(dev);
        if (g.scalar_type() != at::kFloat && g.scalar_type() != at::kDouble) g = g.to(at::kDouble);
        if (!g.is_contiguous()) g = g.contiguous();
        const int gcode = g.scalar_type() == at::kFloat ? GLL_DT_F32 : GLL_DT_F64;
        at::Tensor gradX = at::empty(X.sizes(), X32.options());
        check_rc(gll_backward_batched(&p_, int(B_), X32.data_ptr<float>(), ws_.data_ptr(),
                                      g.data_ptr(), gcode, gradX.data_ptr<float>(),
                                      current_stream(dev.index())),
                 "gll_backward");
        if (diag_ >= 0.0) report_gradient(g, gradX);
        if (gradX.device() != X.device() || gradX.scalar_type() != X.scalar_type())
            gradX = gradX.to(X.device(), X.scalar_type());
        return {gradX};
    }

    // train_and_adversarial.py:177-183 (synchronises: diagnostic mode only)
    void report_gradient(const at::Tensor& g, const at::Tensor& gradX) {
        const double out_norm = at::linalg_vector_norm(gradX).item<double>();
        if (!(out_norm > diag_)) return;
        gll_view v;
        check_rc(gll_workspace_view(&p_, ws_.data_ptr(), &v), "gll_workspace_view");
        const int64_t m = int64_t(p_.n) - p_.base;
        const int64_t off = reinterpret_cast<char*>(v.wadj) - static_cast<char*>(ws_.data_ptr());
        const at::Tensor wadj = ws_.narrow(0, off, 4 * m * p_.C).view(at::kFloat);
        const double gn = at::linalg_vector_norm(g.to(at::kDouble)).item<double>();
        const double wn = at::linalg_vector_norm(wadj.to(at::kDouble)).item<double>();
        pybind11::gil_scoped_acquire gil;
        pybind11::print("possible exploding gradient");
        pybind11::print("grad norm: ", gn);
        pybind11::print("w norm: ", wn);
        pybind11::print("out norm: ", out_norm);
    }
};

// ------------------------------------------------------------------------------------------
// apply(X, label_matrix, tau=0, epsilon='auto', k=25)        GLL.py:14-73
// ------------------------------------------------------------------------------------------
double parse_float(PyObject* o, const char* what) {
    const double v = PyFloat_AsDouble(o);
    if (v == -1.0 && PyErr_Occurred()) {
        PyErr_Clear();
        raise_py(PyExc_TypeError, std::string(what) + " must be a number");
    }
    return v;
}

// epsilon: a number > 0 (fixed, GLL.py:226) or 'auto' (GLL.py:200-205) -> <= 0 for the ABI
double parse_eps(PyObject* o) {
    if (PyUnicode_Check(o)) {
        if (PyUnicode_CompareWithASCIIString(o, "auto") != 0) {
            const char* s = PyUnicode_AsUTF8(o);
            raise_py(PyExc_ValueError,
                     std::string("epsilon must be a number or 'auto', got '") + (s ? s : "?") + "'");
        }
        return 0.0;
    }
    const double e = parse_float(o, "epsilon");
    if (!(e > 0.0)) {
        // GLL.py:240-241 warns for any eps < 1e-10.  The reference uses eps only as the product
        // eps[rows] * eps[cols] (GLL.py:233-234), so a negative eps builds the graph of |eps|;
        // eps = 0 (or NaN) divides by zero there, here it disconnects the graph (W = 0)
        warn_py(PyExc_UserWarning, "Epsilon in KNN is very close to zero.");
        return e < 0.0 ? -e : 1e-30;
    }
    return e;
}

const at::Tensor& tensor_arg(PyObject* o, const char* what) {
    if (!THPVariable_Check(o)) raise_py(PyExc_TypeError, std::string(what) + " must be a Tensor");
    return THPVariable_Unpack(o);
}

PyObject* apply_impl(PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
    static const char* names[] = {"X", "label_matrix", "tau", "epsilon", "k"};
    PyObject* a[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    if (nargs > 5) raise_py(PyExc_TypeError, "apply() takes at most 5 arguments");
    for (Py_ssize_t q = 0; q < nargs; ++q) a[q] = args[q];
    if (kwnames) {
        const Py_ssize_t nk = PyTuple_GET_SIZE(kwnames);
        for (Py_ssize_t q = 0; q < nk; ++q) {
            const char* kn = PyUnicode_AsUTF8(PyTuple_GET_ITEM(kwnames, q));
            int slot = -1;
            for (int t = 0; t < 5 && kn; ++t)
                if (std::strcmp(kn, names[t]) == 0) slot = t;
            if (slot < 0 || a[slot])
                raise_py(PyExc_TypeError, std::string("apply() got an unexpected or repeated "
                                                      "keyword argument '") + (kn ? kn : "?") + "'");
            a[slot] = args[nargs + q];
        }
    }
    if (!a[0] || !a[1]) raise_py(PyExc_TypeError, "apply() needs X and label_matrix");
    const at::Tensor& X = tensor_arg(a[0], "X");
    const at::Tensor& Y = tensor_arg(a[1], "label_matrix");
    const double tau = a[2] ? parse_float(a[2], "tau") : 0.0;
    const double eps = a[3] ? parse_eps(a[3]) : 0.0;
    int64_t k = kDefaultK;
    if (a[4]) {
        k = PyLong_AsLongLong(a[4]);
        if (k == -1 && PyErr_Occurred()) {
            PyErr_Clear();
            raise_py(PyExc_TypeError, "k must be an int");
        }
    }
    if ((X.dim() != 2 && X.dim() != 3) || (Y.dim() != 2 && Y.dim() != X.dim()))
        raise_py(PyExc_ValueError,
                 "X must be n x d (or B x n x d), label_matrix base x C (or B x base x C)");
    const int64_t n = X.size(-2), d = X.size(-1), base = Y.size(-2), C = Y.size(-1);
    const int64_t kk = std::min(k, n);
    if (kk < 2 || kk > kMaxK)
        raise_py(PyExc_ValueError, "k = " + std::to_string(k) + " (n = " + std::to_string(n) +
                                       "): the kNN count incl. self must satisfy 2 <= min(k, n) <= " +
                                       std::to_string(kMaxK));
    // device: X's, or the current one for CPU input (the result goes back to the CPU)
    int devi;
    if (X.is_cuda()) {
        devi = X.device().index();
    } else {
        if (c10::hip::device_count() == 0)
            raise_py(PyExc_RuntimeError, "graphlearninglayer_amd needs a ROCm GPU (no CPU fallback)");
        devi = c10::hip::current_device();
    }
    const c10::Device dev(c10::kCUDA, devi);
    c10::DeviceGuard guard(dev);
    DeviceStatus& st = status_of(devi);
    if (!st.order.empty()) poll(st, false);
    const bool batched = X.dim() == 3;
    const int64_t B = batched ? X.size(0) : 1;
    at::Tensor X32 = features(X, dev);
    at::Tensor Yd = Y.device() == dev ? Y : Y.detach().to(dev);
    const int ycode = dtype_code(Yd);
    if (batched && Y.dim() == 2) Yd = Yd.unsqueeze(0).expand({B, base, C});   // shared labels
    if (batched && Yd.size(0) != B)
        raise_py(PyExc_ValueError, "label_matrix batch " + std::to_string(Yd.size(0)) +
                                       " != " + std::to_string(B));
    if (!Yd.is_contiguous()) Yd = Yd.contiguous();
    gll_problem p = make_problem(n, d, base, C, k, tau, eps, st.sink.data_ptr<int32_t>());
    const size_t nb = gll_workspace_bytes(&p);
    if (nb == 0)
        raise_py(PyExc_ValueError, "unsupported GLL problem n=" + std::to_string(n) + " d=" +
                                       std::to_string(d) + " base=" + std::to_string(base) +
                                       " C=" + std::to_string(C) + " k=" + std::to_string(k));
    const auto opts = X32.options();
    at::Tensor ws = at::empty({int64_t(nb) * B}, opts.dtype(at::kByte));
    at::Tensor U = batched ? at::empty({B, n - base, C}, opts.dtype(at::kDouble))
                           : at::empty({n - base, C}, opts.dtype(at::kDouble));
    const hipStream_t s = current_stream(devi);
    check_rc(gll_forward_batched(&p, int(B), X32.data_ptr<float>(), Yd.data_ptr(), ycode,
                                 ws.data_ptr(), U.data_ptr<double>(), s),
             "gll_forward");
    after_call(st, devi, s);
    if (torch::autograd::compute_requires_grad(X)) {
        auto node = std::shared_ptr<LaplaceBackward>(new LaplaceBackward(),
                                                     torch::autograd::deleteNode);
        node->set_next_edges(torch::autograd::collect_next_edges(X));
        node->X_ = torch::autograd::SavedVariable(X, false);
        node->ws_ = std::move(ws);
        node->p_ = p;
        node->B_ = B;
        node->diag_ = g_grad_diag;
        torch::autograd::set_history(U, node);
    }
    return THPVariable_Wrap(X.is_cuda() ? std::move(U) : U.cpu());
}

PyObject* apply_py(PyObject*, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
    try {
        return apply_impl(args, nargs, kwnames);
    } catch (const PyErrSet&) {
        return nullptr;
    } catch (const c10::Error& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what_without_backtrace());
        return nullptr;
    } catch (const std::exception& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
        return nullptr;
    }
}

PyMethodDef kApplyDef = {
    "apply", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(apply_py)),
    METH_FASTCALL | METH_KEYWORDS,
    "U = LaplaceLearningSparseHard.apply(X, label_matrix, tau=0, epsilon='auto', k=25)\n"
    "(GLL.py:14; k: neighbours incl. self, the reference hard-codes 25)"};

// ------------------------------------------------------------------------------------------
// status API for the Python layer
// ------------------------------------------------------------------------------------------
template <typename F>
void with_py_errors(F f) {
    try {
        f();
    } catch (const PyErrSet&) {
        throw pybind11::error_already_set();
    }
}

}  // namespace

PYBIND11_MODULE(_gll_torch, m) {
    m.doc() = "LaplaceLearningSparseHard.apply over libgll.so (include/gll.h) and its status sink";
    m.add_object("apply", pybind11::reinterpret_steal<pybind11::object>(
                              PyCFunction_NewEx(&kApplyDef, nullptr, m.attr("__name__").ptr())));
    m.def("status_sink", [](int dev) { return int64_t(status_of(dev).sink.data_ptr()); },
          "device address of the sticky status words of device `dev` (gll_problem.status_sink)");
    m.def("note_call", [](int dev) {
              with_py_errors([&] {
                  DeviceStatus& s = status_of(dev);
                  c10::DeviceGuard g(c10::Device(c10::kCUDA, dev));
                  if (!s.order.empty()) poll(s, false);
                  after_call(s, dev, current_stream(dev));
              });
          },
          "count one call that used the sink (Python Function path)");
    m.def("poll_status", [](int dev) {
              with_py_errors([&] {
                  DeviceStatus& s = status_of(dev);
                  if (!s.order.empty()) poll(s, false);
              });
          },
          "raise the warnings of completed status copies of device `dev`");
    m.def("check_status", []() {
              with_py_errors([&] {
                  std::vector<int> devs;
                  {
                      std::lock_guard<std::mutex> lk(g_status_mu);
                      for (int q = 0; q < int(g_status.size()); ++q)
                          if (g_status[q]) devs.push_back(q);
                  }
                  for (int dv : devs) {
                      DeviceStatus& s = status_of(dv);
                      c10::DeviceGuard g(c10::Device(c10::kCUDA, dv));
                      flush(s, dv, current_stream(dv));
                      poll(s, true);
                  }
              });
          },
          "flush every device's status sink now and raise the pending warnings (synchronises)");
    m.def("set_grad_diagnostics", [](double thr) { g_grad_diag = thr; },
          "exploding-gradient report threshold for calls made from now on (< 0: off)");
}
