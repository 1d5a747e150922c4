// torch_ext.cpp -- PyTorch autograd node over the C ABI of include/gll.h.
//
// The reference's LaplaceLearningSparseHard is a Python torch.autograd.Function
// (/root/reference/GLL.py:10-177).  At ~10^4 calls/s its Python forward/backward bodies and
// the GIL hand-off of a Python backward on the autograd thread cost more host time than the
// GPU spends on the whole call, so the node lives here in C++: forward/backward marshal the
// tensors (device, dtype, contiguity), take the workspace from the caching allocator and
// call gll_forward / gll_backward on the current HIP stream.  No numerics here.
// A leading batch dimension (X: B x n x d, label_matrix: B x base x C or shared base x C)
// runs B independent graphs through gll_forward_batched / gll_backward_batched: one launch
// per kernel for all B.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "gll.h"

namespace {

using torch::autograd::AutogradContext;
using torch::autograd::tensor_list;

int dtype_code(at::Tensor& t) {
    switch (t.scalar_type()) {
        case at::kFloat: return GLL_DT_F32;
        case at::kDouble: return GLL_DT_F64;
        case at::kLong: return GLL_DT_I64;
        default: t = t.to(at::kFloat); return GLL_DT_F32;
    }
}

at::Tensor features(const at::Tensor& X, const c10::Device& dev) {
    // the common case (fp32, contiguous, aligned, on the device) needs no new tensor: every
    // dispatcher call here is host time on the step's critical path (~0.5 us each)
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
                         double eps, int64_t max_iter, double rtol, int64_t sink) {
    gll_problem p;
    p.n = int32_t(n);
    p.d = int32_t(d);
    p.base = int32_t(base);
    p.C = int32_t(C);
    p.K = int32_t(std::min<int64_t>(k, n));
    p.max_iter = int32_t(max_iter);
    p.tau = float(tau);
    p.eps = float(eps);
    p.rtol = float(rtol);
    p.flags = 0;
    p.status_sink = reinterpret_cast<int32_t*>(sink);
    return p;
}

class LaplaceLearningFn : public torch::autograd::Function<LaplaceLearningFn> {
   public:
    static at::Tensor forward(AutogradContext* ctx, const at::Tensor& X, const at::Tensor& Y,
                              double tau, double eps, int64_t k, int64_t max_iter, double rtol,
                              int64_t sink) {
        TORCH_CHECK((X.dim() == 2 || X.dim() == 3) && (Y.dim() == 2 || Y.dim() == X.dim()),
                    "X must be n x d (or B x n x d) and label_matrix base x C (or B x base x C)");
        const bool batched = X.dim() == 3;
        const int64_t B = batched ? X.size(0) : 1;
        const c10::Device dev =
            X.is_cuda() ? X.device() : c10::Device(c10::kCUDA, c10::hip::current_device());
        c10::DeviceGuard guard(dev);
        at::Tensor X32 = features(X, dev);
        at::Tensor Yd = Y.device() == dev ? Y : Y.detach().to(dev);
        const int ycode = dtype_code(Yd);
        const int64_t n = X.size(-2), d = X.size(-1), base = Y.size(-2), C = Y.size(-1);
        if (batched && Y.dim() == 2) Yd = Yd.unsqueeze(0).expand({B, base, C});   // shared labels
        TORCH_CHECK(!batched || Yd.size(0) == B, "label_matrix batch ", Yd.size(0), " != ", B);
        if (!Yd.is_contiguous()) Yd = Yd.contiguous();
        gll_problem p = make_problem(n, d, base, C, k, tau, eps, max_iter, rtol, sink);
        const size_t nb = gll_workspace_bytes(&p);
        TORCH_CHECK(nb > 0, "unsupported GLL problem n=", n, " d=", d, " base=", base,
                    " C=", C, " k=", k);
        at::Tensor ws = at::empty({int64_t(nb) * B}, X32.options().dtype(at::kByte));
        at::Tensor U = batched ? at::empty({B, n - base, C}, X32.options().dtype(at::kDouble))
                               : at::empty({n - base, C}, X32.options().dtype(at::kDouble));
        hipStream_t s = c10::hip::getCurrentHIPStream(dev.index()).stream();
        check_rc(gll_forward_batched(&p, int(B), X32.data_ptr<float>(), Yd.data_ptr(), ycode,
                                     ws.data_ptr(), U.data_ptr<double>(), s),
                 "gll_forward");
        ctx->save_for_backward({X});
        ctx->saved_data["ws"] = ws;
        // the scalars as one list (one map entry instead of eight; all exact in a double,
        // the sink address included: 48-bit)
        ctx->saved_data["p"] = std::vector<double>{double(base), double(C), double(k), tau, eps,
                                                   double(max_iter), rtol, double(sink)};
        return X.is_cuda() ? U : U.cpu();
    }

    static tensor_list backward(AutogradContext* ctx, tensor_list grads) {
        const at::Tensor X = ctx->get_saved_variables()[0];
        at::Tensor ws = ctx->saved_data["ws"].toTensor();
        const c10::Device dev = ws.device();
        c10::DeviceGuard guard(dev);
        const int64_t B = X.dim() == 3 ? X.size(0) : 1;
        const auto sv = ctx->saved_data["p"].toDoubleVector();
        gll_problem p = make_problem(X.size(-2), X.size(-1), int64_t(sv[0]), int64_t(sv[1]),
                                     int64_t(sv[2]), sv[3], sv[4], int64_t(sv[5]), sv[6],
                                     int64_t(sv[7]));
        at::Tensor X32 = features(X, dev);
        at::Tensor g = grads[0].device() == dev ? grads[0] : grads[0].to(dev);
        if (g.scalar_type() != at::kFloat && g.scalar_type() != at::kDouble) g = g.to(at::kDouble);
        if (!g.is_contiguous()) g = g.contiguous();
        const int gcode = g.scalar_type() == at::kFloat ? GLL_DT_F32 : GLL_DT_F64;
        at::Tensor gradX = at::empty(X.sizes(), X32.options());
        hipStream_t s = c10::hip::getCurrentHIPStream(dev.index()).stream();
        check_rc(gll_backward_batched(&p, int(B), X32.data_ptr<float>(), ws.data_ptr(),
                                      g.data_ptr(), gcode, gradX.data_ptr<float>(), s),
                 "gll_backward");
        if (gradX.device() != X.device() || gradX.scalar_type() != X.scalar_type())
            gradX = gradX.to(X.device(), X.scalar_type());
        return {gradX, at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(),
                at::Tensor(), at::Tensor()};
    }
};

at::Tensor laplace_learning(const at::Tensor& X, const at::Tensor& Y, double tau, double eps,
                            int64_t k, int64_t max_iter, double rtol, int64_t sink) {
    return LaplaceLearningFn::apply(X, Y, tau, eps, k, max_iter, rtol, sink);
}

}  // namespace

PYBIND11_MODULE(_gll_torch, m) {
    m.doc() = "C++ autograd node of LaplaceLearningSparseHard over libgll.so (include/gll.h)";
    m.def("laplace_learning", &laplace_learning,
          "U = LaplaceLearningSparseHard(X, label_matrix, tau, eps (<=0: auto), k, max_iter, "
          "rtol, status_sink_ptr)");
}
