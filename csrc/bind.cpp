// pybind11 module `_har_native`: host runtime (CSV parser) + kernel launchers.
//
// Launchers take device pointers and the HIP stream as integers (the Python
// side passes `tensor.data_ptr()` and `torch.cuda.current_stream().cuda_stream`),
// so this translation unit needs neither torch nor HIP device headers and the
// kernels stay capturable into hipGraphs.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "har_kernels.h"
#include "host/csv_parser.h"

namespace py = pybind11;
using u = uintptr_t;

template <typename T>
static T* P(u x) { return reinterpret_cast<T*>(x); }
static hipStream_t S(u x) { return reinterpret_cast<hipStream_t>(x); }

static void check(int rc, const char* what) {
  if (rc != 0) {
    std::string msg = std::string(what) + " failed: ";
    if (rc > 0) msg += hipGetErrorString((hipError_t)rc);
    else msg += "contract violation code " + std::to_string(rc);
    throw std::runtime_error(msg);
  }
}

static py::dict csv_parse(py::bytes data, bool header, int threads) {
  std::string_view sv;
  char* ptr;
  Py_ssize_t len;
  PyBytes_AsStringAndSize(data.ptr(), &ptr, &len);
  har::CsvResult r;
  {
    py::gil_scoped_release nogil;
    r = har::parse_csv(ptr, (size_t)len, header, threads);
  }
  py::dict out;
  out["names"] = r.names;
  out["kinds"] = r.kinds;
  py::list dbl, ints, miss, strs;
  for (int j = 0; j < r.ncols; ++j) {
    py::array_t<double> d(r.nrows);
    std::memcpy(d.mutable_data(), r.doubles[j].data(), sizeof(double) * r.nrows);
    py::array_t<int64_t> i(r.nrows);
    std::memcpy(i.mutable_data(), r.ints[j].data(), sizeof(int64_t) * r.nrows);
    py::array_t<bool> m(r.nrows);
    auto* mp = m.mutable_data();
    for (int64_t k = 0; k < r.nrows; ++k) mp[k] = r.missing[j][k] != 0;
    dbl.append(d);
    ints.append(i);
    miss.append(m);
    py::list s;
    if (r.kinds[j] == "string") {
      for (int64_t k = 0; k < r.nrows; ++k) {
        if (r.missing[j][k]) s.append(py::none());
        else s.append(py::str(r.field(j, k)));
      }
    }
    strs.append(s);
  }
  out["doubles"] = dbl;
  out["ints"] = ints;
  out["missing"] = miss;
  out["strings"] = strs;
  out["nrows"] = r.nrows;
  return out;
}

static GemmParams make_gemm(u A, u B, u C, u bias, u mask, u rowsum, int M, int N, int K, int lda, int ldb,
                            int ldc, int ldmask, int k_split, int tile, int64_t slab_stride,
                            int64_t slab_stride_rowsum, float alpha) {
  GemmParams p;
  p.A = P<const void>(A);
  p.B = P<const void>(B);
  p.C = P<void>(C);
  p.bias = P<const float>(bias);
  p.mask = P<const void>(mask);
  p.rowsum = P<float>(rowsum);
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldmask = ldmask;
  p.k_split = k_split;
  p.tile = tile;
  p.slab_stride = slab_stride;
  p.slab_stride_rowsum = slab_stride_rowsum;
  p.alpha = alpha;
  return p;
}

#ifndef HAR_SOURCE_HASH
#define HAR_SOURCE_HASH "unknown"
#endif

static QnArgs qn_args_from_dict(py::dict d) {
  auto I = [&](const char* k) { return d[k].cast<int64_t>(); };
  auto U = [&](const char* k) { return d[k].cast<u>(); };
  QnArgs a;
  a.B = (int)I("B");
  a.T = (int)I("T");
  a.K = (int)I("K");
  a.F = (int)I("F");
  a.m = (int)I("m");
  a.head = (int)I("head");
  a.filled = (int)I("filled");
  a.init = (int)I("init");
  a.nch = (int)I("nch");
  a.fin_it = (int)I("fin_it");
  a.D = I("D");
  a.x = P<float>(U("x"));
  a.g = P<float>(U("g"));
  a.fobj = P<double>(U("fobj"));
  a.l1 = P<const float>(U("l1"));
  a.l2 = P<const float>(U("l2"));
  a.pmask = P<const float>(U("pmask"));
  a.inv_std = P<const float>(U("inv_std"));
  a.S = P<float>(U("S"));
  a.Y = P<float>(U("Y"));
  a.rho = P<double>(U("rho"));
  a.SY = P<double>(U("SY"));
  a.YY = P<double>(U("YY"));
  a.P1 = P<double>(U("P1"));
  a.P2 = P<double>(U("P2"));
  a.P3 = P<double>(U("P3"));
  a.xtrial = P<float>(U("xtrial"));
  a.weff = P<float>(U("weff"));
  a.reg = P<double>(U("reg"));
  a.decr = P<double>(U("decr"));
  a.G = P<const float>(U("G"));
  a.loss = P<const double>(U("loss"));
  a.step_scale = P<float>(U("step_scale"));
  a.active = P<int32_t>(U("active"));
  a.fails = P<int32_t>(U("fails"));
  a.iters = P<int32_t>(U("iters"));
  a.steep = P<int32_t>(U("steep"));
  a.pick = P<int32_t>(U("pick"));
  a.hist = P<double>(U("hist"));
  a.done = P<int32_t>(U("done"));
  a.c1 = d["c1"].cast<double>();
  a.tol = d["tol"].cast<double>();
  return a;
}

// The pointer / shape fields of a solve's L-BFGS arguments, converted from the Python dict ONCE per
// solve; each phase launch then passes only the iteration scalars (a dict conversion per launch cost
// ~20 us of host time, three launches per iteration).
struct QnArgsHolder {
  QnArgs a;
};

// One launch chunk of a LogisticRegression objective evaluation: the evaluate + gradient kernels'
// arguments (pointers fixed for the life of a DeviceLogregSolver).
struct LogregEvalChunk {
  LogregEvalArgs ev;
  LogregGradArgs gr;
  int KP, n_models;
};

// The whole device L-BFGS / OWL-QN solve of a fit as ONE host call (no convergence poll, no
// collective): the same launch sequence as ops/logreg.py DeviceLogregSolver.solve enqueues from
// Python, minus ~60 pybind round trips per fit (the host, not the GPU, bounded a WISDM fit).
struct LogregSolvePlan {
  QnArgs q;
  std::vector<LogregEvalChunk> evT, ev1;  // evaluations of the T trials (first) / 1 per model
  int KP = 8;
  // the persistent solve's barrier counter + timeout flag (2 device words, allocated on first use)
  std::shared_ptr<uint32_t> sync;
  int last_mode = 0;  // 1 = the last solve ran persistent, 0 = as the launch sequence
};

// HAR_LR_PERSISTENT: 0 (default) = the launch sequence, 1 = one cooperative launch when every phase's
// workgroups are co-resident in one round, 2 = one cooperative launch whenever possible.  Measured
// (profiles/r4/lr_persistent.md): the persistent solve is bitwise the sequence but SLOWER on MI355X —
// 1.46 ms vs 1.36 ms of solve kernels for the WISDM fit — back-to-back dependent launches cost less
// than a grid barrier (release fence + counter + acquire fence), so the phases' own latency chains,
// not kernel boundaries, bound an iteration
static int g_lr_persistent = [] {
  const char* e = std::getenv("HAR_LR_PERSISTENT");
  return e ? std::atoi(e) : 0;
}();
static int lr_persistent_mode() { return g_lr_persistent; }

static bool logreg_solve_persistent(LogregSolvePlan& p, int max_iter, hipStream_t s) {
  const int mode = lr_persistent_mode();
  if (mode == 0 || p.evT.size() != 1 || p.ev1.size() != 1) return false;
  if (!p.sync) {
    void* d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(uint32_t)) != hipSuccess) return false;
    p.sync = std::shared_ptr<uint32_t>(static_cast<uint32_t*>(d), [](uint32_t* q) { (void)hipFree(q); });
  }
  const LogregEvalChunk &cT = p.evT[0], &c1 = p.ev1[0];
  // mode 1: only when the widest phase fits one co-resident round (max_grid = 0: the launcher caps
  // the grid at the co-resident count; a wider phase then loops, which the batched CV fits lose on)
  const int rc = har_logreg_solve_persistent(&p.q, &cT.ev, &cT.gr, cT.n_models, &c1.ev, &c1.gr, c1.n_models, p.KP,
                                             max_iter, p.sync.get(), mode == 1 ? -1 : 0, s);
  if (rc == -2) throw std::runtime_error("logreg_solve_persistent: invalid arguments");
  return rc == 0;
}

// last_mode: 1 = the persistent solve ran and completed, 2 = it ran but a grid barrier timed out
// (sync[1] set: blocks went on with unsynchronized x / g / history, so the results are garbage and
// the caller must rerun the fit as the launch sequence — ops/logreg.py does), 0 = the sequence ran
static void logreg_solve_run(LogregSolvePlan& p, int max_iter, int m, hipStream_t s) {
  if (logreg_solve_persistent(p, max_iter, s)) {
    uint32_t flag = 0;  // one blocking 4-byte read: only the opt-in persistent mode pays it
    check(hipMemcpyAsync(&flag, p.sync.get() + 1, sizeof flag, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess
              ? 0 : -1,
          "logreg_solve flag read");
    p.last_mode = flag ? 2 : 1;
    return;
  }
  p.last_mode = 0;
  auto phase = [&](int ph, int head, int filled, int init, int fin_it) {
    QnArgs a = p.q;
    a.head = head;
    a.filled = filled;
    a.init = init;
    a.fin_it = fin_it;
    check(har_lbfgs_phase(&a, p.KP, ph, s), "lbfgs_phase");
  };
  auto evaluate = [&](const std::vector<LogregEvalChunk>& v) {
    for (const auto& c : v) {
      check(har_logreg_eval(&c.ev, c.KP, c.n_models, s), "logreg_eval");
      check(har_logreg_grad(&c.gr, c.KP, c.n_models, s), "logreg_grad");
    }
  };
  phase(1, 0, 0, 1, 0);
  evaluate(p.evT);
  phase(2, 0, 0, 1, 0);
  int head = 0, filled = 0;
  for (int it = 0; it < max_iter; ++it) {
    phase(1, head, filled, 0, 0);
    evaluate(p.ev1);
    phase(2, head, filled, 0, it + 1);
    head = (head + 1) % m;
    filled = filled + 1 < m ? filled + 1 : m;
  }
}

// The flagship MLP training step as ONE host call: the buffers of an engine never move, so their
// pointers, the gradient-reduction regions and the Adam hyper-parameters are fixed once per (engine,
// batch size) and run() enqueues mlp_step_fwd -> mlp_step_bwd -> grad_reduce_adam with only the batch
// pointers changing (three pybind calls with ~20 arguments each and a region list rebuilt in Python
// every step were ~10 us of host time per 70 us step: enough to starve the GPU when not graph-captured).
struct MlpStepPlan {
  u Wf, b0, b1, Wo, bo, dact2, fslab, bloss, bcorr, gw1, gw0, gb0, gb1, step, G, Pw, m, v, Pb;
  int K0, H, C, fslab_w;
  MlpFragSpec frag;
  u gwo, gbo;
  int64_t stride, n;
  float lr, b1c, b2c, eps, wd;
  std::vector<const float*> src;
  std::vector<int64_t> start, len, lds;
  std::vector<int> S;
  u pf_sink = 0;  // 4-byte scratch word of the prefetch workgroups (set once by the engine)
  // mode: 1 reduce + Adam (N = 1), 2 reduce + store G (DP, before the all-reduce), 4 Adam from G;
  // pf / pf_bytes (and pf1 / pf1_bytes): the next step's input rows (and labels), read by the reduction
  // launch's prefetch workgroups
  void run(u X, u y, int B, float scale, int mode, u stream, u pf, int64_t pf_bytes, u pf1, int64_t pf1_bytes) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (mode & 3) {
      check(har_mlp_step_fwd(P<const uint16_t>(X), K0, P<uint16_t>(Wf), P<const float>(b0), P<const float>(b1), H,
                             P<const uint16_t>(Wo), P<const float>(bo), P<const int32_t>(y), B, C, scale,
                             P<uint16_t>(dact2), P<float>(fslab), P<float>(bloss), P<int32_t>(bcorr), s),
            "mlp_step_fwd");
      check(har_mlp_step_bwd(P<const uint16_t>(dact2), P<const uint16_t>(X), K0, P<const uint16_t>(Wf), H,
                             P<const float>(b0), B, P<float>(gw1), P<float>(gw0), P<float>(gb0), P<float>(gb1),
                             stride, P<int32_t>(step), P<const float>(fslab), fslab_w, P<float>(gwo), P<float>(gbo), s),
            "mlp_step_bwd");
    }
    const int gm = mode == 1 ? 1 | 4 : mode == 2 ? 1 | 2 : 4;  // GR_REDUCE 1, GR_STORE 2, GR_ADAM 4
    const int k = (gm & 1) ? (int)src.size() : 0;
    check(har_grad_reduce_adam(k, src.data(), start.data(), len.data(), lds.data(), S.data(), n, P<float>(G),
                               P<float>(Pw), P<float>(m), P<float>(v), P<uint16_t>(Pb), lr, b1c, b2c, eps, wd,
                               P<int32_t>(step), 0, gm, &frag, s, pf && pf_sink ? P<const void>(pf) : nullptr,
                               pf_bytes, P<uint32_t>(pf_sink), P<const void>(pf1), pf1_bytes),
          "grad_reduce_adam");
  }
};

PYBIND11_MODULE(_har_native, m) {
  m.doc() = "har native runtime: host CSV parser + gfx950 HIP kernel launchers";
  // content hash of every source / header / flag the library was built from (tools/build_native.py);
  // ops/_native.py refuses a library whose hash differs from the tree it is imported from
  m.def("source_hash", []() { return std::string(HAR_SOURCE_HASH); });
  m.def("csv_parse", &csv_parse, py::arg("data"), py::arg("header") = true, py::arg("threads") = 0);

  m.def("gemm", [](bool bf16, int layout, int epi, u A, u B, u C, u bias, u mask, u rowsum, int M, int N, int K,
                   int lda, int ldb, int ldc, int ldmask, int k_split, int tile, int64_t slab_stride,
                   int64_t slab_stride_rowsum, float alpha, u stream) {
    GemmParams p = make_gemm(A, B, C, bias, mask, rowsum, M, N, K, lda, ldb, ldc, ldmask, k_split, tile, slab_stride,
                             slab_stride_rowsum, alpha);
    check(bf16 ? har_gemm_bf16(&p, layout, epi, S(stream)) : har_gemm_f32(&p, layout, epi, S(stream)), "gemm");
  });

  m.def("softmax_ce_head_blocks", &har_softmax_ce_head_blocks);
  m.def("softmax_ce_head", [](u H, u W, u bias, u labels, int B, int D, int C, float scale, u dlogits,
                              u block_loss, u block_correct, u logits_out, u stream) {
    check(har_softmax_ce_head(P<const uint16_t>(H), P<const uint16_t>(W), P<const float>(bias),
                              P<const int32_t>(labels), B, D, C, scale, P<uint16_t>(dlogits), P<float>(block_loss),
                              P<int32_t>(block_correct), P<float>(logits_out), S(stream)),
          "softmax_ce_head");
  });

  m.def("adam_step", [](u param, u grad, u slabs, int nslabs, u mm, u vv, u pb, int64_t n, float lr, float b1,
                        float b2, float eps, float wd, float gs, u step, u stream, int tick) {
    check(har_adam_step(P<float>(param), P<const float>(grad), P<const float>(slabs), nslabs, P<float>(mm),
                        P<float>(vv), P<uint16_t>(pb), n, lr, b1, b2, eps, wd, gs, P<int32_t>(step), tick, S(stream)),
          "adam_step");
  });

  m.def("reduce_slabs", [](u slabs, int nslabs, int64_t n, u dst, u stream) {
    check(har_reduce_slabs(P<const float>(slabs), nslabs, n, P<float>(dst), S(stream)), "reduce_slabs");
  });

  m.def("logreg_eval_tiles", &har_logreg_eval_tiles);
  m.def("logreg_eval", [](u dense, int64_t ldd, int Fd, u dense_cols, u cat, int C, u y, u rw, u inv_wsum, u W,
                          int64_t N, int F, int K, int T, int tstride, int model0, int mode, u R, u slab, int KP,
                          int n_models,
                          u stream) {
    LogregEvalArgs a;
    a.dense = P<const float>(dense);
    a.ldd = ldd;
    a.Fd = Fd;
    a.dense_cols = P<const int32_t>(dense_cols);
    a.cat = P<const int32_t>(cat);
    a.C = C;
    a.y = P<const int32_t>(y);
    a.rw = P<const float>(rw);
    a.inv_wsum = P<const float>(inv_wsum);
    a.W = P<const float>(W);
    a.N = N;
    a.F = F;
    a.K = K;
    a.T = T;
    a.tstride = tstride;
    a.model0 = model0;
    a.mode = mode;
    a.R = P<float>(R);
    a.slab = P<float>(slab);
    check(har_logreg_eval(&a, KP, n_models, S(stream)), "logreg_eval");
  });
  // argument holders for logreg_solve_plan: the same positional arguments as logreg_eval /
  // logreg_grad below, without the stream
  py::class_<LogregEvalChunk>(m, "LogregEvalChunk");
  m.def("logreg_eval_chunk", [](py::tuple e, py::tuple g) {
    LogregEvalChunk c{};
    auto U = [](py::handle h) { return h.cast<u>(); };
    auto I = [](py::handle h) { return h.cast<int64_t>(); };
    c.ev.dense = P<const float>(U(e[0]));
    c.ev.ldd = I(e[1]);
    c.ev.Fd = (int)I(e[2]);
    c.ev.dense_cols = P<const int32_t>(U(e[3]));
    c.ev.cat = P<const int32_t>(U(e[4]));
    c.ev.C = (int)I(e[5]);
    c.ev.y = P<const int32_t>(U(e[6]));
    c.ev.rw = P<const float>(U(e[7]));
    c.ev.inv_wsum = P<const float>(U(e[8]));
    c.ev.W = P<const float>(U(e[9]));
    c.ev.N = I(e[10]);
    c.ev.F = (int)I(e[11]);
    c.ev.K = (int)I(e[12]);
    c.ev.T = (int)I(e[13]);
    c.ev.tstride = (int)I(e[14]);
    c.ev.model0 = (int)I(e[15]);
    c.ev.mode = (int)I(e[16]);
    c.ev.R = P<float>(U(e[17]));
    c.ev.slab = P<float>(U(e[18]));
    c.KP = (int)I(e[19]);
    c.n_models = (int)I(e[20]);
    c.gr.slab = P<const float>(U(g[0]));
    c.gr.R = P<const float>(U(g[1]));
    c.gr.col_map = P<const int32_t>(U(g[2]));
    c.gr.csc_rows = P<const int32_t>(U(g[3]));
    c.gr.csc_off = P<const int32_t>(U(g[4]));
    c.gr.col_slice = P<const int32_t>(U(g[5]));
    c.gr.SL = (int)I(g[6]);
    c.gr.inv_std = P<const float>(U(g[7]));
    c.gr.pmask = P<const float>(U(g[8]));
    c.gr.N = I(g[9]);
    c.gr.F = (int)I(g[10]);
    c.gr.Fd = (int)I(g[11]);
    c.gr.K = (int)I(g[12]);
    c.gr.T = (int)I(g[13]);
    c.gr.tstride = (int)I(g[14]);
    c.gr.model0 = (int)I(g[15]);
    c.gr.ntiles = (int)I(g[16]);
    c.gr.G = P<float>(U(g[17]));
    c.gr.loss = P<double>(U(g[18]));
    c.gr.loss_fx = P<float>(U(g[19]));
    if ((int)I(g[20]) != c.KP || (int)I(g[21]) != c.n_models) throw std::runtime_error("logreg_eval_chunk: KP / n mismatch");
    c.gr.col_blk = P<const int32_t>(U(g[22]));
    c.gr.nblk = (int)I(g[23]);
    c.gr.srow = P<const int32_t>(U(g[24]));
    return c;
  });
  py::class_<LogregSolvePlan>(m, "LogregSolvePlan");
  m.def("logreg_solve_plan", [](const QnArgsHolder& h, std::vector<LogregEvalChunk> evT,
                                std::vector<LogregEvalChunk> ev1, int KP) {
    LogregSolvePlan p;
    p.q = h.a;
    p.evT = std::move(evT);
    p.ev1 = std::move(ev1);
    p.KP = KP;
    return p;
  });
  m.def("logreg_solve", [](LogregSolvePlan& p, int max_iter, int m, u stream) {
    logreg_solve_run(p, max_iter, m, S(stream));
    return p.last_mode;
  });
  m.def("logreg_set_persistent", [](int mode) {
    const int old = g_lr_persistent;
    g_lr_persistent = mode;
    return old;
  });
  m.def("logreg_set_spin_limit", [](uint32_t n) { return har_logreg_set_spin_limit(n); });
  m.def("lr_set_stamps", [](uint64_t ev, uint64_t dir, uint64_t upd, uint64_t grd) {
    har_lr_set_stamps(reinterpret_cast<uint64_t*>(ev), reinterpret_cast<uint64_t*>(dir), reinterpret_cast<uint64_t*>(upd),
                      reinterpret_cast<uint64_t*>(grd));
  });
  // the persistent solve's timeout flag (blocking 4-byte read; tests / diagnostics)
  m.def("logreg_solve_flag", [](const LogregSolvePlan& p) {
    uint32_t f = 0;
    if (p.sync) check(hipMemcpy(&f, p.sync.get() + 1, sizeof f, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1,
                      "logreg_solve_flag");
    return (int)f;
  });
  m.def("logreg_grad", [](u slab, u R, u col_map, u csc_rows, u csc_off, u col_slice, int SL, u inv_std, u pmask,
                          int64_t N, int F, int Fd, int K, int T, int tstride, int model0, int ntiles, u G, u loss,
                          u loss_fx, int KP, int n_models, u col_blk, int nblk, u srow, u stream) {
    LogregGradArgs a;
    a.col_blk = P<const int32_t>(col_blk);
    a.nblk = nblk;
    a.srow = P<const int32_t>(srow);
    a.slab = P<const float>(slab);
    a.R = P<const float>(R);
    a.col_map = P<const int32_t>(col_map);
    a.csc_rows = P<const int32_t>(csc_rows);
    a.csc_off = P<const int32_t>(csc_off);
    a.col_slice = P<const int32_t>(col_slice);
    a.SL = SL;
    a.inv_std = P<const float>(inv_std);
    a.pmask = P<const float>(pmask);
    a.N = N;
    a.F = F;
    a.Fd = Fd;
    a.K = K;
    a.T = T;
    a.tstride = tstride;
    a.model0 = model0;
    a.ntiles = ntiles;
    a.G = P<float>(G);
    a.loss = P<double>(loss);
    a.loss_fx = P<float>(loss_fx);
    check(har_logreg_grad(&a, KP, n_models, S(stream)), "logreg_grad");
  });
  m.def("logreg_col_slices", [](u csc_off, int F, int SL, u col_slice, u stream) {
    check(har_logreg_col_slices(P<const int32_t>(csc_off), F, SL, P<int32_t>(col_slice), S(stream)),
          "logreg_col_slices");
  });
  m.def("logreg_summary_tiles", &har_logreg_summary_tiles);
  m.def("logreg_summary", [](int phase, u dense, int64_t ldd, int Fd, u y, u rw, int64_t N, int F, int K, int nspec,
                             u col_map, u csc_rows, u csc_off, u col_slice, int SL, int ntiles, u part, u summ,
                             u srow, u stream) {
    LogregSummaryArgs a;
    a.srow = P<const int32_t>(srow);
    a.dense = P<const float>(dense);
    a.ldd = ldd;
    a.Fd = Fd;
    a.y = P<const int32_t>(y);
    a.rw = P<const float>(rw);
    a.N = N;
    a.F = F;
    a.K = K;
    a.S = nspec;
    a.col_map = P<const int32_t>(col_map);
    a.csc_rows = P<const int32_t>(csc_rows);
    a.csc_off = P<const int32_t>(csc_off);
    a.col_slice = P<const int32_t>(col_slice);
    a.SL = SL;
    a.ntiles = ntiles;
    a.part = P<double>(part);
    a.summ = P<double>(summ);
    check(har_logreg_summary(&a, phase, S(stream)), "logreg_summary");
  });
  m.def("logreg_prepare", [](u summ, u reg, u alpha, int B, int F, int K, int Kp, int standardization,
                             int fit_intercept, int binomial, u inv_std, u inv_wsum, u pmask, u l2, u l1, u x0,
                             u stream) {
    LogregPrepareArgs a;
    a.summ = P<const double>(summ);
    a.reg = P<const float>(reg);
    a.alpha = P<const float>(alpha);
    a.B = B;
    a.F = F;
    a.K = K;
    a.Kp = Kp;
    a.standardization = standardization;
    a.fit_intercept = fit_intercept;
    a.binomial = binomial;
    a.inv_std = P<float>(inv_std);
    a.inv_wsum = P<float>(inv_wsum);
    a.pmask = P<float>(pmask);
    a.l2 = P<float>(l2);
    a.l1 = P<float>(l1);
    a.x0 = P<float>(x0);
    check(har_logreg_prepare(&a, S(stream)), "logreg_prepare");
  });
  m.def("logreg_loss_decode", [](u fx, u loss, int n, u stream) {
    check(har_logreg_loss_decode(P<const float>(fx), P<double>(loss), n, S(stream)), "logreg_loss_decode");
  });
  // one L-BFGS phase (logreg_qn.hip: 1 direction + trials, 2 pick + history + the next direction's
  // dots, finalized by the model's last chunk); the QnArgs fields come from a dict of ints / floats /
  // device pointers
  m.def("qn_chunks", &har_qn_chunks);
  m.def("lbfgs_phase", [](int phase, py::dict d, int KP, u stream) {
    QnArgs a = qn_args_from_dict(d);
    check(har_lbfgs_phase(&a, KP, phase, S(stream)), "lbfgs_phase");
  });
  py::class_<QnArgsHolder>(m, "QnArgs");
  m.def("qn_args", [](py::dict d) { return QnArgsHolder{qn_args_from_dict(d)}; });
  m.def("lbfgs_phase_h", [](const QnArgsHolder& h, int phase, int head, int filled, int init, int fin_it, int KP,
                            u stream) {
    QnArgs a = h.a;
    a.head = head;
    a.filled = filled;
    a.init = init;
    a.fin_it = fin_it;
    check(har_lbfgs_phase(&a, KP, phase, S(stream)), "lbfgs_phase");
  });

  m.def("value_counts", [](u codes, int64_t n, int V, u out, u stream) {
    check(har_value_counts(P<const int64_t>(codes), n, V, P<int64_t>(out), S(stream)), "value_counts");
  });
  m.def("confusion_matrix", [](u label, u pred, int64_t n, int K, u cm, u stream) {
    check(har_confusion_matrix(P<const int32_t>(label), P<const int32_t>(pred), n, K, P<int64_t>(cm), S(stream)),
          "confusion_matrix");
  });

  m.def("regression_moments", [](u y, u yh, int64_t n, u out, u stream) {
    check(har_regression_moments(P<const float>(y), P<const float>(yh), n, P<double>(out), S(stream)),
          "regression_moments");
  });

  m.def("tree_dp_pack", [](u store, int A, int64_t slot, int mb, int K, u cls, u kp, u bw, u woff, u out, u stream) {
    check(har_tree_dp_pack(P<const float>(store), A, slot, mb, K, P<const int32_t>(cls), P<const int32_t>(kp),
                           P<const int32_t>(bw), P<const int64_t>(woff), P<int32_t>(out), S(stream)),
          "tree_dp_pack");
  });
  m.def("tree_dp_unpack", [](u in, int a0, int n, int64_t slot, int mb, int K, u cls, u kp, u bw, u woff,
                             int64_t base, u local, u stream) {
    check(har_tree_dp_unpack(P<const int32_t>(in), a0, n, slot, mb, K, P<const int32_t>(cls), P<const int32_t>(kp),
                             P<const int32_t>(bw), P<const int64_t>(woff), base, P<float>(local), S(stream)),
          "tree_dp_unpack");
  });
  m.def("confusion_matrix_batched", [](u label, u pred, u mask, int64_t n, int B, int K, u cm, u stream) {
    check(har_confusion_matrix_batched(P<const int32_t>(label), P<const int32_t>(pred), P<const uint8_t>(mask), n, B,
                                       K, P<int64_t>(cm), S(stream)),
          "confusion_matrix_batched");
  });
  m.def("roc_pr_sums_batched", [](u s, u y, u ns, int B, int64_t ld, u out, u stream) {
    check(har_roc_pr_sums_batched(P<const float>(s), P<const float>(y), P<const int32_t>(ns), B, ld, P<double>(out),
                                  S(stream)),
          "roc_pr_sums_batched");
  });
  m.def("roc_pr_sums", [](u s, u y, int64_t n, u out, u stream) {
    check(har_roc_pr_sums(P<const float>(s), P<const float>(y), n, P<double>(out), S(stream)), "roc_pr_sums");
  });

  m.def("tree_hist_split", [](u bins, int64_t N, int F, int row_major, u nbins, u rows, u row_w, u node_start, u node_count, int A,
                              u feats, int m, int fc, u label, int K, int maxbins, float min_inst, float min_gain,
                              int impurity, u gain, u feat, u bin, u left, u total, int mode, u ghist, int row_chunks,
                              u cat, int ncat, u onehot, u stream) {
    const TreeSparse sp{P<const int32_t>(cat), ncat, P<const uint8_t>(onehot), F};
    check(har_tree_hist_split(P<const uint8_t>(bins), N, F, row_major, P<const int32_t>(nbins), P<const int32_t>(rows),
                              P<const float>(row_w), P<const int32_t>(node_start), P<const int32_t>(node_count), A,
                              P<const int32_t>(feats), m, fc, P<const int32_t>(label), K, maxbins, min_inst, min_gain,
                              impurity, P<float>(gain), P<int32_t>(feat), P<int32_t>(bin), P<float>(left),
                              P<float>(total), mode, P<float>(ghist), row_chunks, cat ? &sp : nullptr, S(stream)),
          "tree_hist_split");
  });

  m.def("tree_plan", [](u counts, int A, int prows, u plan, int64_t slot_elems, u ghist, int max_big, int by_node,
                        u a_dev, u stream) {
    check(har_tree_plan(P<const int32_t>(counts), A, prows, P<int32_t>(plan), slot_elems, P<float>(ghist), max_big,
                        by_node, P<const int32_t>(a_dev), S(stream)),
          "tree_plan");
  });
  m.def("tree_hist_split_planned", [](u bins, int64_t N, int F, int row_major, u nbins, u rows, u row_w, u node_start,
                                      u node_count, int A, u feats, int m, int fc, u label, int K, int maxbins,
                                      float min_inst, float min_gain, int impurity, u gain, u feat, u bin, u left,
                                      u total, int mode, u ghist, u plan, int prows, int bound, int by_node,
                                      u hprev, u derive_from, u parent_of, u cat, int ncat, u onehot, u stream) {
    const TreeSparse sp{P<const int32_t>(cat), ncat, P<const uint8_t>(onehot), F};
    check(har_tree_hist_split_planned(P<const uint8_t>(bins), N, F, row_major, P<const int32_t>(nbins),
                                      P<const int32_t>(rows), P<const float>(row_w), P<const int32_t>(node_start),
                                      P<const int32_t>(node_count), A, P<const int32_t>(feats), m, fc,
                                      P<const int32_t>(label), K, maxbins, min_inst, min_gain, impurity,
                                      P<float>(gain), P<int32_t>(feat), P<int32_t>(bin), P<float>(left),
                                      P<float>(total), mode, P<float>(ghist), 1, P<const int32_t>(plan), prows, bound,
                                      by_node, P<const float>(hprev), P<const int32_t>(derive_from),
                                      P<const int32_t>(parent_of), cat ? &sp : nullptr, S(stream)),
          "tree_hist_split_planned");
  });

  m.def("forest_predict", [](u X, int64_t n, int F, int ld, u feat, u thr, u left, u right, u leaf, int T, int maxn,
                             int K, int max_depth, int normalize, u out, u stream) {
    check(har_forest_predict(P<const float>(X), n, F, ld, P<const int32_t>(feat), P<const float>(thr),
                             P<const int32_t>(left), P<const int32_t>(right), P<const float>(leaf), T, maxn, K,
                             max_depth, normalize, P<float>(out), S(stream)),
          "forest_predict");
  });

  m.def("tree_init", [](uint64_t seed, int tree0, int ntrees, int64_t row0, int64_t n, std::vector<uint32_t> cdf,
                        u rw, u y, int K, u W, u node_of, u stats, int64_t stride, u bad, u stream) {
    check(har_tree_init(seed, tree0, ntrees, row0, n, cdf.data(), (int)cdf.size(), P<const float>(rw),
                        P<const int32_t>(y), K, P<float>(W), P<int32_t>(node_of), P<float>(stats), stride,
                        P<int32_t>(bad), S(stream)),
          "tree_init");
  });
  m.def("sort_columns", [](u X, int n, int F, int ld, u out, u stream) {
    check(har_sort_columns(P<const float>(X), n, F, ld, P<float>(out), S(stream)), "sort_columns");
  });
  m.def("find_splits_post_sort", [](u sorted, int F, int n, int ns, u out, u stream) {
    check(har_find_splits_post_sort(P<const float>(sorted), F, n, ns, P<float>(out), S(stream)),
          "find_splits_post_sort");
  });
  m.def("poisson_bootstrap", [](uint64_t seed, int tree0, int ntrees, int64_t row0, int64_t n, u out, u stream) {
    check(har_poisson_bootstrap(seed, tree0, ntrees, row0, n, P<uint8_t>(out), S(stream)), "poisson_bootstrap");
  });

  m.def("philox_buckets", [](uint64_t seed, uint32_t stream_id, int64_t row0, int64_t n, u thr, int nthr, u out,
                             u stream) {
    check(har_philox_buckets(seed, stream_id, row0, n, P<const uint32_t>(thr), nthr, P<int32_t>(out), S(stream)),
          "philox_buckets");
  });

  m.def("window_features_mlp", [](u stream, int64_t n_samples, int axes, int window, int stride, int64_t n_windows,
                                  float hz, u mean, u inv_std, float nan_value, u out, int ld_out, u stream_) {
    check(har_window_features_mlp(P<const float>(stream), n_samples, axes, window, stride, n_windows, hz,
                                  P<const float>(mean), P<const float>(inv_std), nan_value, P<uint16_t>(out), ld_out,
                                  S(stream_)),
          "window_features_mlp");
  });
  m.def("window_set_legacy", [](int on) { har_window_set_legacy(on); });
  m.def("window_features", [](u stream, int64_t n_samples, int axes, int window, int stride, int64_t n_windows,
                              float hz, int nbins, u out, int ld_out, u st) {
    check(har_window_features(P<const float>(stream), n_samples, axes, window, stride, n_windows, hz, nbins,
                              P<float>(out), ld_out, S(st)),
          "window_features");
  });

  m.def("grad_reduce_adam", [](std::vector<u> src, std::vector<int64_t> start, std::vector<int64_t> len,
                               std::vector<int64_t> lds, std::vector<int> nsl, int64_t n, u G, u param, u mm, u vv,
                               u pb, float lr, float b1, float b2, float eps, float wd, u step, int tick, int mode,
                               u stream, u frag_dst, int64_t w0_off, int64_t w1_off, int fK0, int fH, int fw1t) {
    const MlpFragSpec frag{P<uint16_t>(frag_dst), w0_off, w1_off, fK0, fH, fw1t};
    const int k = (int)src.size();
    if ((int)start.size() != k || (int)len.size() != k || (int)lds.size() != k || (int)nsl.size() != k)
      throw std::runtime_error("grad_reduce_adam: region lists differ in length");
    std::vector<const float*> sp(k);
    for (int i = 0; i < k; ++i) sp[i] = P<const float>(src[i]);
    check(har_grad_reduce_adam(k, sp.data(), start.data(), len.data(), lds.data(), nsl.data(), n, P<float>(G),
                               P<float>(param), P<float>(mm), P<float>(vv), P<uint16_t>(pb), lr, b1, b2, eps, wd,
                               P<int32_t>(step), tick, mode, frag_dst ? &frag : nullptr, S(stream)),
          "grad_reduce_adam");
  }, py::arg("src"), py::arg("start"), py::arg("len"), py::arg("lds"), py::arg("nsl"), py::arg("n"), py::arg("G"),
     py::arg("param"), py::arg("m"), py::arg("v"), py::arg("pb"), py::arg("lr"), py::arg("b1"), py::arg("b2"),
     py::arg("eps"), py::arg("wd"), py::arg("step"), py::arg("tick"), py::arg("mode"), py::arg("stream"),
     py::arg("frag_dst") = 0, py::arg("w0_off") = 0, py::arg("w1_off") = 0, py::arg("fK0") = 0, py::arg("fH") = 0,
     py::arg("fw1t") = 0);
  // small-batch step: the fused tile kernel, then ONE region reduction of its B / 32 slabs + Adam that
  // refreshes Pb and all three fragment copies (mlp_small.hip)
  m.def("mlp_small_step_max_batch", &har_mlp_small_step_max_batch);
  m.def("mlp_small_step", [](u X, int K0, u Wf, u b0, u b1, int H, u Wo, u bo, u labels, int B, int C, float scale,
                             u slab, int64_t total, int64_t off_w0, int64_t off_b0, int64_t off_w1, int64_t off_b1,
                             int64_t off_wo, int64_t off_bo, u block_loss, u block_correct, u tick, u G, u param,
                             u mm, u vv, u pb, float lr, float b1c, float b2c, float eps, float wd, u step,
                             u stream) {
    const MlpSmallStepArgs a{P<const uint16_t>(X), P<const uint16_t>(Wf), P<const float>(b0), P<const float>(b1),
                             P<const uint16_t>(Wo), P<const float>(bo), P<const int32_t>(labels), B, C, scale,
                             P<float>(slab), total, off_w0, off_b0, off_w1, off_b1, off_wo, off_bo,
                             P<float>(block_loss), P<int32_t>(block_correct), P<int32_t>(tick)};
    check(har_mlp_small_step(&a, K0, H, S(stream)), "mlp_small_step");
    const float* src = P<const float>(slab);
    const int64_t start = 0;
    const int nsl = B / 32;
    const MlpFragSpec frag{P<uint16_t>(Wf), off_w0, off_w1, K0, H, 1};
    check(har_grad_reduce_adam(1, &src, &start, &total, &total, &nsl, total, P<float>(G), P<float>(param),
                               P<float>(mm), P<float>(vv), P<uint16_t>(pb), lr, b1c, b2c, eps, wd, P<int32_t>(step),
                               0, 1 | 4, &frag, S(stream)),
          "mlp_small_step reduce+adam");
  });
  m.def("mlp_pack_frag", [](u pb, u dst, int64_t w0_off, int64_t w1_off, int K0, int H, u stream) {
    const MlpFragSpec f{P<uint16_t>(dst), w0_off, w1_off, K0, H};
    check(har_mlp_pack_frag(P<const uint16_t>(pb), &f, S(stream)), "mlp_pack_frag");
  });
  m.def("reduce_slabs_multi", [](std::vector<u> slabs, std::vector<int> nsl, std::vector<int64_t> n,
                                 std::vector<int64_t> lds, std::vector<u> dst, std::vector<int64_t> ldd, int G,
                                 u tick, u stream) {
    const int k = (int)slabs.size();
    if ((int)nsl.size() != k || (int)n.size() != k || (int)lds.size() != k || (int)dst.size() != k ||
        (int)ldd.size() != k)
      throw std::runtime_error("reduce_slabs_multi: segment lists differ in length");
    std::vector<const float*> sp(k);
    std::vector<float*> dp(k);
    for (int i = 0; i < k; ++i) { sp[i] = P<const float>(slabs[i]); dp[i] = P<float>(dst[i]); }
    check(har_reduce_slabs_multi(k, sp.data(), nsl.data(), n.data(), lds.data(), dp.data(), ldd.data(), G,
                                 P<int32_t>(tick), S(stream)),
          "reduce_slabs_multi");
  });
  m.def("head_fused_blocks", &har_head_fused_blocks);
  m.def("mlp_fwd_head_grid", &har_mlp_fwd_head_grid);
  m.def("mlp_set_stamps", [](u p) { har_mlp_set_stamps(P<uint64_t>(p)); });
  py::class_<MlpStepPlan>(m, "MlpStepPlan")
      .def(py::init([](py::dict d) {
        MlpStepPlan p;
        for (const char* k : {"Wf", "b0", "b1", "Wo", "bo", "dact2", "fslab", "bloss", "bcorr", "gw1", "gw0",
                              "gb0", "gb1", "step", "G", "P", "m", "v", "Pb"}) {
          const u x = d[k].cast<u>();
          if (!strcmp(k, "Wf")) p.Wf = x; else if (!strcmp(k, "b0")) p.b0 = x;
          else if (!strcmp(k, "b1")) p.b1 = x; else if (!strcmp(k, "Wo")) p.Wo = x; else if (!strcmp(k, "bo")) p.bo = x;
          else if (!strcmp(k, "dact2")) p.dact2 = x;
          else if (!strcmp(k, "fslab")) p.fslab = x; else if (!strcmp(k, "bloss")) p.bloss = x;
          else if (!strcmp(k, "bcorr")) p.bcorr = x; else if (!strcmp(k, "gw1")) p.gw1 = x;
          else if (!strcmp(k, "gw0")) p.gw0 = x; else if (!strcmp(k, "gb0")) p.gb0 = x; else if (!strcmp(k, "gb1")) p.gb1 = x;
          else if (!strcmp(k, "step")) p.step = x; else if (!strcmp(k, "G")) p.G = x; else if (!strcmp(k, "P")) p.Pw = x;
          else if (!strcmp(k, "m")) p.m = x; else if (!strcmp(k, "v")) p.v = x; else p.Pb = x;
        }
        p.K0 = d["K0"].cast<int>();
        p.fslab_w = d["fslab_w"].cast<int>();
        p.gwo = d["gwo"].cast<u>();
        p.gbo = d["gbo"].cast<u>();
        p.H = d["H"].cast<int>();
        p.C = d["C"].cast<int>();
        p.stride = d["stride"].cast<int64_t>();
        p.n = d["n"].cast<int64_t>();
        p.lr = d["lr"].cast<float>();
        p.b1c = d["beta1"].cast<float>();
        p.b2c = d["beta2"].cast<float>();
        p.eps = d["eps"].cast<float>();
        p.wd = d["wd"].cast<float>();
        p.frag = MlpFragSpec{P<uint16_t>(p.Wf), d["w0_off"].cast<int64_t>(), d["w1_off"].cast<int64_t>(), p.K0, p.H};
        for (auto r : d["regions"].cast<py::list>()) {  // (start, end, src pointer, #slabs, slab stride)
          auto t = r.cast<py::tuple>();
          const int64_t a = t[0].cast<int64_t>(), e = t[1].cast<int64_t>();
          p.start.push_back(a);
          p.len.push_back(e - a);
          p.src.push_back(P<const float>(t[2].cast<u>()));
          p.S.push_back(t[3].cast<int>());
          p.lds.push_back(t[4].cast<int64_t>());
        }
        return p;
      }))
      .def("run", &MlpStepPlan::run, py::arg("X"), py::arg("y"), py::arg("B"), py::arg("scale"), py::arg("mode"),
           py::arg("stream"), py::arg("pf") = 0, py::arg("pf_bytes") = 0, py::arg("pf1") = 0, py::arg("pf1_bytes") = 0)
      .def_readwrite("pf_sink", &MlpStepPlan::pf_sink);
  m.def("mlp_step_grid", &har_mlp_step_grid);
  m.def("mlp_step_slices", &har_mlp_step_slices);
  m.def("mlp_step_fwd_slab_width", &har_mlp_step_fwd_slab_width);
  m.def("mlp_step_fwd", [](u X, int K0, u Wf, u b0, u b1, int H, u Wo, u bo, u labels, int B, int C, float scale,
                           u dact2, u slab, u block_loss, u block_correct, u stream) {
    check(har_mlp_step_fwd(P<const uint16_t>(X), K0, P<uint16_t>(Wf), P<const float>(b0), P<const float>(b1), H,
                           P<const uint16_t>(Wo), P<const float>(bo), P<const int32_t>(labels), B, C, scale,
                           P<uint16_t>(dact2), P<float>(slab), P<float>(block_loss), P<int32_t>(block_correct),
                           S(stream)),
          "mlp_step_fwd");
  });
  m.def("mlp_step_fwd_infer", [](u X, int K0, u Wf, u b0, u b1, int H, u Wo, u bo, int B, int C, u logits, u pred,
                                 u stream) {
    check(har_mlp_step_fwd_infer(P<const uint16_t>(X), K0, P<const uint16_t>(Wf), P<const float>(b0),
                                 P<const float>(b1), H, P<const uint16_t>(Wo), P<const float>(bo), B, C,
                                 P<float>(logits), P<int32_t>(pred), S(stream)),
          "mlp_step_fwd_infer");
  });
  m.def("mlp_step_bwd", [](u dact2, u X, int K0, u Wf, int H, u b0, int B, u gw1, u gw0, u gb0, u gb1,
                           int64_t stride, u tick, u fslab, int fslab_w, u gwo, u gbo, u stream) {
    check(har_mlp_step_bwd(P<const uint16_t>(dact2), P<const uint16_t>(X), K0, P<const uint16_t>(Wf), H,
                           P<const float>(b0), B, P<float>(gw1), P<float>(gw0), P<float>(gb0), P<float>(gb1), stride,
                           P<int32_t>(tick), P<const float>(fslab), fslab_w, P<float>(gwo), P<float>(gbo), S(stream)),
          "mlp_step_bwd");
  });
  m.def("mlp_fwd_head", [](u X, int K0, u W0, u b0, u W1, u b1, int H, u Wo, u bo, u labels, int B, int C,
                           float scale, u h1, u dact, u slab, u block_loss, u block_correct, u stream) {
    check(har_mlp_fwd_head(P<const uint16_t>(X), K0, P<const uint16_t>(W0), P<const float>(b0),
                           P<const uint16_t>(W1), P<const float>(b1), H, P<const uint16_t>(Wo), P<const float>(bo),
                           P<const int32_t>(labels), B, C, scale, P<uint16_t>(h1), P<uint16_t>(dact), P<float>(slab),
                           P<float>(block_loss), P<int32_t>(block_correct), S(stream)),
          "mlp_fwd_head");
  });
  m.def("mlp_fwd_infer_f32", [](u X, int ldx, int F, int K0, u W0, u b0, u W1, u b1, int H, u Wo, u bo, int B,
                                int C, u logits, u pred, u stream) {
    check(har_mlp_fwd_infer_f32(P<const float>(X), ldx, F, K0, P<const uint16_t>(W0), P<const float>(b0),
                                P<const uint16_t>(W1), P<const float>(b1), H, P<const uint16_t>(Wo), P<const float>(bo),
                                B, C, P<float>(logits), P<int32_t>(pred), S(stream)),
          "mlp_fwd_infer_f32");
  });
  m.def("mlp_fwd_infer", [](u X, int K0, u W0, u b0, u W1, u b1, int H, u Wo, u bo, int B, int C, u logits, u pred,
                            u stream) {
    check(har_mlp_fwd_infer(P<const uint16_t>(X), K0, P<const uint16_t>(W0), P<const float>(b0),
                            P<const uint16_t>(W1), P<const float>(b1), H, P<const uint16_t>(Wo), P<const float>(bo), B,
                            C, P<float>(logits), P<int32_t>(pred), S(stream)),
          "mlp_fwd_infer");
  });
  m.def("head_fused", [](u H, u W, u bias, u labels, int B, int D, int C, float scale, u dlogits, u dH, u block_loss,
                         u block_correct, u stream) {
    check(har_head_fused(P<const uint16_t>(H), P<const uint16_t>(W), P<const float>(bias), P<const int32_t>(labels),
                         B, D, C, scale, P<uint16_t>(dlogits), P<uint16_t>(dH), P<float>(block_loss),
                         P<int32_t>(block_correct), S(stream)),
          "head_fused");
  });

  m.def(
      "reduce_slabs_grouped",
      [](u slabs, int S_, int64_t n, u dst, int G, u stream, u tick, int64_t lds, int64_t ldd) {
        check(har_reduce_slabs_grouped(P<const float>(slabs), S_, n, lds < 0 ? n : lds, P<float>(dst), G,
                                       ldd < 0 ? n : ldd, P<int32_t>(tick), S(stream)),
              "reduce_slabs_grouped");
      },
      py::arg("slabs"), py::arg("S"), py::arg("n"), py::arg("dst"), py::arg("G"), py::arg("stream"),
      py::arg("tick"), py::arg("lds") = -1, py::arg("ldd") = -1);

  m.def("column_stats_workspace", &har_column_stats_workspace);
  m.def("column_stats_f64", [](u X, int64_t n, int ncols, u center, u stats, u ws, u stream) {
    check(har_column_stats_f64(P<const double>(X), n, ncols, P<const double>(center), P<double>(stats),
                               P<double>(ws), S(stream)),
          "column_stats_f64");
  });
  m.def("column_stats", [](u X, int64_t n, int ncols, int ld, u w, u stats, u ws, u stream) {
    check(har_column_stats(P<const float>(X), n, ncols, ld, P<const float>(w), P<double>(stats), P<double>(ws),
                           S(stream)),
          "column_stats");
  });
  m.def("tree_thresholds_hybrid", [](u cat, int64_t n, int ncat, int F, u colmap, u dthr, int ns, int maxb, u ones,
                                     u thr_mat, u nbins, u stream) {
    check(har_tree_thresholds_hybrid(P<const int32_t>(cat), n, ncat, F, P<const int32_t>(colmap), P<const float>(dthr),
                                     ns, maxb, P<int32_t>(ones), P<float>(thr_mat), P<int32_t>(nbins), S(stream)),
          "tree_thresholds_hybrid");
  });
  m.def("tree_bins_hybrid", [](u dense, int64_t n, int Fd, u dense_cols, u cat, int ncat, int F, u thr, int maxb,
                               u nbins, u bins, u stream) {
    check(har_tree_bins_hybrid(P<const float>(dense), n, Fd, P<const int32_t>(dense_cols), P<const int32_t>(cat), ncat,
                               F, P<const float>(thr), maxb, P<const int32_t>(nbins), P<uint8_t>(bins), S(stream)),
          "tree_bins_hybrid");
  });
  m.def("bin_features", [](u X, int64_t n, int F, int ld, u thr, int maxb, u nthr, u bins, u stream) {
    check(har_bin_features(P<const float>(X), n, F, ld, P<const float>(thr), maxb, P<const int32_t>(nthr),
                           P<uint8_t>(bins), S(stream)),
          "bin_features");
  });

  m.def("tree_feature_subsets", [](uint64_t seed, u trees, u nodes, int64_t npairs, int F, int m_, u out, u p_dev,
                                   u stream) {
    check(har_tree_feature_subsets(seed, P<const int32_t>(trees), P<const int32_t>(nodes), npairs, F, m_,
                                   P<int32_t>(out), P<const int32_t>(p_dev), S(stream)),
          "tree_feature_subsets");
  });
  m.def("tree_level_keys", [](u node_of, u cand_idx, int T, int64_t N, int maxn, u key, u stream) {
    check(har_tree_level_keys(P<const int32_t>(node_of), P<const int32_t>(cand_idx), T, N, maxn, P<int32_t>(key),
                              S(stream)),
          "tree_level_keys");
  });
  m.def("tree_level_group", [](u node_of, u cand_idx, u tree_lo, u W, int T, int64_t N, int maxn, int A, int nt_max,
                               u cnt_ws, u counts, u starts, u rows, u row_w, u a_dev, u stream) {
    check(har_tree_level_group(P<const int32_t>(node_of), P<const int32_t>(cand_idx), P<const int32_t>(tree_lo),
                               P<const float>(W), T, N, maxn, A, nt_max, P<int32_t>(cnt_ws), P<int32_t>(counts),
                               P<int32_t>(starts), P<int32_t>(rows), P<float>(row_w), P<const int32_t>(a_dev),
                               S(stream)),
          "tree_level_group");
  });
  m.def("tree_level_group_chunks", [](int64_t N) { return har_tree_level_group_chunks(N); });
  m.def("tree_commit_level", [](int nsplit, u ti, u ni, u cl, u dsi, u rfeat, u rbin, u rgain, u rleft, u rtotal, int K,
                                u thr_mat, int ldthr, int maxn, u feature, u split_bin, u thresh, u left, u right,
                                u gains, u stats, u s_dev, u stream) {
    check(har_tree_commit_level(nsplit, P<const int64_t>(ti), P<const int64_t>(ni), P<const int64_t>(cl),
                                P<const int64_t>(dsi), P<const int32_t>(rfeat), P<const int32_t>(rbin),
                                P<const float>(rgain), P<const float>(rleft), P<const float>(rtotal), K,
                                P<const float>(thr_mat), ldthr, maxn, P<int32_t>(feature), P<int32_t>(split_bin),
                                P<float>(thresh), P<int32_t>(left), P<int32_t>(right), P<float>(gains),
                                P<float>(stats), P<const int32_t>(s_dev), S(stream)),
          "tree_commit_level");
  });
  m.def("tree_partition_split", [](u node_of, u feature, u split_bin, u left, u bins, int T, int64_t N, int maxn,
                                   u stream) {
    check(har_tree_partition_split(P<int32_t>(node_of), P<const int32_t>(feature), P<const int32_t>(split_bin),
                                   P<const int32_t>(left), P<const uint8_t>(bins), T, N, maxn, S(stream)),
          "tree_partition_split");
  });
  m.def("tree_level_decide", [](int A, u gain, u left, u total, int K, int impurity, float min2, u out, u a_dev,
                                u stream) {
    check(har_tree_level_decide(A, P<const float>(gain), P<const float>(left), P<const float>(total), K, impurity, min2,
                                P<float>(out), P<const int32_t>(a_dev), S(stream)),
          "tree_level_decide");
  });
  m.def("tree_frontier", [](int A, int Tn, int maxn, u ct, u cn, u tlo, u dec, u n_nodes, u n_nodes_next, u pos_ws,
                            u ti, u ni, u cl, u dsi, u front, u q_ws, u ct_next, u cn_next, u tlo_next, u cand_idx,
                            u scal, u a_dev, u parent_of, u derive_from, u stream) {
    check(har_tree_frontier(A, Tn, maxn, P<const int32_t>(ct), P<const int32_t>(cn), P<const int32_t>(tlo),
                            P<const float>(dec), P<const int32_t>(n_nodes), P<int32_t>(n_nodes_next),
                            P<int32_t>(pos_ws), P<int64_t>(ti), P<int64_t>(ni), P<int64_t>(cl), P<int64_t>(dsi),
                            P<float>(front), P<int32_t>(q_ws), P<int32_t>(ct_next), P<int32_t>(cn_next),
                            P<int32_t>(tlo_next), P<int32_t>(cand_idx), P<int32_t>(scal), P<const int32_t>(a_dev),
                            P<int32_t>(parent_of), P<int32_t>(derive_from), S(stream)),
          "tree_frontier");
  });
  m.def("tree_root_frontier", [](u stats, int Tn, int K, int64_t tree_stride, int impurity, float min2, int maxn, u ct,
                                 u cn, u tlo, u cand_idx, u scal, u stream) {
    check(har_tree_root_frontier(P<const float>(stats), Tn, K, tree_stride, impurity, min2, maxn, P<int32_t>(ct),
                                 P<int32_t>(cn), P<int32_t>(tlo), P<int32_t>(cand_idx), P<int32_t>(scal), S(stream)),
          "tree_root_frontier");
  });
  m.def("tree_partition", [](u node_of, u lvl_feat, u lvl_bin, u lvl_left, u bins, int T, int64_t N, int maxn,
                             u stream) {
    check(har_tree_partition(P<int32_t>(node_of), P<const int32_t>(lvl_feat), P<const int32_t>(lvl_bin),
                             P<const int32_t>(lvl_left), P<const uint8_t>(bins), T, N, maxn, S(stream)),
          "tree_partition");
  });
  m.def("csv_count_newlines", [](u buf, int64_t n, u counts, u stream) {
    check(har_csv_count_newlines(P<const uint8_t>(buf), n, P<int32_t>(counts), S(stream)), "csv_count_newlines");
  });
  m.def("csv_newline_pos", [](u buf, int64_t n, u block_off, u pos, u stream) {
    check(har_csv_newline_pos(P<const uint8_t>(buf), n, P<const int64_t>(block_off), P<int64_t>(pos), S(stream)),
          "csv_newline_pos");
  });
  m.def("csv_parse_rows", [](u buf, u starts, u ends, int64_t nrows, int ncols, u vals, u hashes, u flags, u fstart,
                             u flen, u stream) {
    check(har_csv_parse_rows(P<const uint8_t>(buf), P<const int64_t>(starts), P<const int64_t>(ends), nrows, ncols,
                             P<double>(vals), P<uint64_t>(hashes), P<uint8_t>(flags), P<int64_t>(fstart),
                             P<int32_t>(flen), S(stream)),
          "csv_parse_rows");
  });

  m.def("cast_pad_bf16", [](u in, int rows, int cin, int ldin, u out, int cout, u stream) {
    check(har_cast_pad_bf16(P<const float>(in), rows, cin, ldin, P<uint16_t>(out), cout, S(stream)), "cast_pad_bf16");
  });
}
