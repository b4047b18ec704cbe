// hipBLASLt extension-API GEMMs with tuned (solution, splitK, wgm) triples -- see blaslt.h.
//
// Host code only (no kernels of its own): it drives the hipBLASLt library PyTorch ships (the
// extension resolves libhipblaslt.so.1 to the copy torch already loaded), so the solution indices
// of a tuning table are those of the kernel library torch's own GEMMs use.  Only entry points that
// library exports are called (it predates GemmInstance::setMaxWorkspaceBytes: the workspace limit
// is enforced here, from isAlgoSupported's requirement).
#include "blaslt.h"

#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <tuple>

namespace {

constexpr size_t kWorkspace = 64ull << 20;    // split-K partials of the largest tuned product fit

const float kOne = 1.f, kZero = 0.f;           // host alpha / beta (read when arguments are built)

std::mutex g_mu;

hipblasLtHandle_t handle() {
  static hipblasLtHandle_t h = [] {
    hipblasLtHandle_t x = nullptr;
    if (hipblasLtCreate(&x) != HIPBLAS_STATUS_SUCCESS) throw std::runtime_error("hipblasLtCreate failed");
    return x;
  }();
  return h;
}

// One split-K workspace per stream: two tuned split-K GEMMs running concurrently on different
// streams must not share their partials buffer.  A stream first seen while it is being captured
// into a HIP graph (torch captures on a side stream of its own, and nothing may be allocated
// during a capture) gets the first stream's workspace: a graph replays on the stream that enqueues
// it, in order with that stream's eager work.
void* workspace(hipStream_t st) {
  static std::map<hipStream_t, void*> ws;
  static void* first = nullptr;
  auto it = ws.find(st);
  if (it != ws.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    if (!first) throw std::runtime_error("blaslt: first GEMM inside a graph capture (run one eagerly first)");
    ws.emplace(st, first);
    return first;
  }
  void* p = nullptr;
  if (hipMalloc(&p, kWorkspace) != hipSuccess) throw std::runtime_error("blaslt workspace alloc failed");
  if (!first) first = p;
  ws.emplace(st, p);
  return p;
}

hipblasOperation_t op(int t) { return t ? HIPBLAS_OP_T : HIPBLAS_OP_N; }
hipDataType dtype(const BltProblem& p) { return p.f16 ? HIP_R_16F : HIP_R_16BF; }

std::unique_ptr<hipblaslt_ext::Gemm> make_gemm(const BltProblem& p, const void* A, const void* B, void* C,
                                               const void* bias) {
  const hipDataType dt = dtype(p);
  auto g = std::make_unique<hipblaslt_ext::Gemm>(handle(), op(p.opA), op(p.opB), dt, dt, dt, dt,
                                                  HIPBLAS_COMPUTE_32F);
  hipblaslt_ext::GemmEpilogue epi;
  hipblaslt_ext::GemmInputs in;
  if (p.bias) {
    epi.setMode(HIPBLASLT_EPILOGUE_BIAS);
    epi.setBiasDataType(dt);
    in.setBias(bias);
  }
  in.setA(A);
  in.setB(B);
  in.setC(C);
  in.setD(C);
  in.setAlpha(&kOne);
  in.setBeta(p.beta1 ? &kOne : &kZero);
  hipblaslt_ext::GemmProblemType pt(op(p.opA), op(p.opB), dt, dt, dt, dt, HIPBLAS_COMPUTE_32F);
  if (g->setProblem(p.m, p.n, p.k, p.batch, p.lda, p.ldb, p.ldc, p.ldc, p.sa, p.sb, p.sc, p.sc, epi, in, pt) !=
      HIPBLAS_STATUS_SUCCESS)
    return nullptr;
  return g;
}

std::vector<hipblasLtMatmulHeuristicResult_t> all_algos(const BltProblem& p) {
  std::vector<hipblasLtMatmulHeuristicResult_t> r;
  const hipDataType dt = dtype(p);
  hipblaslt_ext::getAllAlgos(handle(), hipblaslt_ext::GemmType::HIPBLASLT_GEMM, op(p.opA), op(p.opB), dt, dt,
                             dt, dt, HIPBLAS_COMPUTE_32F, r);
  return r;
}

bool algo_of(int index, hipblasLtMatmulAlgo_t& algo) {
  std::vector<int> idx{index};
  std::vector<hipblasLtMatmulHeuristicResult_t> r;
  if (hipblaslt_ext::getAlgosFromIndex(handle(), idx, r) != HIPBLAS_STATUS_SUCCESS || r.empty()) return false;
  algo = r[0].algo;
  return true;
}

hipblaslt_ext::GemmTuning tuning_of(int splitk, int wgm) {
  hipblaslt_ext::GemmTuning t;
  t.setSplitK((uint16_t)splitk);
  t.setWgm((int16_t)wgm);
  return t;
}

// <0: unsupported; else mean microseconds per call over `iters`
float time_one(hipblaslt_ext::Gemm& g, hipblasLtMatmulAlgo_t algo, int splitk, int wgm, int iters,
               hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  auto t = tuning_of(splitk, wgm);
  size_t need = 0;
  if (g.isAlgoSupported(algo, t, need) != HIPBLAS_STATUS_SUCCESS || need > kWorkspace) return -1.f;
  if (g.initialize(algo, t, workspace(st), true, st) != HIPBLAS_STATUS_SUCCESS) return -1.f;
  for (int i = 0; i < 2; ++i)
    if (g.run(st) != HIPBLAS_STATUS_SUCCESS) return -1.f;
  hipEventRecord(e0, st);
  for (int i = 0; i < iters; ++i) g.run(st);
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / iters;
}

// Initialised problems keyed by shape, tuning, stream AND operand pointers: the model's GEMM
// operands live in preallocated (layer-strided) buffers, so every call site repeats its pointers
// step after step and, after the first step, is a bare kernel launch (also inside HIP-graph
// capture).  Least-recently-used entries are evicted one at a time, so pointers churned by the
// caching allocator (eager multi-rank runs) never flush the hot call sites.
using Key = std::tuple<int, int, long, long, long, long, long, long, long, long, long, long, int, int, int, int, int,
                       int, const void*, const void*, const void*, const void*, const void*>;
constexpr size_t kMaxCached = 8192;

Key key_of(const BltProblem& p, int algo, int splitk, int wgm, const void* A, const void* B, const void* C,
           const void* bias, hipStream_t st) {
  return Key{p.opA, p.opB, p.m, p.n, p.k, p.batch, p.lda, p.ldb, p.ldc, p.sa, p.sb, p.sc, p.f16, p.beta1,
             p.bias, algo, splitk, wgm, A, B, C, bias, (const void*)st};
}

struct Lru {
  std::list<Key> order;     // most recently used first
  std::map<Key, std::pair<std::unique_ptr<hipblaslt_ext::Gemm>, std::list<Key>::iterator>> map;
};

Lru& cache() {
  static Lru c;
  return c;
}

}  // namespace

std::vector<BltResult> dltb_blaslt_sweep(const BltProblem& p, const void* A, const void* B, void* C,
                                         const void* bias, int iters,
                                         const std::vector<int>& splitks, const std::vector<int>& wgms,
                                         int refine, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<BltResult> out;
  auto g = make_gemm(p, A, B, C, bias);
  if (!g) return out;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto algos = all_algos(p);
  std::vector<std::pair<float, size_t>> base;
  for (size_t i = 0; i < algos.size(); ++i) {
    const float us = time_one(*g, algos[i].algo, 0, 0, iters, st, e0, e1);
    if (us < 0) continue;
    base.push_back({us, i});
    out.push_back({hipblaslt_ext::getIndexFromAlgo(algos[i].algo), 0, 0, us,
                   hipblaslt_ext::getSolutionNameFromAlgo(handle(), algos[i].algo)});
  }
  std::sort(base.begin(), base.end());
  if (refine > 0 && (int)base.size() > refine) base.resize(refine);   // refine <= 0: every solution
  for (auto& b : base) {
    auto& a = algos[b.second];
    for (int sk : splitks)
      for (int wg : wgms) {
        if (sk == 0 && wg == 0) continue;
        const float us = time_one(*g, a.algo, sk, wg, iters, st, e0, e1);
        if (us < 0) continue;
        out.push_back({hipblaslt_ext::getIndexFromAlgo(a.algo), sk, wg, us,
                       hipblaslt_ext::getSolutionNameFromAlgo(handle(), a.algo)});
      }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  std::sort(out.begin(), out.end(), [](const BltResult& x, const BltResult& y) { return x.us < y.us; });
  return out;
}

int dltb_blaslt_run(const BltProblem& p, const void* A, const void* B, void* C, const void* bias, int algo,
                    int splitk, int wgm, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto& c = cache();
  const Key key = key_of(p, algo, splitk, wgm, A, B, C, bias, st);
  auto it = c.map.find(key);
  if (it == c.map.end()) {
    hipblasLtMatmulAlgo_t a;
    if (!algo_of(algo, a)) return -1;
    auto g = make_gemm(p, A, B, C, bias);
    if (!g) return -2;
    auto t = tuning_of(splitk, wgm);
    size_t need = 0;
    if (g->isAlgoSupported(a, t, need) != HIPBLAS_STATUS_SUCCESS || need > kWorkspace) return -3;
    if (g->initialize(a, t, workspace(st), true, st) != HIPBLAS_STATUS_SUCCESS) return -4;
    if (c.map.size() >= kMaxCached) {       // evict the least recently used problem
      c.map.erase(c.order.back());
      c.order.pop_back();
    }
    c.order.push_front(key);
    it = c.map.emplace(key, std::make_pair(std::move(g), c.order.begin())).first;
  } else if (it->second.second != c.order.begin()) {
    c.order.splice(c.order.begin(), c.order, it->second.second);
  }
  return it->second.first->run(st) == HIPBLAS_STATUS_SUCCESS ? 0 : -5;
}

// Untuned problems: hipBLASLt's own heuristic choice (its first suggestion, the one torch's
// matmul would also get without TunableOp), initialised once per (problem, pointers, stream) in
// the same LRU cache, so an untuned product -- an fp16 GEMM of the reference-precision DDP/FSDP
// runs, an unbatched weight gradient of a multi-rank step -- is also a bare launch after its first
// call instead of ~25 us of torch-dispatch host time.  The heuristic's pick per problem SHAPE is
// memoised too, so new operand pointers cost one initialise, not another heuristic query.
int dltb_blaslt_run_heuristic(const BltProblem& p, const void* A, const void* B, void* C, const void* bias,
                              hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  static std::map<Key, hipblasLtMatmulAlgo_t> picks;     // shape key (null pointers) -> algo
  auto& c = cache();
  const Key key = key_of(p, -1, 0, 0, A, B, C, bias, st);
  auto it = c.map.find(key);
  if (it == c.map.end()) {
    auto g = make_gemm(p, A, B, C, bias);
    if (!g) return -2;
    const Key shape = key_of(p, -1, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr);
    auto pk = picks.find(shape);
    if (pk == picks.end()) {
      hipblaslt_ext::GemmPreference pref;
      pref.setMaxWorkspaceBytes(kWorkspace);
      std::vector<hipblasLtMatmulHeuristicResult_t> r;
      if (g->algoGetHeuristic(1, pref, r) != HIPBLAS_STATUS_SUCCESS || r.empty()) return -1;
      // solutions observed to fault the GPU in BATCHED form: never run them batched
      // (618464: bf16 TN, faulted as a 16-batch 1024 x 4096 x 8192 weight gradient,
      // profiles/dw_layout_probe_fault_r4.txt; the same solution runs the unbatched TN products --
      // the tied head's data gradient through the cached W^T -- without fault, GPU tests r3/r4)
      static const int kDenyBatched[] = {618464};
      const int idx = hipblaslt_ext::getIndexFromAlgo(r[0].algo);
      for (int d : kDenyBatched)
        if (p.batch > 1 && idx == d) return -6;
      pk = picks.emplace(shape, r[0].algo).first;
    }
    auto t = tuning_of(0, 0);
    size_t need = 0;
    if (g->isAlgoSupported(pk->second, t, need) != HIPBLAS_STATUS_SUCCESS || need > kWorkspace) return -3;
    if (g->initialize(pk->second, t, workspace(st), true, st) != HIPBLAS_STATUS_SUCCESS) return -4;
    if (c.map.size() >= kMaxCached) {
      c.map.erase(c.order.back());
      c.order.pop_back();
    }
    c.order.push_front(key);
    it = c.map.emplace(key, std::make_pair(std::move(g), c.order.begin())).first;
  } else if (it->second.second != c.order.begin()) {
    c.order.splice(c.order.begin(), c.order, it->second.second);
  }
  return it->second.first->run(st) == HIPBLAS_STATUS_SUCCESS ? 0 : -5;
}

std::string dltb_blaslt_name(int algo) {
  std::lock_guard<std::mutex> lk(g_mu);
  hipblasLtMatmulAlgo_t a;
  if (!algo_of(algo, a)) return "";
  return hipblaslt_ext::getSolutionNameFromAlgo(handle(), a);
}
