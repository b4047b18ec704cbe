// hipBLASLt extension-API GEMMs with per-shape tuned solutions (host code, csrc/blaslt.cpp).
//
// torch's matmul path (and TunableOp) picks among hipBLASLt solutions with their built-in split-K
// and workgroup mapping.  The extension API also exposes both as run-time tuning parameters
// (hipblaslt_ext::GemmTuning: splitK, wgm); on the small per-layer products of a 2048-token
// micro-batch (grids of 128-256 tiles on 256 CUs) those two knobs decide the wave count and which
// operand panels share an XCD's L2.  blaslt_sweep times every solution x tuning for one problem;
// blaslt_run executes a chosen (solution index, splitK, wgm) triple, caching the initialised
// hipblaslt_ext::Gemm per problem so a repeat call with the same pointers is a bare launch.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

struct BltProblem {
  int opA = 0, opB = 0;          // 0 = N, 1 = T (column-major BLAS convention)
  long m = 0, n = 0, k = 0, batch = 1;
  long lda = 0, ldb = 0, ldc = 0;
  long sa = 0, sb = 0, sc = 0;   // batch strides (elements)
  int f16 = 0;                   // 0 = bf16, 1 = fp16 operands and output, fp32 compute
  int beta1 = 0;                 // 1: D = A B + C (accumulate into the output)
  int bias = 0;                  // 1: D += bias[m] (epilogue; the bias has the output's format)
};

struct BltResult {
  int algo;
  int splitk;
  int wgm;
  float us;
  std::string name;
};

// Time all solutions (default tuning), then the fastest `refine` of them (all of them when
// refine <= 0: a large-tile solution is slow alone but can win with split-K) under every
// (splitK, wgm) pair.  A, B, C must be device buffers of the problem's extents; C is overwritten.
std::vector<BltResult> dltb_blaslt_sweep(const BltProblem& p, const void* A, const void* B, void* C,
                                         const void* bias, int iters, const std::vector<int>& splitks,
                                         const std::vector<int>& wgms, int refine, hipStream_t st);

// D (+)= A B with solution `algo` (an index from the sweep) and tuning (0 = solution default).
// Returns 0 on success, a negative code when the solution does not support the problem.
int dltb_blaslt_run(const BltProblem& p, const void* A, const void* B, void* C, const void* bias, int algo,
                    int splitk, int wgm, hipStream_t st);

// D (+)= A B with hipBLASLt's heuristic solution for an untuned problem (memoised per shape).
int dltb_blaslt_run_heuristic(const BltProblem& p, const void* A, const void* B, void* C, const void* bias,
                              hipStream_t st);

// Solution name of an algo index (validation of stored tables against the loaded library).
std::string dltb_blaslt_name(int algo);
